#!/bin/bash
# round 5: SQ counters of the kNN scan (retrieval leg, tools/retr_bench.py) in one
# --pmc pass: where the scan's waves spend their cycles
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/knn_pmc
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $R/gpurun_out/knn_pmc -o run -- python3 $R/tools/retr_bench.py > $R/gpurun_out/knn_pmc.log 2>&1 || { echo PMC_FAILED; tail -5 $R/gpurun_out/knn_pmc.log; exit 1; }
find $R/gpurun_out/knn_pmc -name "*.csv" | head
