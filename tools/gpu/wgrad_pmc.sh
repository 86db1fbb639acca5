#!/bin/bash
# PMC counters of single weight-gradient launches (separate passes, kernel trace only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/wpmc
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
P2="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_INSTS_MFMA"
for job in "dense 0 1" "conv 7 27" "conv 3 19"; do
  set -- $job
  tag="$1_$2_$3"
  timeout -s KILL 90 rocprofv3 --pmc $P1 -d $R/gpurun_out/wpmc/${tag}_p1 -o run --output-format csv -- python3 $R/tools/wgrad_one.py $1 $2 $3 > $R/gpurun_out/wpmc/${tag}_p1.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc $P2 -d $R/gpurun_out/wpmc/${tag}_p2 -o run --output-format csv -- python3 $R/tools/wgrad_one.py $1 $2 $3 > $R/gpurun_out/wpmc/${tag}_p2.log 2>&1 || exit 1
  echo "$tag done"
done
