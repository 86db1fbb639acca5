#!/bin/bash
# round-4 closing measurement: PMC traffic per leg with the committed table
# (tools/gpu/r4_pmc.sh), the traffic files put where bench.py reads them, then
# the default bench line exactly as the driver runs it and rocprofv3 kernel
# statistics of its C2 leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu/r4_pmc.sh || exit 1
cp gpurun_out/r4_pmc_traffic.json gpurun_out/r4_embed_pmc_traffic.json gpurun_out/r4_c5_pmc_traffic.json profiles/
s0=$(date +%s)
timeout -k 10 900 python -u bench.py > gpurun_out/r4_final_bench.json 2> gpurun_out/r4_final_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/r4_final_bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - s0 )) s"; tail -c 300 gpurun_out/r4_final_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r4 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > $R/gpurun_out/r4_prof_bench.json 2> $R/gpurun_out/r4_prof_bench.err || { echo PROF_FAILED; tail -20 $R/gpurun_out/r4_prof_bench.err; exit 1; }
echo prof done
