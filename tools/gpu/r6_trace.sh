#!/bin/bash
# round 6: a rocprofv3 kernel trace of the C2 step (every kernel, torch's too) and
# its timeline gaps (tools/trace_gaps.py); then the bench's N=2 rehearsal (gloo,
# two ranks sharing the one GPU)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
C2="--no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --no-loss-check --no-profile"
( cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/r6_trace && \
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r6_trace -o run -- \
    python3 $R/bench.py $C2 --steps 3 --warmup 2 > $R/gpurun_out/r6_trace.log 2>&1 ) || { echo TRACE_FAILED; tail -5 gpurun_out/r6_trace.log; exit 1; }
f=$(find gpurun_out/r6_trace -name "*kernel_trace.csv" | head -1)
python3 tools/trace_gaps.py "$f" > gpurun_out/r6_trace_gaps.txt 2>&1; head -60 gpurun_out/r6_trace_gaps.txt
rm -f "$f.gz"; gzip -k "$f" && mv "$f.gz" gpurun_out/r6_kernel_trace.csv.gz
[ "$1" = "gloo" ] || exit 0
ARTSBIR_DIST_BACKEND=gloo timeout -k 10 800 python -u bench.py --gpus 2 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r6_gloo2.log 2>&1; rc=$?
tail -c 1500 gpurun_out/r6_gloo2.log; exit $rc
