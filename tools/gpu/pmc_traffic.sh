#!/bin/bash
# HBM traffic per kernel: separate PMC passes (FETCH_SIZE, WRITE_SIZE) for the
# training step and for the retrieval leg, kernel trace only
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for leg in train retr; do
  if [ $leg = train ]; then ARGS="--no-cpu-baseline --no-retrieval --steps 2 --warmup 1"; else ARGS="--no-cpu-baseline --batch 8 --steps 1 --warmup 1"; fi
  mkdir -p $R/gpurun_out/pmc_$leg
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$R/gpurun_out/pmc_$leg/pmc_$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d -o run -- python3 $R/bench.py $ARGS > $d.log 2>&1 || { echo PMC_FAILED $leg $c; tail -5 $d.log; exit 1; }
  done
done
echo pmc done
