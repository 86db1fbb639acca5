#!/bin/bash
# round 2 measurement, part A: warm the autotune cache (saved), then the PMC
# traffic passes on the timed launches only (cache loaded: no tuning trials)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
TC=$R/gpurun_out/tune_r2.txt
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-retrieval --no-embed --no-c5 --no-profile --steps 3 --warmup 2 --tune-cache $TC > gpurun_out/warm.json 2> gpurun_out/warm.err || { echo WARM_FAILED; tail -5 gpurun_out/warm.err; exit 1; }
cut -c1-200 gpurun_out/warm.json; wc -l $TC
cd /tmp && export TMPDIR=/tmp
for leg in train retr; do
  if [ $leg = train ]; then ARGS="--no-cpu-baseline --no-retrieval --no-embed --no-c5 --no-profile --steps 2 --warmup 1 --tune-cache $TC"; else ARGS="--no-cpu-baseline --no-embed --no-c5 --no-profile --batch 8 --steps 1 --warmup 1"; fi
  mkdir -p $R/gpurun_out/pmc_$leg
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$R/gpurun_out/pmc_$leg/pmc_$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d -o run -- python3 $R/bench.py $ARGS > $d.log 2>&1 || { echo PMC_FAILED $leg $c; tail -5 $d.log; exit 1; }
  done
done
cd $R && python3 profiles/summarize_pmc.py gpurun_out/pmc_train gpurun_out/pmc_retr gpurun_out/r2_pmc_traffic.json && echo pmc done
