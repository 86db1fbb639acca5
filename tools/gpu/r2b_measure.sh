#!/bin/bash
# round-2 closing measurement: warm the autotune cache, PMC traffic of the timed
# launches (cache loaded, separate FETCH_SIZE / WRITE_SIZE passes), the default
# bench line with that cache and traffic file, rocprofv3 kernel statistics of
# the C2 leg and of the C5 step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
TC=$R/gpurun_out/tune_r2b.txt
rm -f $TC
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-retrieval --no-embed --no-c5 --no-profile --steps 3 --warmup 2 --tune-cache $TC > gpurun_out/warm.json 2> gpurun_out/warm.err || { echo WARM_FAILED; tail -5 gpurun_out/warm.err; exit 1; }
cut -c1-160 gpurun_out/warm.json
cd /tmp && export TMPDIR=/tmp
for leg in train retr; do
  if [ $leg = train ]; then ARGS="--no-cpu-baseline --no-retrieval --no-embed --no-c5 --no-profile --steps 2 --warmup 1 --tune-cache $TC"; else ARGS="--no-cpu-baseline --no-embed --no-c5 --no-profile --batch 8 --steps 1 --warmup 1"; fi
  mkdir -p $R/gpurun_out/pmc_$leg
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$R/gpurun_out/pmc_$leg/pmc_$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d -o run -- python3 $R/bench.py $ARGS > $d.log 2>&1 || { echo PMC_FAILED $leg $c; tail -5 $d.log; exit 1; }
  done
done
cd $R && python3 profiles/summarize_pmc.py gpurun_out/pmc_train gpurun_out/pmc_retr gpurun_out/r2b_pmc_traffic.json || exit 1
echo pmc done
ARTSBIR_PMC_TRAFFIC=$R/gpurun_out/r2b_pmc_traffic.json timeout -k 10 700 python -u bench.py --tune-cache $TC > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_full.err; exit 1; }
cut -c1-300 gpurun_out/bench_full.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r2b -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --tune-cache $TC > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/bench_prof.err || { echo PROF_FAILED; tail -20 $R/gpurun_out/bench_prof.err; exit 1; }
echo prof done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c5b -o run --output-format csv -- python3 $R/tools/c5_step.py 512 fp8 > $R/gpurun_out/c5_prof.log 2>&1 || { echo C5PROF_FAILED; tail -20 $R/gpurun_out/c5_prof.log; exit 1; }
echo c5 done
