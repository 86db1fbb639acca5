#!/bin/bash
# round bench: parity tests, PMC traffic, default bench.py line (CPU baselines + retrieval), rocprofv3 stats
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/gpu/pmc_traffic.sh || exit 1
python3 profiles/summarize_pmc.py gpurun_out/pmc_train gpurun_out/pmc_retr profiles/r1_pmc_traffic.json
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_full.err; exit 1; }
cp profiles/r1_pmc_traffic.json gpurun_out/r1_pmc_traffic.json
cat gpurun_out/bench_full.json | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_final -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_final_prof.json 2> $R/gpurun_out/bench_final_prof.err || { echo PROF_FAILED; tail -20 $R/gpurun_out/bench_final_prof.err; exit 1; }
echo done
