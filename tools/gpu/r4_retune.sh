#!/bin/bash
# round 4 (late): re-tune every shape of every leg at the final kernel set
# (bench.py --tune-cache none --tune-save) -> gpurun_out/tune_r4b.txt, then C2
# legs alternated with the committed table and the new one
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --no-cpu-baseline --tune-cache none --tune-save gpurun_out/tune_r4b.txt > gpurun_out/r4_retune_bench.json 2> gpurun_out/r4_retune_bench.err || { tail -5 gpurun_out/r4_retune_bench.err; exit 1; }
echo "retune done: $(wc -l < gpurun_out/tune_r4b.txt) keys"
for t in old new old new; do
  if [ $t = old ]; then T=profiles/tune_r4.txt; else T=gpurun_out/tune_r4b.txt; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --tune-cache $T > gpurun_out/r4_rt_$t.json 2> gpurun_out/r4_rt_$t.err || { tail -20 gpurun_out/r4_rt_$t.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('$t C2',d['value'],d['ms_per_step'])" gpurun_out/r4_rt_$t.json
done
