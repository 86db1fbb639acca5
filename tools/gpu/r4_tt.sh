#!/bin/bash
# round 4 (late): the committed table (a) against it with the re-tune's 3x3
# 14^2 weight-gradient picks (b: loader-free halo kernel) and also its 1x1
# weight-gradient picks (c): C2 legs alternated
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for t in a b c a b c; do
  if [ $t = a ]; then T=profiles/tune_r4.txt; else T=tools/tt/$t.txt; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --tune-cache $T > gpurun_out/r4_tt_$t.json 2> gpurun_out/r4_tt_$t.err || { tail -20 gpurun_out/r4_tt_$t.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('$t C2',d['value'],d['ms_per_step'],round(d['roofline']['streams_kernel_ms']['side1']/5,2))" gpurun_out/r4_tt_$t.json
done
