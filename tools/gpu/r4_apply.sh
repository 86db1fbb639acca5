#!/bin/bash
# round 4: the BN-backward apply pass alone (tools/apply_bench.py) at several
# workgroup targets (ARTSBIR_BNB_WGS, minimum unit rows ARTSBIR_BNB_MINROWS),
# then C2 bench legs at the old (2048, 1) and the new default (16384, 8)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for w in "2048 1" "16384 8" "32768 8" "16384 4" "32768 16"; do
  set -- $w
  echo "== wgs $1 minrows $2"
  ARTSBIR_BNB_WGS=$1 ARTSBIR_BNB_MINROWS=$2 timeout -k 10 120 python3 -u tools/apply_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
for w in "2048 1" "16384 8" "2048 1" "16384 8"; do
  set -- $w
  ARTSBIR_BNB_WGS=$1 ARTSBIR_BNB_MINROWS=$2 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > gpurun_out/r4_apply_$1.json 2> gpurun_out/r4_apply_$1.err || { tail -20 gpurun_out/r4_apply_$1.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('wgs $1 C2',d['value'],d['ms_per_step'])" gpurun_out/r4_apply_$1.json
done
