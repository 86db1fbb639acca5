#!/bin/bash
# round 4: workgroup sizing of the forward act_pool / block_out passes
# (ARTSBIR_CG_WGS / ARTSBIR_CG_MINROWS): C2 bench legs alternated, old (2048, 1)
# against the new default (16384, 8), then the elementwise parity tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for w in "2048 1" "16384 8" "2048 1" "16384 8"; do
  set -- $w
  ARTSBIR_CG_WGS=$1 ARTSBIR_CG_MINROWS=$2 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > gpurun_out/r4_cg_$1.json 2> gpurun_out/r4_cg_$1.err || { tail -20 gpurun_out/r4_cg_$1.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline']['per_kernel'];print('cg $1 C2',d['value'],d['ms_per_step'],{k:round(v['avg_us'],1) for k,v in r.items() if 'act_pool' in k or 'block_out' in k or 'bn_bwd_apply' in k})" gpurun_out/r4_cg_$1.json
done
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_modules_gpu.py tests/test_encoder_gpu.py tests/test_c2_gpu.py tests/test_c1_gpu.py tests/test_fused_gpu.py -m gpu > gpurun_out/r4_cg_tests.log 2>&1 || { tail -30 gpurun_out/r4_cg_tests.log; exit 1; }
tail -1 gpurun_out/r4_cg_tests.log
