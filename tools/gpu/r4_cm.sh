#!/bin/bash
# (measured slower: the PP_CM code was removed again; re-add it to rerun)
# round 4 (late): pp256's chunk-major K walk for the 3x3 convs (production)
# against the tap-major one (diagnostic build art-sbir_amd/build_var/libtm.so,
# pp256.hip with -DPP_CM=0): candidate-22 parity tests, conv shapes
# (tools/pp_bench.py, candidate 22), fused dgrads (tools/dgrad_bench.py), C2 legs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pgemm_gpu.py tests/test_fused_gpu.py tests/test_c2_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r4_cm_tests.log 2>&1 || { tail -30 gpurun_out/r4_cm_tests.log; exit 1; }
tail -1 gpurun_out/r4_cm_tests.log
for v in tm cm; do
  if [ $v = cm ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/lib$v.so; fi
  echo "== $v"
  timeout -k 10 300 python3 -u tools/pp_bench.py --cands 22 --only conv --rounds 2 2>&1 | grep -v "amdgpu.ids\|round" | grep "3x3" || exit 1
  CFGS=22 SHAPES=0,1,2 timeout -k 10 300 python3 -u tools/dgrad_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
for v in tm cm tm cm; do
  if [ $v = cm ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/lib$v.so; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > gpurun_out/r4_cm_$v.json 2> gpurun_out/r4_cm_$v.err || { tail -20 gpurun_out/r4_cm_$v.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline']['per_kernel'];print('$v C2',d['value'],d['ms_per_step'],{k:round(v['avg_us'],1) for k,v in r.items() if k.startswith('pp256')})" gpurun_out/r4_cm_$v.json
done
