#!/bin/bash
# (PP_EJB=4 is now the default; the old base is -DPP_EJB=2)
# round 4: pp256 epilogue operand batches (diagnostic build
# art-sbir_amd/build_var/libej4.so: pp256.hip with -DPP_EJB=4) against the
# production build: candidate 22 on the fused BN-backward dgrad shapes
# (tools/dgrad_bench.py), then a C2 bench leg each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for v in base ej4; do
  if [ $v = base ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/lib$v.so; fi
  echo "== $v"
  CFGS=22 timeout -k 10 300 python3 -u tools/dgrad_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
for v in base ej4 base ej4; do
  if [ $v = base ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/lib$v.so; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > gpurun_out/r4_ej_$v.json 2> gpurun_out/r4_ej_$v.err || { tail -20 gpurun_out/r4_ej_$v.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('$v C2',d['value'],d['ms_per_step'])" gpurun_out/r4_ej_$v.json
done
