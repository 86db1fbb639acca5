#!/bin/bash
# (measured neutral: the PG_NT_FWD knob was removed again; re-add it to rerun)
# round 4: non-temporal output stores in the persistent forward conv's epilogue
# (pstream with BN statistics; diagnostic build art-sbir_amd/build_var/libntf.so,
# pgemm.hip with -DPG_NT_FWD=1) against the production build: C2 legs alternated
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for v in base ntf base ntf; do
  if [ $v = base ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/lib$v.so; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > gpurun_out/r4_ntf_$v.json 2> gpurun_out/r4_ntf_$v.err || { tail -20 gpurun_out/r4_ntf_$v.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline']['per_kernel'];print('$v C2',d['value'],d['ms_per_step'],{k:round(v['avg_us'],1) for k,v in r.items() if 'pstream' in k or 'act_pool' in k or 'block_out' in k})" gpurun_out/r4_ntf_$v.json
done
