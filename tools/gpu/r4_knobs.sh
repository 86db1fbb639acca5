#!/bin/bash
# (measured and rejected: the two knobs were removed again; re-add them to rerun)
# round 4: LayerNorm-backward block count (ARTSBIR_LNB_BLOCKS) on the C5 step
# and the BN-backward reduction's workgroup target (ARTSBIR_BNR_WGS) on C2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for b in 512 2048 512 2048 1024; do
  echo "== LN bwd blocks $b"
  ARTSBIR_LNB_BLOCKS=$b ARTSBIR_TUNE_CACHE=profiles/tune_r4.txt timeout -k 10 300 python3 tools/c5_step.py 512 fp8 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done
for w in 2048 8192 2048 8192; do
  ARTSBIR_BNR_WGS=$w timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > gpurun_out/r4_bnr_$w.json 2> gpurun_out/r4_bnr_$w.err || { tail -20 gpurun_out/r4_bnr_$w.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline']['per_kernel'];print('bnr $w C2',d['value'],d['ms_per_step'],{k:round(v['avg_us'],1) for k,v in r.items() if 'reduce' in k})" gpurun_out/r4_bnr_$w.json
done
