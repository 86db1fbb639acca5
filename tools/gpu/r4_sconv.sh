#!/bin/bash
# round 4 (late): sconv's persistent grid sized by LDS and register occupancy:
# direct-conv parity (candidate 20), then C2 and embedding legs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pgemm_gpu.py tests/test_fused_gpu.py tests/test_encoder_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu -k "20 or sconv or stem or encoder" > gpurun_out/r4_sconv_tests.log 2>&1 || { tail -30 gpurun_out/r4_sconv_tests.log; exit 1; }
tail -1 gpurun_out/r4_sconv_tests.log
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-c5 --no-retrieval --no-preprocess > gpurun_out/r4_sconv_$i.json 2> gpurun_out/r4_sconv_$i.err || { tail -20 gpurun_out/r4_sconv_$i.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline']['per_kernel'];print('C2',d['value'],d['ms_per_step'],'embed',d['embed']['value'],{k:round(v['avg_us'],1) for k,v in r.items() if 'sconv' in k})" gpurun_out/r4_sconv_$i.json
done
