#!/bin/bash
# A/B inside the overlapped C2 step: the 3x3 fused-BN-backward dgrads that the
# standalone tuner puts on the 256x256 tile (148 KB of LDS, one workgroup per CU)
# forced onto smaller-LDS tiles that can share a CU with weight-gradient workgroups
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out scratch_dg3
python - <<'PY'
base = open("profiles/tune_r3s2.txt").read().splitlines()
for cand in (16, 13, 14):
    out = []
    for l in base:
        f = l.split()
        if f and f[0] == "c" and f[6] == "3" and f[15] != "0" and f[16] == "0":
            f[16] = str(cand)
        out.append(" ".join(f))
    open(f"scratch_dg3/c{cand}.txt", "w").write("\n".join(out) + "\n")
PY
for t in profiles/tune_r3s2.txt scratch_dg3/c16.txt scratch_dg3/c13.txt scratch_dg3/c14.txt profiles/tune_r3s2.txt scratch_dg3/c16.txt; do
  timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --tune-cache $t > gpurun_out/dg3_out.json 2> gpurun_out/dg3_out.err || { echo FAIL $t; tail -5 gpurun_out/dg3_out.err; exit 1; }
  python -c "import json,sys; l=json.load(open('gpurun_out/dg3_out.json')); print(sys.argv[1], l['value'], l['ms_per_step'], l['allocator']['step_ms'])" $t
done
