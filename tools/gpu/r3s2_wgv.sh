#!/bin/bash
# A/B of weight-gradient tile / split choices inside the overlapped C2 step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out scratch_wgv
# v1/v2/v3: the 56^2 256->64 and 256->128 weight gradients on 64x256 @ 512 / 768
# workgroups, or 64x128 @ 256; v4: every pipelined weight gradient one split level finer
python - <<'PY'
base = open("profiles/tune_r3s2.txt").read().splitlines()
tgt = lambda f: f[1:6] in (["3612672", "56", "56", "256", "64"], ["3612672", "56", "56", "256", "128"])
V = {"v1": lambda f, c: 21 if tgt(f) else None, "v2": lambda f, c: 12 if tgt(f) else None,
     "v3": lambda f, c: 31 if tgt(f) else None, "v4": lambda f, c: c - 9 if 27 <= c < 36 else None}
for k, fn in V.items():
    out = []
    for l in base:
        f = l.split()
        if f and f[0] == "w" and fn(f, int(f[-1])) is not None:
            f[-1] = str(fn(f, int(f[-1])))
        out.append(" ".join(f))
    open(f"scratch_wgv/{k}.txt", "w").write("\n".join(out) + "\n")
PY
for t in profiles/tune_r3s2.txt scratch_wgv/v1.txt scratch_wgv/v2.txt scratch_wgv/v3.txt scratch_wgv/v4.txt profiles/tune_r3s2.txt; do
  timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --tune-cache $t > gpurun_out/wgv_out.json 2> gpurun_out/wgv_out.err || { echo FAIL $t; tail -5 gpurun_out/wgv_out.err; exit 1; }
  python -c "import json,sys; l=json.load(open('gpurun_out/wgv_out.json')); print(sys.argv[1], l['value'], l['ms_per_step'], l['allocator']['step_ms'])" $t
done
