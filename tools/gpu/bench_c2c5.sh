#!/bin/bash
# C2 bench line (no CPU baselines / retrieval) with the C5 leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-retrieval --steps 5 --warmup 2 --c5 --c5-batch 512 > gpurun_out/bench_c2c5.json 2> gpurun_out/bench_c2c5.err; rc=$?
echo "rc=$rc"; tail -2 gpurun_out/bench_c2c5.err
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_c2c5.json").read().strip().splitlines()[-1])
print("C2", d["value"], d["ms_per_step"], d.get("allocator", {}).get("step_ms"), "loss0", d.get("loss_step0"), d.get("loss_step0_rel_diff"))
r = d.get("roofline") or {}
print("roof", r.get("kernel"), r.get("frac"), r.get("achieved"))
print("embed", (d.get("embed") or {}).get("value"))
print("C5", d.get("c5"))
pk = r.get("per_kernel", {})
for k, v in sorted(pk.items(), key=lambda kv: -kv[1].get("share_s", 0))[:14]:
    print("  ", k, v)
PY
exit $rc
