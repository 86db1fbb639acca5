#!/bin/bash
# round 4: HBM traffic of the fused BN-backward dgrad candidates on single shapes
# (tools/dgrad_bench.py, SHAPES 3 = 14^2 1024 <- 256 kind 3 res1, 6 = 56^2 256 <- 64
# kind 3 res1): FETCH_SIZE and WRITE_SIZE passes, per kernel name
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/bnbpmc
cd /tmp && export TMPDIR=/tmp
for sh in 3 6; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$R/gpurun_out/bnbpmc/s${sh}_$c
    rm -rf $d
    SHAPES=$sh CFGS=16,18,19,22,0 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d -o run -- python3 $R/tools/dgrad_bench.py > $d.log 2>&1 || { echo "FAIL $sh $c"; tail -5 $d.log; exit 1; }
  done
  grep -v amdgpu $R/gpurun_out/bnbpmc/s${sh}_FETCH_SIZE.log
  python3 - $R $sh <<'PY'
import csv, sys, collections, glob
R, sh = sys.argv[1], sys.argv[2]
out = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"{R}/gpurun_out/bnbpmc/s{sh}_{c}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[(r["Dispatch_Id"], r["Kernel_Name"])].append(float(r["Counter_Value"]))
    per = collections.defaultdict(list)
    for (disp, name), v in acc.items():
        per[name].append(sum(v))
    for name, v in per.items():
        out.setdefault(name, {})[c] = sum(v) / len(v)
for name, d in out.items():
    if "bnb" in name or "kernel" in name:
        fs = d.get("FETCH_SIZE", 0) * 1024 * 2  # KB, x2 gfx950 correction (summarize_pmc.py)
        ws = d.get("WRITE_SIZE", 0) * 1024
        print(f"shape {sh} {name[:80]:80s} fetch {fs/1e9:6.3f} GB write {ws/1e9:6.3f} GB")
PY
done
