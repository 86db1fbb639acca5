#!/bin/bash
# HBM traffic of the forward 1x1 expansion convs (fwd_bench, one shape per pass, FETCH_SIZE / WRITE_SIZE passes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/fpmc
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  d=$R/gpurun_out/fpmc/$c
  ONLY=0,1,2 CFGS=0,10 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d -o run -- python3 $R/tools/fwd_bench.py > $d.log 2>&1 || { echo PMC_FAILED $c; tail -5 $d.log; exit 1; }
done
cd $R && python3 - <<'PY'
import csv, glob, collections
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/fpmc/{c}/**/*counter_collection.csv", recursive=True)
    if not f: print("no csv", c); continue
    rows = list(csv.DictReader(open(f[0])))
    agg = collections.OrderedDict()
    for r in rows:
        k = (r["Kernel_Name"][:60], r.get("Grid_Size", r.get("Grid_Size_X", "")))
        agg.setdefault(k, []).append(float(r["Counter_Value"]))
    for k, v in agg.items():
        if "pgemm" in k[0] or "pstream" in k[0]:
            print(c, k, len(v), "avg MB", round(sum(v) / len(v) / 1024, 1))
PY
