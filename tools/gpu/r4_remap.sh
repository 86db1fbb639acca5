#!/bin/bash
# round 4: the XCD remap of pp256 on the C5 NT GEMM shapes: read bytes by
# request size and time with the remap (default) and in dispatch order
# (ARTSBIR_PG_DBG=4)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/remap
cd /tmp && export TMPDIR=/tmp
for v in 0 4; do
  d=$R/gpurun_out/remap/dbg$v
  rm -rf $d
  ARTSBIR_PG_DBG=$v timeout -s KILL 300 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ --output-format csv -d $d -o run -- python3 $R/tools/pp_bench.py --cands 22 --rounds 1 --only nt > $d.log 2>&1 || { echo "FAIL $v"; tail -5 $d.log; exit 1; }
  ARTSBIR_PG_DBG=$v timeout -k 10 300 python3 $R/tools/pp_bench.py --cands 22 --rounds 2 --only nt 2>&1 | grep -v "amdgpu\|^round" | sed "s/^/dbg$v /"
  python3 - $d $R <<'PY'
import sys, glob, csv, collections
sys.path.insert(0, sys.argv[2] + "/profiles")
import summarize_pmc as sp
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
tr = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
# per dispatch: read bytes, in dispatch order (the 6 NT shapes x 6 calls per shape)
per = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for r in csv.DictReader(open(f)):
    names[r["Dispatch_Id"]] = r["Kernel_Name"]
    per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
rows = [(int(d), 32 * c["TCC_EA0_RDREQ_32B"] + 64 * c["TCC_EA0_RDREQ_64B"] + 128 * c["TCC_EA0_RDREQ_128B"])
        for d, c in per.items() if "pp256" in names[d]]
rows.sort()
print("pp256 dispatches", len(rows), "read GB each:", " ".join(f"{b / 1e9:.2f}" for _, b in rows))
PY
done
