#!/bin/bash
# issue / wait breakdown (SQ counters, one pass) of the forward 1x1 persistent conv and the 256x256 dense GEMM
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/sq
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES"
ONLY=0,2 CFGS=10,0 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $R/gpurun_out/sq/fwd -o run -- python3 $R/tools/fwd_bench.py > $R/gpurun_out/sq/fwd.log 2>&1 || { echo SQ_FAILED; tail -5 $R/gpurun_out/sq/fwd.log; exit 1; }
cd $R && python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/sq/fwd/**/*counter_collection.csv", recursive=True)[0]
agg = collections.OrderedDict()
for r in csv.DictReader(open(f)):
    if "pgemm" not in r["Kernel_Name"] and "pstream" not in r["Kernel_Name"]:
        continue
    k = (r["Kernel_Name"][:48], r.get("Grid_Size", ""), r["Dispatch_Id"])
    agg.setdefault(k, {})[r["Counter_Name"]] = float(r["Counter_Value"])
seen = set()
for (kn, g, d), v in agg.items():
    wc = v.get("SQ_WAVE_CYCLES", 0) or 1
    print(kn, g, d, {c: round(v.get(c, 0) / wc, 3) for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS")},
          "mfma_busy/busy", round(v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(v.get("SQ_BUSY_CYCLES", 1), 1), 3))
PY
