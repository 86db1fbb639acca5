#!/bin/bash
# request-size read counters on known byte counts: tools/dgrad_bench.py shape 6
# (56^2 x 256 <- 64, kind 3 res1) per candidate, one pass of
# TCC_EA0_RDREQ_32B/_64B/_128B + TCC_EA0_RDREQ
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/reqchk
cd /tmp && export TMPDIR=/tmp
d=$R/gpurun_out/reqchk/s6
rm -rf $d
SHAPES=6 CFGS=16,18,22,0 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ --output-format csv -d $d -o run -- python3 $R/tools/dgrad_bench.py > $d.log 2>&1 || { echo FAIL; tail -5 $d.log; exit 1; }
python3 - $d <<'PY'
import sys, csv, glob, collections
sys.path.insert(0, sys.argv[1].rsplit("/gpurun_out", 1)[0] + "/profiles")
import summarize_pmc as sp
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
for k, (n, b, nreq, rd) in sp.load_req(f).items():
    print(f"{k:45s} {n:3d} launches  read {b / n / 1e9:7.3f} GB/launch  sized/rdreq {nreq / rd if rd else 0:.3f}")
PY
