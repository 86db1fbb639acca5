#!/bin/bash
# round 5 (after the prefetch-depth fix and chunk balancing): kNN scan timing ablations (diagnostic builds art-sbir_amd/build_var/libknnabl{1,2,3}.so,
# hipcc -DKNN_ABL=n on retrieval.hip, linked with the other objects of build/;: 1 no list work, 2 no MFMAs, 3 neither; wrong results by design):
# rocprofv3 statistics of the retrieval leg per build, the scan kernel's average duration
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in 0 1 2 3; do
  if [ $v = 0 ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libknnabl$v.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/knn_abl$v -o run --output-format csv -- python3 $R/tools/retr_bench.py > $R/gpurun_out/knn_abl$v.log 2>&1 || { echo "FAIL $v"; tail -5 $R/gpurun_out/knn_abl$v.log; exit 1; }
  python3 - $v $R <<'PY'
import csv, sys
v, R = sys.argv[1], sys.argv[2]
for r in csv.DictReader(open(f"{R}/gpurun_out/knn_abl{v}/run_kernel_stats.csv")):
    if "knn_scan_v2" in r["Name"]:
        print("abl", v, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
