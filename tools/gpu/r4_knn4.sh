#!/bin/bash
# round 4: kNN scan with a four-stage ring (three tiles in flight) against the
# three-stage one: parity tests of each build (ARTSBIR_LIB), then rocprofv3
# statistics of the retrieval leg; variants: art-sbir_amd/build_var/libknn4{a,b}.so
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for v in 0 a b; do
  if [ $v = 0 ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libknn4$v.so; fi
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_retrieval_gpu.py -m gpu -p no:cacheprovider > gpurun_out/knn4_$v.tests.log 2>&1 || { echo "TESTS FAIL $v"; tail -20 gpurun_out/knn4_$v.tests.log; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/knn4_$v.tests.log)"
  (cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/knn4_$v -o run --output-format csv -- python3 $R/tools/retr_bench.py > $R/gpurun_out/knn4_$v.log 2>&1) || { echo "FAIL $v"; tail -5 gpurun_out/knn4_$v.log; exit 1; }
  grep -o '"ms": [0-9.]*' gpurun_out/knn4_$v.log | head -1
  python3 - $v $R <<'PY'
import csv, sys
v, R = sys.argv[1], sys.argv[2]
for r in csv.DictReader(open(f"{R}/gpurun_out/knn4_{v}/run_kernel_stats.csv")):
    if "knn_scan_v2" in r["Name"]:
        print("scan", v, r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
