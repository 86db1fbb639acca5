#!/bin/bash
# round 5: kNN scan ablations at three vs four LDS stages (diagnostic builds
# build_var/libknn_a<abl>_n<nst>.so: hipcc -DKNN_ABL=<abl> -DKNN_NST=<nst> on
# retrieval.hip; abl 1 no list work, 3 neither list work nor MFMAs; wrong results
# by design): rocprofv3 average of knn_scan_v2_kernel<32> on the retrieval leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in base a3_n3 a3_n4 a1_n4 a0_n4; do
  if [ $v = base ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libknn_$v.so; fi
  rm -rf $R/gpurun_out/knn4_$v
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/knn4_$v -o run --output-format csv -- python3 $R/tools/retr_bench.py > $R/gpurun_out/knn4_$v.log 2>&1 || { echo "FAIL $v"; tail -5 $R/gpurun_out/knn4_$v.log; exit 1; }
  python3 - $v $R <<'PY'
import csv, sys
v, R = sys.argv[1], sys.argv[2]
for r in csv.DictReader(open(f"{R}/gpurun_out/knn4_{v}/run_kernel_stats.csv")):
    if "knn_scan_v2" in r["Name"]:
        print(v, r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
