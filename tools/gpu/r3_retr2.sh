#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for kb in 0 1; do
ARTSBIR_KNN_STAT=1 ARTSBIR_KNN_KB=$kb timeout -k 10 300 python -u tools/retr_leg.py 2>&1 | grep noise || exit 1
done
