#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
ARTSBIR_KNN_STAT=1 ARTSBIR_KNN_KB=1 timeout -k 10 300 python -u tools/retr_leg.py 2>&1 | grep noise || exit 1
