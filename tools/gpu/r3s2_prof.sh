#!/bin/bash
# per-(kernel, shape) profile of the C2 step with the current tune table:
# overlapped (as timed) and main stream alone
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/step_profile.py --tune-cache profiles/tune_r3s2.txt --top 90 > gpurun_out/s2_prof_overlap.txt 2>&1 || { echo PROF_FAILED; tail -5 gpurun_out/s2_prof_overlap.txt; exit 1; }
timeout -k 10 300 python -u tools/step_profile.py --tune-cache profiles/tune_r3s2.txt --mode skip --top 90 > gpurun_out/s2_prof_main.txt 2>&1 || { echo PROF_FAILED; tail -5 gpurun_out/s2_prof_main.txt; exit 1; }
head -3 gpurun_out/s2_prof_overlap.txt; head -3 gpurun_out/s2_prof_main.txt
