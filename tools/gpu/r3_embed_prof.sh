#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/embed_pass.py 3 --profile > gpurun_out/r3_embed_prof.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r3_embed_prof.txt | head -45; exit $rc
