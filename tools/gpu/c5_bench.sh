#!/bin/bash
# C5 leg only (ViT-B/16 fp8 triplet step), small steps; memory and time check first at a reduced batch
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --no-cpu-baseline --no-retrieval --no-embed --no-loss-check --no-profile --steps 2 --warmup 1 --c5 --c5-batch ${C5B:-512} > gpurun_out/c5.json 2> gpurun_out/c5.err; rc=$?
echo "rc=$rc"; tail -3 gpurun_out/c5.err; python3 -c "import json; d=json.loads(open('gpurun_out/c5.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('c5'))"
