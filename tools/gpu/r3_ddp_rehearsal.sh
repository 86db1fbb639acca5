#!/bin/bash
# N = 2 rehearsal of bench.py's data-parallel path on the one-GPU box: two ranks
# share the device over gloo (RCCL needs one GPU per rank); smaller batches so
# both ranks' activations fit the 288 GB
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
ARTSBIR_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --batch 96 --c5-batch 64 \
  --no-cpu-baseline --no-profile > gpurun_out/r3_ddp2.json 2> gpurun_out/r3_ddp2.err; rc=$?
echo "rc=$rc"; tail -c 1500 gpurun_out/r3_ddp2.json; grep -iE "error|Traceback" gpurun_out/r3_ddp2.err | head -5; exit $rc
