#!/bin/bash
# Rehearse the N>1 bench path on ONE GPU: 2 ranks, gloo host collectives, both on cuda:0
# (RCCL refuses two ranks on one device; the 8-GPU RCCL run is the driver's).
#   /usr/local/graft/bin/gpurun --timeout 600 -- 'bash tools/rehearse_multi.sh'
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out"
cd "$ROOT"
EG_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --ballots 2000 \
  > gpurun_out/rehearse_gloo2.log 2>&1
tail -2 gpurun_out/rehearse_gloo2.log
