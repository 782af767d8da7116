#!/bin/bash
# Rehearse the N>1 bench path on ONE GPU: NPROC ranks (default 2), gloo host collectives,
# all on cuda:0 (RCCL refuses two ranks on one device; the 8-GPU RCCL run is the driver's).
# With more than 2 ranks the fixed-base window is lowered (FBW, default 20 = 8 GB per table)
# so that every rank's g and K tables fit in one GPU's 288 GB together.
#   /usr/local/graft/bin/gpurun --timeout 600 -- 'NPROC=4 bash tools/rehearse_multi.sh'
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
NPROC=${NPROC:-2}
if [ "$NPROC" -gt 2 ]; then FBW=${FBW:-20}; else FBW=${FBW:-22}; fi
mkdir -p "$ROOT/gpurun_out"
cd "$ROOT"
EG_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$NPROC" \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus "$NPROC" --steps 2 --warmup 1 --ballots 2000 \
  --fb-window "$FBW" --modexp-n 65536 > "gpurun_out/rehearse_gloo$NPROC.log" 2>&1
tail -2 "gpurun_out/rehearse_gloo$NPROC.log"
