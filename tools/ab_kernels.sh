#!/bin/bash
# Per-kernel durations of one verify workload for each A/B library (tools/_ab/libeg_<name>.so):
#   bash tools/ab_kernels.sh head norm
# rocprofv3 kernel-trace stats only (no counters), one process per library.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
for name in "$@"; do
  OUT=$ROOT/gpurun_out/abk_$name
  mkdir -p "$OUT"
  EG_LIB=$ROOT/tools/_ab/libeg_$name.so AB_NB=${AB_NB:-10000} AB_WB=${AB_WB:-22} timeout -k 10 300 \
    rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- python3 tools/ab_verify_once.py > "$OUT/log.txt" 2>&1
  echo "$name done"
done
