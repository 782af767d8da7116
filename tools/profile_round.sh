#!/bin/bash
# Kernel-trace + PMC profile of the default bench command (run on the GPU box via gpurun):
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/profile_round.sh r01'
# Passes (separate processes; PMC passes never combine with trace domains):
#   1. rocprofv3 --kernel-trace --stats   (per-kernel durations; k_pow average)
#   2. --pmc FETCH_SIZE                   (TCC memory-side reads, KB; x2 on gfx950)
#   3. --pmc WRITE_SIZE
#   4. --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
# then tools/prof_summary.py folds the CSVs into profiles/<tag>_*.
set -eo pipefail
TAG=${1:-r02}
BENCH_ARGS=${BENCH_ARGS:-}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 bench.py $BENCH_ARGS > "$OUT/bench_trace.log" 2>&1
echo "trace pass done"
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
  -- python3 bench.py --cpu-sample 0 $BENCH_ARGS > "$OUT/bench_fetch.log" 2>&1
echo "fetch pass done"
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
  -- python3 bench.py --cpu-sample 0 $BENCH_ARGS > "$OUT/bench_write.log" 2>&1
echo "write pass done"
timeout -k 10 420 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d "$OUT/sq" -o run --output-format csv \
  -- python3 bench.py --cpu-sample 0 $BENCH_ARGS > "$OUT/bench_sq.log" 2>&1
echo "sq pass done"
python3 tools/prof_summary.py --dir "$OUT" --tag "$TAG"
