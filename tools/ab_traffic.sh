#!/bin/bash
# Interleaved A/B of k_pow builds through bench.py, with PMC passes (run on the GPU box via gpurun):
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'VARIANTS="base x2 peel" bash tools/ab_traffic.sh r03d'
# Each variant is a prebuilt library tools/_ab/libeg_<name>.so (tools/ab_mm.py build(), the
# flags of __graft_entry__), loaded through EG_LIB:
#   base: the production kernel;
#   x2:   -DEG_TRAFFIC_X2=1, whose comb multiplies also read a far job's table entry (an L2
#         miss) into a discarded LDS word -- more HBM bytes per launch at a nearly equal VALU count;
#   peel, loop2, head: any other source revision built the same way (r03d: the peeled CIOS step;
#         r03j: the op loop with the multiply kinds split from the handlers).
# Rounds of bench runs (base, x2, ..., base, x2, ...) give ballots/s and the held clock; one
# FETCH_SIZE, one WRITE_SIZE and one SQ pass per variant give HBM bytes and VALU instructions per
# launch; tools/ab_traffic_summary.py folds them into one JSON.
set -eo pipefail
TAG=${1:-r03d}
VARIANTS=${VARIANTS:-base x2}
ROUNDS=${ROUNDS:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/ab_traffic_$TAG
ARGS="--cpu-sample 0 --ct-encrypt 0 --modexp-n 0"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
for lib in $VARIANTS; do
  test -f "tools/_ab/libeg_$lib.so" || { echo "missing tools/_ab/libeg_$lib.so (build it in the container)"; exit 1; }
done
for round in $(seq 1 "$ROUNDS"); do
  for lib in $VARIANTS; do
    EG_LIB=$ROOT/tools/_ab/libeg_$lib.so timeout -k 10 240 python3 bench.py $ARGS > "$OUT/bench_${lib}_$round.log" 2>&1
    echo "bench $lib round $round: $(python3 -c 'import json, sys; print(json.loads(open(sys.argv[1]).read().splitlines()[-1])["value"])' "$OUT/bench_${lib}_$round.log")"
  done
done
for lib in $VARIANTS; do
  EG_LIB=$ROOT/tools/_ab/libeg_$lib.so timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/${lib}_FETCH_SIZE" -o run \
    --output-format csv -- python3 bench.py $ARGS > "$OUT/bench_${lib}_FETCH_SIZE.log" 2>&1
  EG_LIB=$ROOT/tools/_ab/libeg_$lib.so timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/${lib}_WRITE_SIZE" -o run \
    --output-format csv -- python3 bench.py $ARGS > "$OUT/bench_${lib}_WRITE_SIZE.log" 2>&1
  EG_LIB=$ROOT/tools/_ab/libeg_$lib.so timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE -d "$OUT/${lib}_SQ" \
    -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/bench_${lib}_SQ.log" 2>&1
  echo "pmc $lib done"
done
python3 tools/ab_traffic_summary.py --dir "$OUT" --variants $VARIANTS > "$OUT/summary.json"
cat "$OUT/summary.json"
