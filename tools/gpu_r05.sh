#!/bin/bash
# Round-5 GPU checks on one MI355X (gpurun): every step under its own time limit, chained so the first
# failure ends the call.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'STEPS=ftest FTESTS="tests/test_gpu_mexp.py" bash tools/gpu_r05.sh r05a'
set -eo pipefail
TAG=${1:-r05a}
STEPS=${STEPS:-tests,bench}
mkdir -p gpurun_out
if [[ $STEPS == *ftest* ]]; then
  timeout -k 10 900 python -u -m pytest ${FTESTS} -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gpu_tests_focus.log 2>&1
  echo "ftest: $(tail -n 1 gpurun_out/${TAG}_gpu_tests_focus.log)"
fi
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gpu_tests.log 2>&1
  echo "tests: $(tail -n 1 gpurun_out/${TAG}_gpu_tests.log)"
fi
if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
  echo "smoke: $(tail -n 1 gpurun_out/${TAG}_smoke.log)"
fi
if [[ $STEPS == *percall* ]]; then
  timeout -k 10 600 python tools/percall_workflow.py ${PERCALL_ARGS} > gpurun_out/${TAG}_percall.json \
    2> gpurun_out/${TAG}_percall.err
  echo "percall: $(tail -c 1500 gpurun_out/${TAG}_percall.json)"
fi
if [[ $STEPS == *shapes* ]]; then
  timeout -k 10 900 python tools/coalesce_shapes.py > gpurun_out/${TAG}_coalesce_shapes.json 2> gpurun_out/${TAG}_coalesce_shapes.err
  echo "shapes: $(grep -E 'blocking|crossover' gpurun_out/${TAG}_coalesce_shapes.json | tr -d '\n')"
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1
  echo "bench: $(tail -c 400 gpurun_out/${TAG}_bench.log)"
fi
if [[ $STEPS == *gloo8* ]]; then
  # bench.py's N = 8 launcher shape on one MI355X: 8 ranks, host (gloo) exchange, 12-bit tables so
  # eight ranks' fixed-base tables share the card
  timeout -k 10 900 env EG_DIST_BACKEND=gloo python bench.py --gpus 8 --steps 2 --warmup 1 --ballots 2000 \
    --fb-window 12 > gpurun_out/${TAG}_rehearse_gloo8.log 2>&1
  echo "gloo8: $(tail -c 600 gpurun_out/${TAG}_rehearse_gloo8.log)"
fi
if [[ $STEPS == *ctpmc* ]]; then
  # constant-time per-wave kernel: VALU instructions per dispatch for exponent 0 against 2^256-1
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 420 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d gpurun_out/${TAG}_ctpmc -o run --output-format csv \
    -- python3 tools/ct_schedule.py > gpurun_out/${TAG}_ctpmc.log 2>&1
  python3 tools/ct_schedule_summary.py gpurun_out/${TAG}_ctpmc gpurun_out/${TAG}_ctpmc.log > gpurun_out/${TAG}_ct_schedule.txt
  echo "ctpmc: $(tail -n 8 gpurun_out/${TAG}_ct_schedule.txt)"
fi
if [[ $STEPS == *abfb* ]]; then
  # LDS-staged fixed-base tables against the HBM radix tables
  timeout -k 10 600 python tools/ab_fb_lds.py ${ABFB_N:-262144} ${ABFB_ROUNDS:-5} > gpurun_out/${TAG}_ab_fb_lds.json \
    2> gpurun_out/${TAG}_ab_fb_lds.err
  echo "abfb: $(tail -c 900 gpurun_out/${TAG}_ab_fb_lds.json)"
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  AB_ROUNDS=1 timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_abfb_pmc -o run --output-format csv \
    -- python3 tools/ab_fb_lds.py ${ABFB_N:-262144} > gpurun_out/${TAG}_abfb_pmc.log 2>&1
  python3 tools/ab_fb_lds_pmc.py gpurun_out/${TAG}_abfb_pmc ${ABFB_N:-262144} > gpurun_out/${TAG}_abfb_traffic.txt
  echo "abfb pmc: $(cat gpurun_out/${TAG}_abfb_traffic.txt)"
fi
if [[ $STEPS == *abw4* ]]; then
  # k_pow at 4 waves/SIMD (EG_MIN_WAVES=4: 128 VGPRs, spills to AGPRs / scratch) against 3, per clock,
  # three interleaved rounds of the configs[1] verify
  AB_MODE=verify AB_NB=10000 AB_WB=22 timeout -k 10 1200 python tools/ab_mm.py w3= w4=-DEG_MIN_WAVES=4 w3= \
    w4=-DEG_MIN_WAVES=4 w3= w4=-DEG_MIN_WAVES=4 > gpurun_out/${TAG}_ab_w4.log 2>&1
  echo "abw4: $(tail -c 900 gpurun_out/${TAG}_ab_w4.log)"
fi
if [[ $STEPS == *lat* ]]; then
  # per-wave latency A/B (tools/ab_wave_latency.py), interleaved; LAT_ENVS: ';'-separated env sets
  IFS=';' read -ra LE <<< "${LAT_ENVS:-EG_WAVE_R2L=256;EG_WAVE_R2L=0}"
  for r in $(seq ${LAT_ROUNDS:-2}); do
    for envs in "${LE[@]}"; do
      env $envs timeout -k 10 ${LAT_TIMEOUT:-300} python tools/ab_wave_latency.py ${LAT_CALLS:-200} >> gpurun_out/${TAG}_wave_latency.jsonl \
        2>> gpurun_out/${TAG}_wave_latency.err
    done
  done
  echo "lat: $(cat gpurun_out/${TAG}_wave_latency.jsonl)"
fi
if [[ $STEPS == *evid* ]]; then
  # configs[4] full pipeline at one GPU's 125,000-ballot share; the N = 2 launcher shape at configs[2]'s
  # full per-rank shard (125,000 ballots per rank) over gloo, both ranks on this one MI355X
  timeout -k 10 600 python bench.py --pipeline full > gpurun_out/${TAG}_bench_pipeline_config4.log 2>&1
  echo "pipe: $(tail -c 300 gpurun_out/${TAG}_bench_pipeline_config4.log)"
  timeout -k 10 600 env EG_DIST_BACKEND=gloo python bench.py --gpus 2 --ballots 125000 --steps 2 --warmup 1 \
    > gpurun_out/${TAG}_rehearse_gloo2_config2_full.log 2>&1
  echo "gloo2: $(tail -c 300 gpurun_out/${TAG}_rehearse_gloo2_config2_full.log)"
fi
