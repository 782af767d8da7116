#!/bin/bash
# Round-4 GPU checks on one MI355X (gpurun): the GPU suite, the default bench line and the 2-rank
# gloo rehearsal of bench.py's N > 1 path (cpu_baseline + vs_baseline on rank 0's line).
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/gpu_r04.sh r04a'
set -eo pipefail
TAG=${1:-r04a}
STEPS=${STEPS:-tests,bench,gloo2}
mkdir -p gpurun_out
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gpu_tests.log 2>&1
  echo "tests: $(tail -n 1 gpurun_out/${TAG}_gpu_tests.log)"
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1
  echo "bench: $(tail -c 300 gpurun_out/${TAG}_bench.log)"
fi
if [[ $STEPS == *gloo2* ]]; then
  timeout -k 10 300 env EG_DIST_BACKEND=gloo python bench.py --gpus 2 --ballots 20000 --steps 2 --warmup 1 \
    --modexp-n 4096 --cpu-seconds 4 > gpurun_out/${TAG}_rehearse_gloo2.log 2>&1
  echo "gloo2: $(tail -c 300 gpurun_out/${TAG}_rehearse_gloo2.log)"
fi
if [[ $STEPS == *ftest* ]]; then
  timeout -k 10 600 python -u -m pytest ${FTESTS} -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gpu_tests_focus.log 2>&1
  echo "ftest: $(tail -n 1 gpurun_out/${TAG}_gpu_tests_focus.log)"
fi
if [[ $STEPS == *shapes* ]]; then
  timeout -k 10 900 python tools/coalesce_shapes.py > gpurun_out/${TAG}_coalesce_shapes.json 2> gpurun_out/${TAG}_coalesce_shapes.err
  echo "shapes: $(grep -E 'blocking|crossover' gpurun_out/${TAG}_coalesce_shapes.json | tr -d '\n')"
fi
if [[ $STEPS == *abcomb* ]]; then
  # interleaved same-box A/B of the verifier's selection comb (rows x column blocks), per shader clock
  AB_MODE=verify AB_NB=10000 AB_WB=22 timeout -k 10 900 python tools/ab_mm.py cur= cur@sel42= cur@sel44= cur= \
    cur@sel42= cur@sel44= cur= cur@sel42= cur@sel44= > gpurun_out/${TAG}_ab_selcomb.log 2>&1
  echo "abcomb: $(tail -c 600 gpurun_out/${TAG}_ab_selcomb.log)"
fi
if [[ $STEPS == *rccl* ]]; then
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29541 tools/rccl_selfcheck.py > gpurun_out/${TAG}_rccl_selfcheck.log 2>&1
  echo "rccl: $(tail -n 2 gpurun_out/${TAG}_rccl_selfcheck.log)"
fi
if [[ $STEPS == *ptest* ]]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_comm.py -m gpu -x -v --timeout 300 \
    --timeout-method thread > gpurun_out/${TAG}_gpu_tests_pipeline.log 2>&1
  echo "ptest: $(tail -n 1 gpurun_out/${TAG}_gpu_tests_pipeline.log)"
fi
if [[ $STEPS == *pipe1* ]]; then
  timeout -k 10 600 python bench.py --pipeline full > gpurun_out/${TAG}_bench_pipeline_config4.log 2>&1
  echo "pipe1: $(tail -c 400 gpurun_out/${TAG}_bench_pipeline_config4.log)"
fi
if [[ $STEPS == *pipeg2* ]]; then
  timeout -k 10 600 env EG_DIST_BACKEND=gloo python bench.py --gpus 2 --pipeline full --ballots 20000 --steps 1 \
    --warmup 1 --modexp-n 0 --cpu-seconds 4 > gpurun_out/${TAG}_rehearse_gloo2_pipeline.log 2>&1
  echo "pipeg2: $(tail -c 400 gpurun_out/${TAG}_rehearse_gloo2_pipeline.log)"
fi
if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
  echo "smoke: $(tail -n 1 gpurun_out/${TAG}_smoke.log)"
fi
if [[ $STEPS == *driver* ]]; then
  # the driver's N = 1 command
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_driver_args.log 2>&1
  echo "driver: $(tail -c 300 gpurun_out/${TAG}_bench_driver_args.log)"
fi
echo all done
