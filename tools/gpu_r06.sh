#!/bin/bash
# Round-6 GPU checks on one MI355X (gpurun): every step under its own time limit, chained so the first
# failure ends the call.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'STEPS=kara,gloo8 bash tools/gpu_r06.sh r06d'
set -eo pipefail
TAG=${1:-r06a}
STEPS=${STEPS:-tests,bench}
mkdir -p gpurun_out
if [[ $STEPS == *ftest* ]]; then
  timeout -k 10 900 python -u -m pytest ${FTESTS} -m gpu -x -v --timeout 600 --timeout-method thread \
    > gpurun_out/${TAG}_gpu_tests_focus.log 2>&1
  echo "ftest: $(tail -n 1 gpurun_out/${TAG}_gpu_tests_focus.log)"
fi
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 \
    > gpurun_out/${TAG}_gpu_tests.log 2>&1
  echo "tests: $(tail -n 1 gpurun_out/${TAG}_gpu_tests.log)"
fi
if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
  echo "smoke: $(tail -n 1 gpurun_out/${TAG}_smoke.log)"
fi
if [[ $STEPS == *kara* ]]; then
  # separated product-then-REDC against the interleaved CIOS multiply (the price of any Karatsuba level)
  [[ -x tools/_ub_karatsuba ]] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize \
    -o tools/_ub_karatsuba tools/ubench_karatsuba.hip
  timeout -k 10 300 tools/_ub_karatsuba ${KARA_ITERS:-128} ${KARA_ROUNDS:-5} > gpurun_out/${TAG}_ubench_karatsuba.json
  echo "kara: $(cat gpurun_out/${TAG}_ubench_karatsuba.json | tail -c 400)"
fi
if [[ $STEPS == *threads* ]]; then
  # the caller's nthreads (RunRemoteWorkflowTest.java:140,180) through the per-element drop-in
  timeout -k 10 900 python -u tools/percall_threads.py ${THREADS:-11,32,64,128,256,512} \
    > gpurun_out/${TAG}_percall_threads.json 2> gpurun_out/${TAG}_percall_threads.err
  echo "threads: $(tail -n 12 gpurun_out/${TAG}_percall_threads.err)"
fi
if [[ $STEPS == *b125k* ]]; then
  # configs[2]'s per-GPU shard at N = 1 (the weak-scaling curve's per-GPU normaliser)
  timeout -k 10 400 python -u bench.py --gpus 1 --ballots 125000 --steps 5 --warmup 1 \
    > gpurun_out/${TAG}_bench_125k.log 2> gpurun_out/${TAG}_bench_125k.err
  echo "b125k: $(tail -c 300 gpurun_out/${TAG}_bench_125k.log)"
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
if [[ $STEPS == *pipe* ]]; then
  # configs[4] full pipeline at one GPU's 125,000-ballot share (bench.py --pipeline full)
  timeout -k 10 600 python bench.py --pipeline full > gpurun_out/${TAG}_bench_pipeline_config4.log 2>&1
  echo "pipe: $(tail -c 300 gpurun_out/${TAG}_bench_pipeline_config4.log)"
fi
if [[ $STEPS == *prof* ]]; then
  bash tools/profile_round.sh ${TAG}
fi
if [[ $STEPS == *ab142* ]]; then
  # 142 CIOS steps (R = 2^4118, the default) against all 144 (EG_CIOS_FULL=1), per shader clock, three
  # interleaved rounds of the configs[1] verify
  AB_MODE=verify AB_NB=10000 AB_WB=22 timeout -k 10 900 python tools/ab_mm.py s142= s144=-DEG_CIOS_FULL=1 s142= \
    s144=-DEG_CIOS_FULL=1 s142= s144=-DEG_CIOS_FULL=1 > gpurun_out/${TAG}_ab_steps.log 2>&1
  echo "ab142: $(tail -c 900 gpurun_out/${TAG}_ab_steps.log)"
fi
if [[ $STEPS == *strictfail* ]]; then
  # --strict-rccl against a real RCCL refusal: 2 ranks on one device (EG_RANKS_SHARE_GPU=1); the run must
  # fail (non-zero) on every rank, quickly, with no host-exchange line
  set +e
  t0=$SECONDS
  timeout -k 10 300 env EG_RANKS_SHARE_GPU=1 python bench.py --gpus 2 --steps 1 --warmup 1 \
    --ballots 2000 --fb-window 12 --cpu-sample 0 --modexp-n 0 --ct-encrypt 0 > gpurun_out/${TAG}_strict_fail.log 2>&1
  rc=$?
  set -e
  echo "exit status $rc after $((SECONDS - t0)) s" >> gpurun_out/${TAG}_strict_fail.log
  echo "strictfail: rc=$rc $(tail -c 800 gpurun_out/${TAG}_strict_fail.log)"
  [[ $rc -ne 0 && $rc -ne 124 && $rc -ne 137 && $rc -ne 127 ]]
fi
