set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --durations=15 --timeout 600 --timeout-method thread > gpurun_out/r03c_gpu_tests.log 2>&1
timeout -k 10 300 env EG_DIST_BACKEND=gloo python bench.py --gpus 2 --ballots 20000 --steps 2 --warmup 1 --modexp-n 4096 > gpurun_out/r03c_rehearse_gloo2.log 2>&1
