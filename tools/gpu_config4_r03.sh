#!/bin/bash
# configs[4] evidence on one MI355X (gpurun): the full GPU suite, one GPU's 125,000-ballot share of
# configs[4] as a bench line, and 1M ballots x 100 selections end to end (5 guardians, quorum 3,
# 2 missing, 1,000 spoiled).
set -eo pipefail
TAG=${1:-r03i}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --durations=15 --timeout 600 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1
echo "gpu tests: $(tail -1 gpurun_out/${TAG}_gpu_tests.log)"
timeout -k 10 400 python bench.py --manifest large --ballots 125000 --steps 2 --warmup 1 --cpu-sample 0 --ct-encrypt 0 \
  --modexp-n 0 > gpurun_out/${TAG}_bench_config4_shard125k.log 2>&1
echo "config4 shard done"
timeout -k 10 600 python -u tools/run_workflow.py -nguardians 5 -quorum 3 -navailable 3 -nballots 1000000 \
  -ncontests 20 -nselections 5 -fbwindow 22 -chunk 125000 -nspoiled 1000 > gpurun_out/${TAG}_workflow_1M_20x5_config4.log 2>&1
echo all done
