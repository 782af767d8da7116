#!/bin/bash
# Round-3 closing evidence on one MI355X (gpurun): full GPU suite + kernel-trace/PMC profile of the
# default bench (tools/gpu_round_check.sh), a clean default bench line, configs[4] at one GPU,
# the 100k-ballot workflow with 2,000 spoiled ballots and the 2-rank gloo rehearsal of bench.py.
set -eo pipefail
TAG=${1:-r03g}
bash tools/gpu_round_check.sh "$TAG"
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_final.log 2>&1
echo "bench: $(tail -c 200 gpurun_out/${TAG}_bench_final.log)"
timeout -k 10 300 python bench.py --manifest large --ballots 10000 --cpu-sample 0 --ct-encrypt 0 --modexp-n 0 \
  > gpurun_out/${TAG}_bench_config4_10k.log 2>&1
timeout -k 10 300 python -u tools/run_workflow.py -nguardians 5 -quorum 3 -navailable 3 -nballots 100000 -chunk 100000 \
  -nspoiled 2000 > gpurun_out/${TAG}_workflow_100k_spoiled2000.log 2>&1
timeout -k 10 300 env EG_DIST_BACKEND=gloo python bench.py --gpus 2 --ballots 20000 --steps 2 --warmup 1 \
  --modexp-n 4096 > gpurun_out/${TAG}_rehearse_gloo2.log 2>&1
echo all done
