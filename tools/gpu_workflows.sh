#!/bin/bash
# Round evidence of the non-bench configs on one MI355X (run through gpurun):
#   configs[0] (3 guardians, quorum 3, 25 ballots, gRPC trustees), configs[3] shape (5 guardians,
#   quorum 3, 2 missing; 1,000 ballots of which 50 spoiled), the trustee throughput bench, and
#   1M ballots end to end (configs[2] tally size, 2,000 spoiled).
set -eo pipefail
TAG=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/run_workflow.py -nguardians 3 -quorum 3 -nballots 25 > gpurun_out/${TAG}_workflow_config0.log 2>&1
timeout -k 10 300 python -u tools/run_workflow.py -nguardians 5 -quorum 3 -navailable 3 -nballots 1000 -nspoiled 50 > gpurun_out/${TAG}_workflow_config3_spoiled.log 2>&1
timeout -k 10 300 python -u tools/bench_trustee.py --texts 100000 > gpurun_out/${TAG}_bench_trustee.log 2>&1
timeout -k 10 600 python -u tools/run_workflow.py -nguardians 5 -quorum 3 -navailable 3 -nballots 1000000 -fbwindow 22 -chunk 250000 -nspoiled 2000 > gpurun_out/${TAG}_workflow_1M_4x5_w22_spoiled.log 2>&1
if [[ ${WORKFLOW_LARGE:-0} == 1 ]]; then
  # configs[4]'s manifest at 1M ballots through gRPC trustee processes (round 6)
  timeout -k 10 900 python -u tools/run_workflow.py -nguardians 5 -quorum 3 -navailable 3 -nballots 1000000 -ncontests 20 \
    -fbwindow 22 -chunk 125000 -nspoiled 500 > gpurun_out/${TAG}_workflow_1M_20x5_w22_spoiled.log 2>&1
fi
