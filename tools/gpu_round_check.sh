#!/bin/bash
# Round-end evidence on one MI355X (run through gpurun):
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/gpu_round_check.sh r03d'
# the full -m gpu suite, then the kernel-trace + PMC profile of the default bench command
# (tools/profile_round.sh), on the library in the tree.
set -eo pipefail
TAG=${1:-r03d}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --durations=15 --timeout 600 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
echo "gpu tests: $(tail -1 gpurun_out/${TAG}_gpu_tests.log)"
if [ "${PROFILE:-1}" = 1 ]; then bash tools/profile_round.sh "$TAG"; fi
