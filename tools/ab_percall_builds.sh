#!/bin/bash
# Per-element workflow rates of several builds on one box, interleaved over two rounds (the
# per-element rates move from box to box with the host).  A build is a git worktree under _ab/<name>
# (git worktree add _ab/<name> <rev>, then its __graft_entry__.build()), or "new" for this tree, or
# "env:<VAR=value>[,VAR=value...]" for this tree under that environment (e.g. env:EG_COALESCE_WINDOW_US=20).
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/ab_percall_builds.sh r05j b92 new'
set -eo pipefail
TAG=${1:?tag}
shift
N=${N:-1100}  # ballots; T: caller threads (default 11)
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out"
OUT="$ROOT/gpurun_out/${TAG}_ab_percall_builds.log"
: > "$OUT"
for round in 1 2; do
  for b in "$@"; do
    envs=()
    if [[ $b == new ]]; then bin="$ROOT/electionguard-remote_amd/host/_build/percall_workflow"
    elif [[ $b == env:* ]]; then bin="$ROOT/electionguard-remote_amd/host/_build/percall_workflow"; IFS=, read -ra envs <<< "${b#env:}"
    else bin="$ROOT/_ab/$b/electionguard-remote_amd/host/_build/percall_workflow"; fi
    echo "round $round $b: $(env "${envs[@]}" timeout -k 10 300 "$bin" "$N" "${T:-11}" | tail -n 1)" >> "$OUT"
    tail -n 1 "$OUT" | cut -c1-80
  done
done
