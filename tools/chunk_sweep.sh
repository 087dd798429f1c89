#!/bin/bash
# Raft.cfg exhausted on one GPU at each chunk size (successor slots per chunk) given as an argument
# (0 = the default); prints the closing line per size.  Each run under its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
mkdir -p gpurun_out/chunk
for G in "$@"; do
  echo "== chunk $G ($(date +%T))"
  timeout -k 10 240 python -u tools/explore.py ${CFG:-3 2 3 3} --budget 200 --chunk "$G" > "gpurun_out/chunk/$G.log" 2>&1 || { tail -5 "gpurun_out/chunk/$G.log"; exit 1; }
  tail -n 1 "gpurun_out/chunk/$G.log"
done
