#!/bin/bash
# The -m gpu suite, then Raft.cfg at the default chunk and at 2^27 slots, then configs[3] at the
# default; every GPU step under its own limit, stopping at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/chunk_sweep.sh 0 134217728 || exit 1
CFG="5 1 3 3" bash tools/chunk_sweep.sh 0 || exit 1
