#!/bin/bash
# Full GPU pass: the -m gpu suite, then tools/gpu_session.sh with whatever steps the env selects
# (default: bench + rocprof per-level + PMC).  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
if [ -z "$BENCH$PROF$PMC$EXPLORE$TESTK" ]; then BENCH=1 PROF=1 PMC=1; fi
BENCH=$BENCH PROF=$PROF PMC=$PMC EXPLORE="$EXPLORE" TESTK="$TESTK" bash tools/gpu_session.sh
