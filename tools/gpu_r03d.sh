#!/bin/bash
# Round-3 check of the trace's host tier (huge-page blocks + pinned staging): the -m gpu suite, the
# myrun.sh drop-in (when scratch_myrun/ holds the user's spec; shell wall incl. process exit), and the
# default bench line; each GPU step under its own limit, stopping at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=gpurun_out/r03d
mkdir -p $O
export TMPDIR=/tmp
echo "== tests ($(date +%T))"
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
if [ -d scratch_myrun ]; then
  echo "== myrun ($(date +%T))"
  bash tools/gpu_myrun.sh || exit 1
fi
echo "== bench ($(date +%T))"
timeout -k 10 480 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
echo "== done ($(date +%T))"
