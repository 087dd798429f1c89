#!/bin/bash
# Round-3: the -m gpu suite, then the one-rank RCCL sharded Raft.cfg exhaustion with and without the
# commit's parents-with-winners list (RMC_NZLIST), each step under its own limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=gpurun_out/r03f
mkdir -p $O
export TMPDIR=/tmp
echo "== tests ($(date +%T))"
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for v in nz1 nz0; do
  echo "== rccl1 $v ($(date +%T))"
  if [ $v = nz0 ]; then export RMC_NZLIST=0; fi
  timeout -k 10 240 python -u tools/explore.py 3 2 3 3 --rccl1 --budget 200 > $O/rccl1_$v.log 2>&1 || { tail -5 $O/rccl1_$v.log; exit 1; }
  grep RESULT $O/rccl1_$v.log
done
echo "== done ($(date +%T))"
