#!/bin/bash
# Round-3 A/B of the commit's parents-with-winners list (RMC_NZLIST) on one box: the -m gpu suite,
# Raft.cfg exhausted with and without it (tools/gpu_ab.sh), then the default bench line and the
# myrun.sh drop-in (when scratch_myrun/ holds the user's spec); each step under its own limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
mkdir -p gpurun_out/r03e
export TMPDIR=/tmp
TESTS=1 bash tools/gpu_ab.sh nz1= nz0=RMC_NZLIST=0 || exit 1
python tools/phase_sums.py gpurun_out/ab/nz1.log gpurun_out/ab/nz0.log || true
echo "== bench ($(date +%T))"
timeout -k 10 480 python -u bench.py > gpurun_out/r03e/bench.json 2> gpurun_out/r03e/bench.err || { tail gpurun_out/r03e/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r03e/bench.json')); a=d['at_scale']; print('bench', d['value'], d['ms_per_step'], a['seconds_to_exhaust'], a['first_run_seconds_incl_allocation'])"
if [ -d scratch_myrun ]; then
  echo "== myrun ($(date +%T))"
  bash tools/gpu_myrun.sh || exit 1
fi
echo "== done ($(date +%T))"
