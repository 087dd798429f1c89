#!/bin/bash
# Round-3 measurement session: PMC passes over Raft.cfg's first 40 levels, the default bench line,
# and the drop-in launcher's phase times (scratch_myrun/ holds the user's Raft.tla / Raft.cfg when present).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
step pmc_raftcfg
OUT=gpurun_out/pmc_raftcfg CFG="3 2 3 3 --levels 40" LIMIT=150 bash tools/pmc_scale.sh || exit 1
step bench
timeout -k 10 480 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ -d scratch_myrun ]; then
  step myrun
  ( cd scratch_myrun && RMC_LAUNCHER_TIMES=1 timeout -k 10 200 bash ../tla-raft_amd/myrun.sh > ../gpurun_out/myrun_stdout.txt 2> ../gpurun_out/myrun_stderr.txt; cp raft.log ../gpurun_out/myrun_raft.log ) || exit 1
  grep "raftmc:" gpurun_out/myrun_raft.log gpurun_out/myrun_stderr.txt; tail -3 gpurun_out/myrun_raft.log
fi
if [ -f tla-raft_amd/build_prof/librmc.so ]; then
  step phase_prof
  RMC_LIBRARY=tla-raft_amd/build_prof/librmc.so timeout -k 10 200 python -u tools/phase_prof.py 3 2 3 3 --levels 40 > gpurun_out/phase_raftcfg_l40.txt 2>&1 || { tail -5 gpurun_out/phase_raftcfg_l40.txt; exit 1; }
  cat gpurun_out/phase_raftcfg_l40.txt
fi
echo "== done ($(date +%T))"
