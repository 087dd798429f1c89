#!/bin/bash
# Round-3 record of the final tree on one GPU box, every GPU step under its own time limit, stopping
# at the first failure: smoke, the default bench line, rocprofv3 kernel stats of bench (configs[1])
# and of Raft.cfg's exhaustion, PMC passes over Raft.cfg's first 40 levels, the one-rank RCCL
# sharded Raft.cfg exhaustion, and the myrun.sh drop-in (when scratch_myrun/ holds the user's spec).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=gpurun_out/final
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
step tests_commit_list
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread -k commit_list > $O/gpu_tests_commit_list.log 2>&1 || { tail -20 $O/gpu_tests_commit_list.log; exit 1; }
tail -1 $O/gpu_tests_commit_list.log
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step bench
timeout -k 10 480 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
step rocprof_bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_c2" -o bench -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-probe-peak --no-scale > $O/prof_c2.log 2>&1 || { tail -20 $O/prof_c2.log; exit 1; }
step rocprof_raftcfg
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_raftcfg" -o run -- python3 "$R/tools/explore.py" 3 2 3 3 --budget 200 > $O/prof_raftcfg.log 2>&1 || { tail -20 $O/prof_raftcfg.log; exit 1; }
grep RESULT $O/prof_raftcfg.log
step pmc_raftcfg
OUT=$O/pmc_raftcfg CFG="3 2 3 3 --levels 40" LIMIT=150 bash tools/pmc_scale.sh || exit 1
step rccl1
timeout -k 10 240 python -u tools/explore.py 3 2 3 3 --rccl1 --budget 200 > $O/rccl1_raftcfg.log 2>&1 || { tail -5 $O/rccl1_raftcfg.log; exit 1; }
grep RESULT $O/rccl1_raftcfg.log
if [ -d scratch_myrun ]; then
  step myrun
  bash tools/gpu_myrun.sh || exit 1
fi
echo "== done ($(date +%T))"
