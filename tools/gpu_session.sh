#!/bin/bash
# One GPU-box session, steps picked by env (each with its own time limit; stop at the first failure):
#   BENCH=1     default bench line              PROF=1   rocprofv3 kernel trace + per-level view
#   PMC=1       PMC passes (tools/pmc.sh)       TESTK=expr   pytest -m gpu -k expr
#   EXPLORE="n V E R budget"   one configuration level by level (tools/explore.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
if [ -n "$BENCH" ]; then
  step bench
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [ -n "$PROF" ]; then
  step rocprof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-probe-peak --no-scale > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
  python tools/prof_levels.py gpurun_out/prof/bench_kernel_trace.csv 37 --per-level > gpurun_out/prof_levels.txt && head -12 gpurun_out/prof_levels.txt
fi
if [ -n "$PMC" ]; then
  step pmc
  bash tools/pmc.sh && python tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_c2.json || exit 1
fi
if [ -n "$EXPLORE" ]; then
  set -- $EXPLORE
  step "explore $1 $2 $3 $4"
  timeout -k 10 $(( $5 + 120 )) python -u tools/explore.py $1 $2 $3 $4 --budget $5 > gpurun_out/explore_n$1_v$2_e$3_r$4.log 2>&1 || { tail -5 gpurun_out/explore_n$1_v$2_e$3_r$4.log; exit 1; }
  tail -4 gpurun_out/explore_n$1_v$2_e$3_r$4.log
fi
if [ -n "$TESTK" ]; then
  step "tests -k $TESTK"
  timeout -k 10 600 python -u -m pytest tests/ -m gpu -k "$TESTK" -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_k.log 2>&1 || { tail -30 gpurun_out/gpu_tests_k.log; exit 1; }
  tail -3 gpurun_out/gpu_tests_k.log
fi
echo "== done ($(date +%T))"
