#!/bin/bash
# One GPU-box session: smoke, the default bench line, rocprofv3 kernel stats of the bench workload,
# PMC passes (one counter group per run, MI355X_MICROARCH.md rocprofv3 section).  Every GPU step
# has its own time limit; the script stops at the first failure.
#   TESTS=1   also run the -m gpu suite first
#   NOBENCH=1 skip the default bench line (profiles only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
if [ -n "$TESTS" ]; then
  step tests
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
if [ -z "$NOBENCH" ]; then
  step bench
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-probe-peak --no-scale > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
python tools/prof_levels.py gpurun_out/prof/bench_kernel_trace.csv > gpurun_out/prof_levels.txt && cat gpurun_out/prof_levels.txt
step pmc
bash tools/pmc.sh && python tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_c2.json
echo "== done ($(date +%T))"
