#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel stats, big-level exploration.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
step tests
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
step bench
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ -n "$PROFILE" ]; then
  step rocprof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-probe-peak --no-scale > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*stats*"
  python tools/prof_levels.py gpurun_out/prof/bench_kernel_trace.csv > gpurun_out/prof_levels.txt && cat gpurun_out/prof_levels.txt
fi
if [ -n "$EXPLORE" ]; then
  step explore
  timeout -k 10 300 python -u tools/explore.py $EXPLORE > gpurun_out/explore.log 2>&1 || { tail -5 gpurun_out/explore.log; exit 1; }
  tail -4 gpurun_out/explore.log
fi
echo "== done ($(date +%T))"
