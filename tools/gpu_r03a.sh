#!/bin/bash
# Round-3 first GPU session: full -m gpu suite, smoke, default bench line, at-scale PMC passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
step tests
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
step bench
timeout -k 10 420 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
step pmc_scale
bash tools/pmc_scale.sh || exit 1
echo "== done ($(date +%T))"
