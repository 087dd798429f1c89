#!/bin/bash
# A/B timing on one GPU box: Raft.cfg exhausted level by level (tools/explore.py 3 2 3 3) once per
# variant, each under its own limit; stops at the first failure.  Variants: "name=ENV=VAL,ENV=VAL"
# (RMC_LIBRARY selects a tools/build_variant.sh build), e.g.
#   bash tools/gpu_ab.sh base= nosplit=RMC_SPLIT_MIN=0 ce0=RMC_LIBRARY=tla-raft_amd/build_ce0/librmc.so
# CFG (default "3 2 3 3"), TESTS=1 (the -m gpu suite first) and BENCHC2=1 (bench.py's configs[1] line
# per variant) are read from the environment.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
CFG=${CFG:-3 2 3 3}
if [ -n "$TESTS" ]; then
  echo "== tests ($(date +%T))"
  timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/ab/gpu_tests.log 2>&1 || { tail -30 gpurun_out/ab/gpu_tests.log; exit 1; }
  tail -1 gpurun_out/ab/gpu_tests.log
fi
for v in "$@"; do
  name=${v%%=*}; envs=${v#*=}
  echo "== $name [$envs] ($(date +%T))"
  ( IFS=','; for e in $envs; do [ -n "$e" ] && export "$e"; done; unset IFS
    exec timeout -k 10 ${LIMIT:-240} python -u tools/explore.py $CFG --budget ${BUDGET:-200} ) > gpurun_out/ab/$name.log 2>&1 || { tail -5 gpurun_out/ab/$name.log; exit 1; }
  grep RESULT gpurun_out/ab/$name.log
  if [ -n "$BENCHC2" ]; then  # the headline line (configs[1]) with the same variant
    ( IFS=','; for e in $envs; do [ -n "$e" ] && export "$e"; done; unset IFS
      exec timeout -k 10 120 python -u bench.py --workload c2 --no-cpu-baseline --no-probe-peak ) > gpurun_out/ab/$name.bench.json 2> gpurun_out/ab/$name.bench.err || { tail -5 gpurun_out/ab/$name.bench.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['ms_per_step'])" gpurun_out/ab/$name.bench.json
  fi
done
echo "== done ($(date +%T))"
