#!/bin/bash
# configs[1] (bench.py's headline line) per variant on one box, each under its own limit; stops at the
# first failure.  Variants: "name=ENV=VAL,ENV=VAL" as tools/gpu_ab.sh (RMC_LIBRARY: a build_variant.sh build).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
mkdir -p gpurun_out/c2ab
for v in "$@"; do
  name=${v%%=*}; envs=${v#*=}
  ( IFS=','; for e in $envs; do [ -n "$e" ] && export "$e"; done; unset IFS
    exec timeout -k 10 120 python -u bench.py --workload c2 --no-cpu-baseline --no-probe-peak ) > gpurun_out/c2ab/$name.json 2> gpurun_out/c2ab/$name.err || { tail -5 gpurun_out/c2ab/$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/c2ab/$name.json "$name [$envs]"
done
