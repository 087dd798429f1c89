#!/bin/bash
# Device-loop submission sweep on configs[1]: bench ms/step for each (levels per group, groups
# ahead, microseconds of waiting between stream queries[, library build dir]) given as "G:A:Q[:DIR]"
# arguments (DIR e.g. build_n3w6c1g32 from tools/build_variant.sh; default build).  One bench process per
# variant, each under its own time limit; stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
mkdir -p gpurun_out/dl_sweep
for v in "$@"; do
  IFS=: read -r G A Q D <<< "$v"
  D=${D:-build}
  echo "== G=$G A=$A Q=$Q lib=$D ($(date +%T))"
  RMC_LIBRARY="$R/tla-raft_amd/$D/librmc.so" RMC_DL_GROUP=$G RMC_DL_AHEAD=$A RMC_DL_QUERY_US=$Q timeout -k 10 120 python -u bench.py --steps 40 --warmup 5 \
    --no-cpu-baseline --no-probe-peak --workload c2 > "gpurun_out/dl_sweep/$G-$A-$Q-$D.json" 2> "gpurun_out/dl_sweep/$G-$A-$Q-$D.err" \
    || { tail -5 "gpurun_out/dl_sweep/$G-$A-$Q-$D.err"; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['value'])" "gpurun_out/dl_sweep/$G-$A-$Q-$D.json"
done
