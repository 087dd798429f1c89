#!/bin/bash
# A/B of kernel build variants on the bench workload (configs[1]), one box: the phase profile of the
# expansion and commit on configs[1], then bench.py's ms per exhaustion per variant (no CPU baseline,
# no at-scale leg).
# usage: tools/gpu_ab_c2.sh OUTDIR variant [variant ...]   (variant "default" = tla-raft_amd/build)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=gpurun_out/$1
shift
mkdir -p "$O"
if [ -f tla-raft_amd/build_prof/librmc.so ]; then
  echo "== phase profile ($(date +%T))"
  RMC_LIBRARY=tla-raft_amd/build_prof/librmc.so timeout -k 10 120 python -u tools/phase_prof.py 3 1 2 3 > "$O/phase_c2.txt" 2>&1 || { tail -5 "$O/phase_c2.txt"; exit 1; }
  cat "$O/phase_c2.txt"
fi
for rep in 1 2; do
  for v in "$@"; do
    lib=tla-raft_amd/build_$v/librmc.so
    [ "$v" = default ] && lib=tla-raft_amd/build/librmc.so
    RMC_LIBRARY=$lib timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-probe-peak --no-scale > "$O/bench_${v}_$rep.json" 2> "$O/bench_${v}_$rep.err" || { tail -5 "$O/bench_${v}_$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['value'])" "$O/bench_${v}_$rep.json" "$v"
  done
done
echo "== done ($(date +%T))"
