#!/bin/bash
# Round-4 A/B of kernel build variants on Raft.cfg (tools/build_variant.sh), one box, each run under
# its own time limit: the phase profile of the expansion, then full exhaustions per variant.
# usage: tools/gpu_ab_r04.sh OUTDIR variant [variant ...]   (variant "default" = tla-raft_amd/build)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=gpurun_out/$1
shift
mkdir -p "$O"
if [ -f tla-raft_amd/build_prof/librmc.so ]; then
  echo "== phase profile ($(date +%T))"
  RMC_LIBRARY=tla-raft_amd/build_prof/librmc.so timeout -k 10 240 python -u tools/phase_prof.py 3 2 3 3 --levels 40 > "$O/phase.txt" 2>&1 || { tail -5 "$O/phase.txt"; exit 1; }
  cat "$O/phase.txt"
fi
for v in "$@"; do
  lib=tla-raft_amd/build_$v/librmc.so
  [ "$v" = default ] && lib=tla-raft_amd/build/librmc.so
  echo "== $v ($(date +%T))"
  RMC_LIBRARY=$lib timeout -k 10 200 python -u tools/explore.py 3 2 3 3 --budget 150 > "$O/raftcfg_$v.log" 2>&1 || { tail -5 "$O/raftcfg_$v.log"; exit 1; }
  grep RESULT "$O/raftcfg_$v.log"
done
echo "== done ($(date +%T))"
