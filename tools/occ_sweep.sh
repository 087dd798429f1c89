#!/bin/bash
# Occupancy sweep at scale: Raft.cfg (n3 V2 E3 R3) exhausted once per library build dir given as
# an argument (tools/build_variant.sh n3w<W>c<C>g<G>; "build" = the default), each under its own
# time limit; prints the last level line (total time) per build.  Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
mkdir -p gpurun_out/occ
for D in "$@"; do
  echo "== $D ($(date +%T))"
  RMC_LIBRARY="$R/tla-raft_amd/$D/librmc.so" timeout -k 10 240 python -u tools/explore.py ${CFG:-3 2 3 3} --budget 200 \
    > "gpurun_out/occ/$D.log" 2>&1 || { tail -5 "gpurun_out/occ/$D.log"; exit 1; }
  tail -n 3 "gpurun_out/occ/$D.log"
done
