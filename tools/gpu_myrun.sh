#!/bin/bash
# The drop-in (tla-raft_amd/myrun.sh) on the user's Raft.tla / Raft.cfg copied into scratch_myrun/ for
# this call (never committed), with the launcher's phase times and the shell's wall time.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R/scratch_myrun" || exit 1
mkdir -p ../gpurun_out
sha256sum Raft.tla Raft.cfg > ../gpurun_out/myrun_inputs.sha256
export RMC_LAUNCHER_TIMES=1
s=$(date +%s%N)
timeout -k 10 200 bash ../tla-raft_amd/myrun.sh > /dev/null 2>&1 || exit 1
e=$(date +%s%N)
cp raft.log ../gpurun_out/myrun_raft.log
echo "myrun.sh wall $(( (e - s) / 1000000 )) ms" | tee -a ../gpurun_out/myrun_raft.log
grep "raftmc:\|Finished" ../gpurun_out/myrun_raft.log
