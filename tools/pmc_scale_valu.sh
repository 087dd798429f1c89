#!/bin/bash
# VALU-issue fraction of the expansion at scale: one kernel-trace pass (durations) and one SQ pass
# (SQ_INSTS_VALU per dispatch) over the same exploration (tools/explore.py $CFG, default 3 servers /
# 2 values / MaxElection 2: 18.5 M states, levels of up to ~10^6 parents).  Separate passes, each
# under its own limit.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
mkdir -p gpurun_out/valu
export TMPDIR=/tmp
CFG=${CFG:-3 2 2 3}
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/valu/kt" -o run -- python3 "$R/tools/explore.py" $CFG > gpurun_out/valu/kt.log 2>&1 || { echo "trace pass failed"; tail -5 gpurun_out/valu/kt.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d "$R/gpurun_out/valu/sq" -o run -- python3 "$R/tools/explore.py" $CFG > gpurun_out/valu/sq.log 2>&1 || { echo "sq pass failed"; tail -5 gpurun_out/valu/sq.log; exit 1; }
find gpurun_out/valu -name "*.csv" | sort
