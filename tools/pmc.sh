#!/bin/bash
# PMC passes over bench.py (one counter group per run, MI355X_MICROARCH.md rocprofv3 section).
#   WORKLOAD=raftcfg (default): one Raft.cfg exhaustion per pass (the headline's split kernels)
#   WORKLOAD=c2: bench.py --workload c2 --steps 5 --warmup 1 per pass (bench.py PMC_RUNS = 6 exhaustions)
# then tools/pmc_summary.py gpurun_out/pmc profiles/rNN_pmc_$WORKLOAD.json
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
WORKLOAD=${WORKLOAD:-raftcfg}
if [ "$WORKLOAD" = c2 ]; then
  ARGS="--workload c2 --steps 5 --warmup 1 --no-cpu-baseline --no-probe-peak"
else
  ARGS="--workload $WORKLOAD --steps 1 --warmup 0 --no-configs1 --no-cpu-baseline --no-probe-peak"
fi
pass() {
  name=$1; shift
  echo "== pmc $name ($(date +%T))"
  timeout -s KILL ${LIMIT:-150} rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/pmc/$name" -o run -- python3 "$R/bench.py" $ARGS > "gpurun_out/pmc/$name.log" 2>&1 || { echo "pass $name failed"; tail -5 "gpurun_out/pmc/$name.log"; return 1; }
}
pass fetch FETCH_SIZE && pass write WRITE_SIZE && pass sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR && pass tcc TCC_HIT_sum TCC_MISS_sum
