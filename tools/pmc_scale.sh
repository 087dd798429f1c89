#!/bin/bash
# PMC passes over one at-scale exhaustion (tools/explore.py, 3 servers / 2 values / MaxElection 2:
# 18.5M states, levels of up to ~10^6 states): where the expansion and commit kernels spend cycles.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
mkdir -p gpurun_out/pmcs
export TMPDIR=/tmp
pass() {
  name=$1; shift
  echo "== pmc $name ($(date +%T))"
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/pmcs/$name" -o run -- python3 "$R/tools/explore.py" 3 2 2 3 > "gpurun_out/pmcs/$name.log" 2>&1 || { echo "pass $name failed"; tail -5 "gpurun_out/pmcs/$name.log"; return 1; }
}
pass sqa SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU && \
pass sqb SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH && \
pass fetch FETCH_SIZE && pass write WRITE_SIZE && pass tcc TCC_HIT_sum TCC_MISS_sum && \
python tools/pmc_summary.py gpurun_out/pmcs gpurun_out/pmc_scale.json
