#!/bin/bash
# PMC passes over one at-scale run (tools/explore.py $CFG, default 3 servers / 2 values / MaxElection 2:
# 18.5M states, levels of up to ~10^6 states; CFG="3 2 3 3 --levels 44" takes Raft.cfg's first 44
# expansions, 7.5 G states): where the expansion, probe and commit kernels spend cycles (tools/pmc_scale_report.py).
# OUT (default gpurun_out/pmcs) is the output directory.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
OUT=${OUT:-gpurun_out/pmcs}
CFG=${CFG:-3 2 2 3}
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {
  name=$1; shift
  echo "== pmc $name ($(date +%T))"
  timeout -s KILL ${LIMIT:-120} rocprofv3 --pmc "$@" --output-format csv -d "$R/$OUT/$name" -o run -- python3 "$R/tools/explore.py" $CFG > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; tail -5 "$OUT/$name.log"; return 1; }
}
pass sqa SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU && \
pass sqb SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH && \
pass fetch FETCH_SIZE && pass write WRITE_SIZE && pass tcc TCC_HIT_sum TCC_MISS_sum && \
python tools/pmc_summary.py "$OUT" "$OUT.json"
