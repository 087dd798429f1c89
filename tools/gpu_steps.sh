#!/bin/bash
# GPU session steps on one box, each under its own time limit, stopping at the first
# failure.  usage: tools/gpu_steps.sh OUTDIR step [step ...]
#   tests        pytest -m gpu (whole suite)        tests:K  pytest -m gpu -k K
#   raftcfg      Raft.cfg exhausted level by level (tools/explore.py)
#   prof_raftcfg rocprofv3 kernel stats of the same
#   bench        bench.py default line (Raft.cfg, 10 steps)   benchd  the driver's line (--steps 20 --warmup 5)
#   prof_bench   rocprofv3 kernel stats of bench's headline (Raft.cfg, 2 timed steps)
#   prof_c2      rocprofv3 kernel stats of bench --workload c2 (configs[1])
#   pmc_bench    tools/pmc.sh over bench's headline (one Raft.cfg exhaustion per pass) + pmc_summary.py
#   pmc_c2       ... over bench.py --workload c2 (configs[1])
#   c4           configs[3] as deep as one GPU goes  rccl1       Raft.cfg through a one-rank RCCL communicator
#   prof_rccl1   rocprofv3 kernel stats of the rccl1 run
#   c4split      configs[3] on one GPU with the 48 GB seen set / 200 GB ring split
#   n4e3         4 servers, 1 value, MaxElection 3 as deep as one GPU goes (DESIGN.md section 9's E2->E3 factor)
#   pmc_raftcfg  PMC passes over Raft.cfg's first 40 expansions + tools/pmc_scale_report.py
#   myrun        tools/gpu_myrun.sh (the drop-in on scratch_myrun/)   smoke  __graft_entry__.smoke()
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=gpurun_out/$1
shift
mkdir -p "$O"
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
for s in "$@"; do
  step "$s"
  case "$s" in
    tests) timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
           tail -2 "$O/tests.log" ;;
    tests:*) k=${s#tests:}; timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -k "$k" > "$O/tests_$k.log" 2>&1 || { tail -30 "$O/tests_$k.log"; exit 1; }
           tail -2 "$O/tests_$k.log" ;;
    raftcfg) timeout -k 10 300 python -u tools/explore.py 3 2 3 3 --budget 200 > "$O/raftcfg.log" 2>&1 || { tail -20 "$O/raftcfg.log"; exit 1; }
           tail -4 "$O/raftcfg.log" ;;
    prof_raftcfg) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_raftcfg" -o run -- python3 "$R/tools/explore.py" 3 2 3 3 --budget 200 > "$O/prof_raftcfg.log" 2>&1 || { tail -20 "$O/prof_raftcfg.log"; exit 1; }
           grep RESULT "$O/prof_raftcfg.log"; find "$O/prof_raftcfg" -name '*kernel_stats.csv' -exec head -12 {} \; ;;
    bench) timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail "$O/bench.err"; exit 1; }
           cut -c1-600 "$O/bench.json" ;;
    benchd) timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > "$O/benchd.json" 2> "$O/benchd.err" || { tail "$O/benchd.err"; exit 1; }
           cut -c1-600 "$O/benchd.json" ;;
    prof_bench) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_bench" -o bench -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-configs1 --no-cpu-baseline --no-probe-peak > "$O/prof_bench.log" 2>&1 || { tail -20 "$O/prof_bench.log"; exit 1; }
           tail -c 700 "$O/prof_bench.log"; find "$O/prof_bench" -name '*kernel_stats.csv' -exec head -12 {} \; ;;
    c2) timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 5 --no-cpu-baseline --no-probe-peak > "$O/c2.json" 2> "$O/c2.err" || { tail "$O/c2.err"; exit 1; }
           cut -c1-400 "$O/c2.json" ;;
    prof_c2) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_c2" -o bench -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-probe-peak --workload c2 > "$O/prof_c2.log" 2>&1 || { tail -20 "$O/prof_c2.log"; exit 1; }
           find "$O/prof_c2" -name '*kernel_stats.csv' -exec head -12 {} \; ;;
    pmc_bench) rm -rf gpurun_out/pmc; WORKLOAD=raftcfg bash tools/pmc.sh || exit 1
           python tools/pmc_summary.py gpurun_out/pmc "$O/pmc_headline_raftcfg.json" && rm -rf gpurun_out/pmc ;;
    pmc_c2) rm -rf gpurun_out/pmc; WORKLOAD=c2 bash tools/pmc.sh || exit 1
           python tools/pmc_summary.py gpurun_out/pmc "$O/pmc_c2.json" && rm -rf gpurun_out/pmc ;;
    c4) timeout -k 10 300 python -u tools/explore.py 5 1 3 3 --budget 150 > "$O/c4.log" 2>&1 || { tail -20 "$O/c4.log"; exit 1; }
           tail -4 "$O/c4.log" ;;
    c4split) timeout -k 10 300 python -u tools/explore.py 5 1 3 3 --seen-mem-gb 48 --frontier-mem-gb 200 --budget 200 > "$O/c4split.log" 2>&1 || { tail -20 "$O/c4split.log"; exit 1; }
           tail -4 "$O/c4split.log" ;;
    n4e3) timeout -k 10 420 python -u tools/explore.py 4 1 3 3 --budget 360 > "$O/n4e3.log" 2>&1 || { tail -20 "$O/n4e3.log"; exit 1; }
           tail -4 "$O/n4e3.log" ;;
    n4e3split) timeout -k 10 420 python -u tools/explore.py 4 1 3 3 --seen-mem-gb ${SEEN_GB:-120} --frontier-mem-gb ${RING_GB:-140} --budget 360 > "$O/n4e3split.log" 2>&1 || { tail -20 "$O/n4e3split.log"; exit 1; }
           tail -4 "$O/n4e3split.log" ;;
    prof_rccl1) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_rccl1" -o run -- python3 "$R/tools/explore.py" 3 2 3 3 --rccl1 --budget 200 > "$O/prof_rccl1.log" 2>&1 || { tail -20 "$O/prof_rccl1.log"; exit 1; }
           grep RESULT "$O/prof_rccl1.log"; find "$O/prof_rccl1" -name '*kernel_stats.csv' -exec head -24 {} \; ;;
    rccl1) timeout -k 10 300 python -u tools/explore.py 3 2 3 3 --rccl1 --budget 200 > "$O/rccl1.log" 2>&1 || { tail -5 "$O/rccl1.log"; exit 1; }
           tail -4 "$O/rccl1.log" ;;
    pmc_raftcfg) OUT=$O/pmc_raftcfg CFG="3 2 3 3 --levels 40" LIMIT=150 bash tools/pmc_scale.sh || exit 1
           python tools/pmc_scale_report.py "$O/pmc_raftcfg" "$O/pmc_scale_raftcfg_levels.json" --workload "Raft.cfg, first 40 expansions" ;;
    myrun) bash tools/gpu_myrun.sh || exit 1 ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { cat "$O/smoke.log"; exit 1; }
           tail -1 "$O/smoke.log" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
