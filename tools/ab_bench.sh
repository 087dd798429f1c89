#!/bin/bash
# A/B of library builds on bench.py's headline (warm Raft.cfg exhaustions), one process per run, in the
# order given (repeat a name to interleave): usage tools/ab_bench.sh OUTDIR name=path/to/librmc.so ...
# ("name=" alone: the default build; "name=lib|--chunk-successors 67108864": extra bench.py arguments).  Each run: 1 warmup + 2 timed exhaustions; prints ms_per_step and the
# split expansion's average launch.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=gpurun_out/$1
shift
mkdir -p "$O"
i=0
for spec in "$@"; do
  name=${spec%%=*}; lib=${spec#*=}; extra=""
  case "$lib" in *"|"*) extra=${lib#*|}; lib=${lib%%|*} ;; esac  # name=lib|--bench-args
  i=$((i + 1))
  ( [ -n "$lib" ] && export RMC_LIBRARY="$lib"
    timeout -k 10 200 python -u bench.py --steps ${STEPS:-2} --warmup 1 --no-configs1 --no-cpu-baseline --no-probe-peak $extra ) \
    > "$O/$i.$name.json" 2> "$O/$i.$name.err" || { echo "run $i $name failed"; tail -n 5 "$O/$i.$name.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read()); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],1), 'ms/step; expand avg', r['avg_launch_ms'], 'ms x', r['launches'])" "$O/$i.$name.json" "$name"
done
