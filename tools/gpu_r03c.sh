#!/bin/bash
# Round-3 configs[3] record on one GPU box (each step under its own limit, stop at the first failure):
# configs[3] level by level with the memory split set for it (48 GB seen set, 200 GB ring, 2^27-slot
# chunks) and with the defaults, then bench.py's two sharded legs through a one-rank RCCL
# communicator (tools/sharded_legs_check.py), and where a large run's teardown goes
# (tools/teardown_probe.cpp, built into tools/build/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
O=gpurun_out/c4
mkdir -p $O
export TMPDIR=/tmp
echo "== c4 split ($(date +%T))"
timeout -k 10 300 python -u tools/explore.py 5 1 3 3 --seen-mem-gb 48 --frontier-mem-gb 200 --chunk 134217728 --budget 250 > $O/c4_split.log 2>&1 || { tail -5 $O/c4_split.log; exit 1; }
tail -2 $O/c4_split.log
echo "== c4 default ($(date +%T))"
timeout -k 10 300 python -u tools/explore.py 5 1 3 3 --budget 250 > $O/c4_default.log 2>&1 || { tail -5 $O/c4_default.log; exit 1; }
tail -2 $O/c4_default.log
echo "== sharded legs, one-rank RCCL ($(date +%T))"
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29650 timeout -k 10 600 python -u tools/sharded_legs_check.py $O/sharded_legs_rccl1.json > $O/sharded_legs.log 2>&1 || { tail -20 $O/sharded_legs.log; exit 1; }
cut -c1-600 $O/sharded_legs_rccl1.json
echo "== teardown probe ($(date +%T))"
for m in pinned pinned-exit thp thp-exit pageable pageable-exit device device-exit; do
  case $m in device*) gb=240;; *) gb=64;; esac
  t0=$(date +%s%N)
  timeout -k 10 200 tools/build/teardown_probe $m $gb >> $O/teardown.txt 2>&1 || { cat $O/teardown.txt; exit 1; }
  echo "$m $gb GB: process wall $(( ($(date +%s%N) - t0) / 1000000 )) ms" >> $O/teardown.txt
done
cat $O/teardown.txt
echo "== done ($(date +%T))"
