#!/usr/bin/env python3
"""Step a small configuration level by level at W virtual shards, printing each level (debug aid).
usage: dbg_shard.py N V E R W [shard_min] [chunk_successors] [seeded]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-raft_amd"))
import raftmc  # noqa: E402

a = sys.argv[1:]
n, V, E, R, W = map(int, a[:5])
smin = int(a[5]) if len(a) > 5 else 1
chunk = int(a[6]) if len(a) > 6 else 3000
seeded = len(a) > 7 and a[7] == "seeded"
cfg = raftmc.ModelConfig(n_servers=n, n_vals=V, max_election=E, max_restart=R, virtual_shards=W,
                         shard_min_states=smin, chunk_successors=chunk,
                         spec_variant=raftmc.SPEC_SEEDED if seeded else raftmc.SPEC_RAFT)
mc = raftmc.ModelChecker(cfg)
print("created", flush=True)
ls = mc.init()
print(ls, flush=True)
while ls.status == "ok":
    ls = mc.step()
    print(ls.level, ls.status, ls.expanded, ls.generated, ls.new_states, ls.total_distinct, ls.queue, flush=True)
r = mc.result()
print("RESULT", r.status, r.distinct, r.generated, r.depth, r.queue, flush=True)
