#!/usr/bin/env python3
"""Run one configuration level by level on the GPU and print TLC-style progress per level.

usage: explore.py N V E R [--budget SECONDS] [--levels L] [--seeded] [--chunk G] [--seenlog2 K] [--rccl1 [--shard-min K]]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-raft_amd"))
import raftmc  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("n", type=int)
ap.add_argument("V", type=int)
ap.add_argument("E", type=int)
ap.add_argument("R", type=int)
ap.add_argument("--budget", type=float, default=120)
ap.add_argument("--levels", type=int, default=0, help="stop after expanding this many levels (0: no limit)")
ap.add_argument("--seeded", action="store_true")
ap.add_argument("--chunk", type=int, default=0)
ap.add_argument("--seenlog2", type=int, default=0)
ap.add_argument("--json", default="")
ap.add_argument("--compact-log2", type=int, default=0)
ap.add_argument("--seen-mem-gb", type=float, default=0)
ap.add_argument("--frontier-mem-gb", type=float, default=0)
ap.add_argument("--rccl1", action="store_true", help="the sharded protocol on a one-rank RCCL communicator")
ap.add_argument("--shard-min", type=int, default=0)
ap.add_argument("--us", action="store_true", help="phase kernel times in microseconds")
a = ap.parse_args()
extra = dict(world_size=1, rank=0, comm_unique_id=raftmc.comm_unique_id()) if a.rccl1 else {}
cfg = raftmc.ModelConfig(n_servers=a.n, n_vals=a.V, max_election=a.E, max_restart=a.R,
                         spec_variant=raftmc.SPEC_SEEDED if a.seeded else raftmc.SPEC_RAFT,
                         chunk_successors=a.chunk, seen_log2=a.seenlog2, compact_log2=a.compact_log2,
                         seen_mem_bytes=int(a.seen_mem_gb * 2**30), frontier_mem_bytes=int(a.frontier_mem_gb * 2**30),
                         shard_min_states=a.shard_min, **extra)
t0 = time.time()
mc = raftmc.ModelChecker(cfg)
print(f"create {time.time() - t0:.2f}s", flush=True)
ls = mc.init()
t1 = time.time()
rows = []
stopped = ""
while ls.status == "ok" and time.time() - t1 < a.budget and not (a.levels and ls.level >= a.levels):
    try:
        ls = mc.step()
    except raftmc.RmcError as e:  # capacity: report how far one GPU got
        stopped = str(e)
        print(f"STOPPED at level {ls.level + 1}: {e}", flush=True)
        break
    el = time.time() - t1
    ms = " ".join(f"{x * 1e3:.0f}" if a.us else f"{x:.1f}" for x in ls.kernel_ms)
    print(f"L{ls.level:3d} F={ls.expanded:>11d} G={ls.generated:>12d} N={ls.new_states:>11d} "
          f"tot={ls.total_distinct:>12d} {ls.seconds * 1e3:9.1f}ms [{ms}] el={el:.1f}s "
          f"{ls.total_distinct / el:.3e} ds/s rec={ls.new_bytes / max(1, ls.new_states):.1f}B self={ls.self_loops}",
          flush=True)
    rows.append(ls.__dict__)
if stopped:
    sys.exit(0)
r = mc.result()
print("RESULT", r.status, "generated", r.generated, "distinct", r.distinct, "depth", r.depth,
      "seconds", round(r.seconds, 3), "seen_slots", r.seen_slots, "x", r.seen_slot_bytes, "B; ring",
      r.frontier_ring_bytes, "B; frontier peak", r.frontier_peak_bytes, "B", flush=True)
if a.json:
    with open(a.json, "w") as f:
        json.dump(dict(result=r.__dict__ | {"levels": None}, levels=rows), f)
