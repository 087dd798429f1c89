#!/usr/bin/env python3
"""Time the sharded path (block-cyclic levels, fingerprint-owner election) run as
virtual shards on one GPU -- every shard's work in one process, device copies as the transport -- against
the single-GPU path.  The shards run one after another, so the extra time over one GPU is the sharding
overhead (routing, owner election, record exchange, host round trips per round), not a speed-up.

usage: shard_timing.py [n V E R] [--shard-min K] [--reps R] [--shards 1,2,4,8] [--rccl1]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-raft_amd"))
import raftmc  # noqa: E402

PH = ["count", "expand", "wincount", "commit", "exchange", "other"]


def timed(cfg, reps):
    with raftmc.ModelChecker(cfg) as mc:
        mc.run()
        t0 = time.perf_counter()
        for _ in range(reps):
            mc.reset()
            res = mc.run()
        dt = (time.perf_counter() - t0) / reps
        ms = [0.0] * 6
        for ls in res.levels:
            for i in range(6):
                ms[i] += ls.kernel_ms[i]
        return res, dt, ms


ap = argparse.ArgumentParser()
ap.add_argument("cfg", nargs="*", type=int, default=[3, 1, 2, 3])
ap.add_argument("--shard-min", type=int, default=1)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--shards", default="1,2,4,8", help="virtual shard counts (1 = the single-GPU path)")
ap.add_argument("--rccl1", action="store_true", help="also the sharded protocol on a one-rank RCCL communicator "
                "(world_size 1 + unique id): its own collectives, self send/recv")
a = ap.parse_args()
n, V, E, R = a.cfg
base = None
runs = [(int(x), False) for x in a.shards.split(",")] + ([(1, True)] if a.rccl1 else [])
for vs, rccl in runs:
    extra = dict(world_size=1, rank=0, comm_unique_id=raftmc.comm_unique_id()) if rccl else {}
    cfg = raftmc.ModelConfig(n_servers=n, n_vals=V, max_election=E, max_restart=R, device=0,
                             virtual_shards=vs if vs > 1 else 0, shard_min_states=a.shard_min, timing_phases=0x3F,
                             **extra)
    res, dt, ms = timed(cfg, a.reps)
    base = base or dt
    tot = sum(ms) or 1.0
    print(f"{'rccl-1' if rccl else 'shards=' + str(vs)}: {res.distinct} distinct, depth {res.depth}, {dt * 1e3:.2f} ms/exhaustion "
          f"({dt / base:.2f}x one GPU), kernel ms " + ", ".join(f"{PH[i]} {ms[i]:.1f}" for i in range(6) if ms[i]) +
          f"; exchange {100 * ms[4] / tot:.0f} % of kernel time", flush=True)
