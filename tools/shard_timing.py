#!/usr/bin/env python3
"""Time the sharded (fingerprint-owner) path with virtual shards on one GPU against the fused
single-GPU path, on BASELINE configs[1]: where the per-level exchange cost goes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-raft_amd"))
import raftmc  # noqa: E402


def timed(cfg, reps=5):
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


for vs in [1, 2, 4, 8]:
    cfg = raftmc.ModelConfig(n_servers=3, n_vals=1, max_election=2, max_restart=3, device=0,
                             virtual_shards=vs if vs > 1 else 0, timing_phases=0x3F)
    res, dt, ms = timed(cfg)
    print(f"shards={vs}: {res.distinct} distinct, depth {res.depth}, {dt * 1e3:.2f} ms/exhaustion, "
          f"{res.distinct / dt / 1e6:.1f} M states/s; phase ms {[round(x, 2) for x in ms]}", flush=True)
