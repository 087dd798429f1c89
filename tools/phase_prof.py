#!/usr/bin/env python3
"""Where k_expand's time goes, phase by phase (shader clock summed over waves).

Needs a library built with -DRMC_PHASE_PROF (tools/build_variant.sh prof), selected with
RMC_LIBRARY=.../librmc.so.  Runs one configuration for --levels BFS levels (or to the end) and
prints each phase's share of the waves' time in k_expand:
  0 load parent record (+ message hash rows)   1 evaluate actions (one candidate per lane)
  2 TLC-order ranks, error keys               3 staging of the successor rows (fused level)
  4 parent content matrix, successor row inputs, acting-row contents; a split chunk's hash context
  5 signatures, coset ranks and sizes    6 hash tasks (coset minimum)
  7 seen-set probe + election (fused levels)

usage: RMC_LIBRARY=tla-raft_amd/build_prof/librmc.so python tools/phase_prof.py N V E R [--levels L]"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-raft_amd"))
import raftmc  # noqa: E402

NAMES = ["load parent", "evaluate actions", "ranks + error keys", "staging", "hash inputs, acting-row contents (split: hash context)",
         "signatures, coset ranks", "hash tasks (coset minimum)", "seen-set probe + election (fused)",
         # k_commit (slots 8-15)
         "commit: header wait (+ parents w/o winners)", "commit: record + election words + staged rows",
         "commit: winner test", "-", "commit: rebuild, encode, seen insert, trace, invariants",
         "commit: scan + record writes", "-", "-"]

ap = argparse.ArgumentParser()
ap.add_argument("n", type=int)
ap.add_argument("V", type=int)
ap.add_argument("E", type=int)
ap.add_argument("R", type=int)
ap.add_argument("--levels", type=int, default=1000)
ap.add_argument("--device-levels", type=int, default=0)
ap.add_argument("--items", action="store_true", help="split chunks expand with k_expand_items: its phases in slots 0-6")
a = ap.parse_args()
if a.items:
    NAMES[:8] = ["items: record offsets + copy into LDS", "items: decode cores, message scan",
                 "items: message pass (hash sums, votes, classes)", "items: hash context write, item scan",
                 "items: evaluate (action, key list)", "items: ranks + staging",
                 "items: per-parent counts, error keys, round sync", "items: class lists (+ round start)"]
cfg = raftmc.ModelConfig(n_servers=a.n, n_vals=a.V, max_election=a.E, max_restart=a.R, device_levels=a.device_levels)
mc = raftmc.ModelChecker(cfg)
lib = raftmc.load_library()
if not hasattr(lib, "rmc_debug_phases"):
    sys.exit("this librmc.so was not built with -DRMC_PHASE_PROF")
buf = (ctypes.c_ulonglong * 16)()
lib.rmc_debug_phases(buf, 1)
ls = mc.init()
t = time.time()
lv = 0
while ls.status == "ok" and lv < a.levels:
    ls = mc.step()
    lv += 1
el = time.time() - t
lib.rmc_debug_phases(buf, 0)
res = mc.result()
print(f"config n{a.n}_v{a.V}_e{a.E}_r{a.R}: {lv} levels, {res.distinct} distinct, {el:.2f} s")
for lo, what in ((0, "k_expand"), (8, "k_commit")):
    tot = sum(buf[lo:lo + 8]) or 1
    print(f" {what}: share of its waves' time")
    for i in range(lo, lo + 8):
        if buf[i]:
            print(f"  {i} {NAMES[i]:46s} {100.0 * buf[i] / tot:6.2f} %  ({buf[i] / 1e9:.2f} G wave-clocks)")
