"""Order-sensitivity probe fixtures from the C oracle.

The VIEW (Raft.tla:38) hides restartCount / valSent / pendingResponse / electionCount
(Raft.tla:34-36), so which concrete state represents a fingerprint class -- the first one TLC
discovers -- could in principle change what is reachable later.  For each configuration the
oracle explores the state space three times: in TLC -workers 1 order (order 0), with every
level's parents visited in reverse and each parent's successors reversed (order 1), and with a
seeded shuffle of every level (order 2).  Identical per-level distinct/generated counts in all
three say the configuration's partition does not depend on discovery order -- the assumption
behind any multi-worker or multi-GPU order.

usage: python tests/golden/make_order_probe.py n V E R [seeded] ...   (writes order_probe.json)
"""
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import c_oracle  # noqa: E402


def run(n, V, E, Rr, seeded, order):
    lib = c_oracle()
    lib.orc_set_order.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64]
    h = lib.orc_create(n, V, E, Rr, int(seeded), 0, 1, 0)
    lib.orc_set_order(h, order, 12345)
    v = lib.orc_run(h, 0)
    cap = 256
    d = (ctypes.c_uint64 * cap)()
    g = (ctypes.c_uint64 * cap)()
    depth = lib.orc_levels(h, d, g, cap)
    out = {"verdict": int(v), "distinct": lib.orc_distinct(h), "generated": lib.orc_generated(h), "depth": depth,
           "levels": list(d[:depth]), "gen_per_level": list(g[:depth])}
    lib.orc_destroy(h)
    return out


def same(a, b):
    """Same partition: identical per-level counts; a run stopped by an invariant violation is compared on
    the levels it completed, plus the depth of the violation (the counterexample's length)."""
    if a["verdict"] != b["verdict"] or a["depth"] != b["depth"]:
        return False
    if a["verdict"] == 0:
        return a["levels"] == b["levels"] and a["gen_per_level"] == b["gen_per_level"]
    k = a["depth"] - 1
    return a["levels"][:k] == b["levels"][:k] and a["gen_per_level"][:k - 1] == b["gen_per_level"][:k - 1]


def main():
    a = sys.argv[1:]
    cfgs = []
    i = 0
    while i < len(a):
        n, V, E, Rr = map(int, a[i:i + 4])
        i += 4
        seeded = i < len(a) and a[i] == "seeded"
        if seeded:
            i += 1
        cfgs.append((n, V, E, Rr, seeded))
    path = os.environ.get("ORDER_PROBE_OUT", os.path.join(HERE, "order_probe.json"))
    for (n, V, E, Rr, seeded) in cfgs:
        t = time.time()
        runs = {str(o): run(n, V, E, Rr, seeded, o) for o in (0, 1, 2)}
        key = f"{'seeded_' if seeded else ''}n{n}_v{V}_e{E}_r{Rr}"
        rec = {"n": n, "V": V, "E": E, "R": Rr, "seeded": seeded, "orders": runs,
               "order_insensitive": all(same(runs[o], runs["0"]) for o in runs),
               "oracle_seconds": round(time.time() - t, 1)}
        out = json.load(open(path)) if os.path.exists(path) else {}
        out[key] = rec
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        print(key, "insensitive" if rec["order_insensitive"] else "ORDER-SENSITIVE", rec["oracle_seconds"], "s",
              flush=True)


if __name__ == "__main__":
    main()
