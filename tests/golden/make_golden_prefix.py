"""Prefix golden levels from the C oracle (oracle/raft_oracle.c, TLC -workers 1 BFS).

For configurations whose full state space the single-threaded oracle cannot exhaust in
reasonable time (Raft.cfg as shipped: n3 V2 E3 R3; the 5-server config n5 V1 E3 R3), run the
oracle until `max_states` distinct states and keep only the levels it completed:

  levels[k]        distinct states at BFS level k+1, for every level fully discovered
  gen_per_level[k] successors generated while expanding level k+1, for every level fully
                   expanded (one fewer than `levels`)

The GPU test (tests/test_gpu.py::test_prefix_levels_match_c_oracle) runs the same configuration
level by level and compares those prefixes exactly.

usage: python tests/golden/make_golden_prefix.py [--mt THREADS | --lean THREADS SEEN_SLOTS] MAX_STATES n V E R [...]
writes tests/golden/levels_prefix.json (merged with what is there)

--mt runs oracle/raft_mt.c's level-synchronous BFS (the same restatement, same first-wins
semantics) on THREADS host threads and stops at the first level boundary past MAX_STATES, so
every reported level is complete (used for the 5-server configs[3], whose exact canonical form
costs 120 permutations per successor).

--lean runs oracle/raft_prefix.c (same semantics, packed records, seen set of SEEN_SLOTS 16-B slots
sized once, winners regenerated instead of stored) for Raft.cfg's deep prefix: 35 levels, 984 M
states, in ~55 GB; it must reproduce the levels already recorded, and adds max |msgs| per level.
"""
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import c_oracle  # noqa: E402

V_LIMIT_NAMES = {0: "ok", 1: "invariant", 2: "assert", 3: "eval_error", 4: "deadlock"}


def run_prefix(n, V, E, Rr, max_states):
    lib = c_oracle()
    h = lib.orc_create(n, V, E, Rr, 0, 0, 1, 0)
    t = time.time()
    v = lib.orc_run(h, max_states)
    dt = time.time() - t
    cap = 256
    d = (ctypes.c_uint64 * cap)()
    g = (ctypes.c_uint64 * cap)()
    depth = lib.orc_levels(h, d, g, cap)
    distinct = lib.orc_distinct(h)
    max_nm = lib.orc_max_msgs(h)
    lib.orc_destroy(h)
    if v == 0:  # exhausted: every level is complete
        levels, gens = list(d[:depth]), list(g[:depth])
    else:
        # stopped while expanding level `depth - 1` (its successors land in level `depth`):
        # levels 1..depth-1 are fully discovered, levels 1..depth-2 fully expanded
        levels, gens = list(d[:depth - 1]), list(g[:depth - 2])
    return {"n": n, "V": V, "E": E, "R": Rr, "max_states": max_states, "stopped_at_distinct": distinct,
            "exhausted": v == 0, "levels": levels, "gen_per_level": gens, "max_msgs_seen": max_nm,
            "oracle_seconds": round(dt, 1), "source": "c", "invariants": ["Inv"], "check_deadlock": False}


def run_prefix_mt(n, V, E, Rr, max_states, threads):
    lib = ctypes.CDLL(os.path.join(HERE, "..", "..", "oracle", "build", "libraft_mt.so"))
    lib.orc_mt_levels.argtypes = [ctypes.c_int] * 5 + [ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                                       ctypes.POINTER(ctypes.c_uint64), ctypes.c_int,
                                                       ctypes.POINTER(ctypes.c_uint64),
                                                       ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int)]
    cap = 256
    d = (ctypes.c_uint64 * cap)()
    g = (ctypes.c_uint64 * cap)()
    dist, gen, depth = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
    t = time.time()
    v = lib.orc_mt_levels(n, V, E, Rr, threads, max_states, d, g, cap, ctypes.byref(dist), ctypes.byref(gen),
                          ctypes.byref(depth))
    dt = time.time() - t
    D = depth.value
    assert v in (0, 2), f"unexpected verdict {v}"
    # levels 1..D all complete; levels 1..D-1 expanded (level D too when the run exhausted)
    levels, gens = list(d[:D]), list(g[:D if v == 0 else D - 1])
    return {"n": n, "V": V, "E": E, "R": Rr, "max_states": max_states, "stopped_at_distinct": dist.value,
            "exhausted": v == 0, "levels": levels, "gen_per_level": gens, "oracle_seconds": round(dt, 1),
            "source": f"c_mt{threads}", "invariants": ["Inv"], "check_deadlock": False}


def run_prefix_lean(n, V, E, Rr, max_states, threads, seen_slots):
    """oracle/raft_prefix.c: the same level-synchronous first-wins BFS with packed records, a seen set
    sized once (seen_slots x 16 B) and no stored candidates, for prefixes of ~10^9 states in the
    build container's memory.  Also records each level's largest |msgs|."""
    lib = ctypes.CDLL(os.path.join(HERE, "..", "..", "oracle", "build", "libraft_prefix.so"))
    P64 = ctypes.POINTER(ctypes.c_uint64)
    lib.orc_prefix_levels.argtypes = [ctypes.c_int] * 5 + [ctypes.c_uint64, ctypes.c_uint64, P64, P64,
                                                           ctypes.POINTER(ctypes.c_int), ctypes.c_int, P64, P64,
                                                           ctypes.POINTER(ctypes.c_int)]
    cap = 256
    d, g, m = (ctypes.c_uint64 * cap)(), (ctypes.c_uint64 * cap)(), (ctypes.c_int * cap)()
    dist, gen, depth = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
    t = time.time()
    v = lib.orc_prefix_levels(n, V, E, Rr, threads, max_states, seen_slots, d, g, m, cap, ctypes.byref(dist),
                              ctypes.byref(gen), ctypes.byref(depth))
    dt = time.time() - t
    D = depth.value
    assert v in (0, 2), f"unexpected verdict {v}"
    return {"n": n, "V": V, "E": E, "R": Rr, "max_states": max_states, "stopped_at_distinct": dist.value,
            "exhausted": v == 0, "levels": list(d[:D]), "gen_per_level": list(g[:D if v == 0 else D - 1]),
            "max_msgs_per_level": list(m[:D]), "max_msgs_seen": max(m[:D]), "oracle_seconds": round(dt, 1),
            "source": f"c_lean{threads}", "invariants": ["Inv"], "check_deadlock": False}


def main():
    args = sys.argv[1:]
    threads = lean = 0
    if args and args[0] == "--mt":
        threads, args = int(args[1]), args[2:]
    elif args and args[0] == "--lean":  # --lean THREADS SEEN_SLOTS
        threads, lean, args = int(args[1]), int(args[2]), args[3:]
    max_states = int(args[0])
    a = list(map(int, args[1:]))
    cfgs = [tuple(a[i:i + 4]) for i in range(0, len(a), 4)]
    path = os.environ.get("GOLDEN_PREFIX_OUT", os.path.join(HERE, "levels_prefix.json"))
    for (n, V, E, Rr) in cfgs:
        if lean:
            r = run_prefix_lean(n, V, E, Rr, max_states, threads, lean)
            old = (json.load(open(path)) if os.path.exists(path) else {}).get(f"n{n}_v{V}_e{E}_r{Rr}")
            if old:  # the lean run must reproduce the prefix already recorded
                k = min(len(old["levels"]), len(r["levels"]))
                assert r["levels"][:k] == old["levels"][:k], "lean prefix disagrees with the recorded one"
                k = min(len(old["gen_per_level"]), len(r["gen_per_level"]))
                assert r["gen_per_level"][:k] == old["gen_per_level"][:k], "lean generated counts disagree"
                r["previous_source"] = old["source"]
        elif threads:
            r = run_prefix_mt(n, V, E, Rr, max_states, threads)
        else:
            r = run_prefix(n, V, E, Rr, max_states)
        out = json.load(open(path)) if os.path.exists(path) else {}
        out[f"n{n}_v{V}_e{E}_r{Rr}"] = r
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        print(n, V, E, Rr, "levels", len(r["levels"]), "states", sum(r["levels"]), r["oracle_seconds"], "s",
              flush=True)


if __name__ == "__main__":
    main()
