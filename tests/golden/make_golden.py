#!/usr/bin/env python3
"""Generate the committed golden fixtures from the oracles (run in the build container).

The reference ships no expected results (no TLC jar, no raft.log: /root/reference/.gitignore:1-3),
so every fixture here comes from the CPU restatements in oracle/:

* levels.json      per-level distinct/generated counts, depth, verdict for small and mid configs.
                   Small configs are computed by BOTH oracle/raft_ref.py and oracle/raft_oracle.c
                   and must agree; the larger ones by the C restatement alone (source field).
* successors.json  sampled reachable states with their successors in TLC order (keys + states),
                   plus server-permuted copies (same symmetry class) -- Python oracle.
* traces.json      counterexamples: the seeded commit bug, debug invariants that
                   are FALSE early, and a deadlock trace (check_deadlock on) -- Python oracle.

Usage: python tests/golden/make_golden.py [--big]
  (--big adds n3/V2/E2 = 18.5M states and n3/V1/E3 = 60.2M states: ~25 min of C-oracle time)
"""
import argparse
import ctypes
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import raft_ref as R  # noqa: E402

ORC = os.path.join(ROOT, "oracle", "build", "libraft_oracle.so")


def c_oracle():
    lib = ctypes.CDLL(ORC)
    lib.orc_create.restype = ctypes.c_void_p
    lib.orc_create.argtypes = [ctypes.c_int] * 6 + [ctypes.c_uint32, ctypes.c_int]
    lib.orc_run.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    for f in ("orc_generated", "orc_distinct", "orc_queue_left"):
        getattr(lib, f).restype = ctypes.c_uint64
        getattr(lib, f).argtypes = [ctypes.c_void_p]
    for f in ("orc_depth", "orc_violated", "orc_max_msgs", "orc_trace_len"):
        getattr(lib, f).argtypes = [ctypes.c_void_p]
    lib.orc_levels.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                               ctypes.c_int]
    lib.orc_destroy.argtypes = [ctypes.c_void_p]
    return lib


VERDICTS = {0: "ok", 1: "invariant", 2: "assert", 3: "eval_error", 4: "deadlock"}
INV_BIT = {"Inv": 0, "NoSplitVote": 1, "RaftCanCommt": 2, "FollowerCanCommit": 3, "CommitAll": 4,
           "NoAllCommit": 5, "ExistLeaderAndCandidate": 6}


def run_c(n, V, E, Rr, seeded=False, invs=("Inv",), deadlock=False):
    lib = c_oracle()
    mask = 0
    for i in invs:
        mask |= 1 << INV_BIT[i]
    h = lib.orc_create(n, V, E, Rr, int(seeded), int(deadlock), mask, 1)
    v = lib.orc_run(h, 0)
    d = (ctypes.c_uint64 * 1024)()
    g = (ctypes.c_uint64 * 1024)()
    L = lib.orc_levels(h, d, g, 1024)
    out = dict(verdict=VERDICTS[v], generated=lib.orc_generated(h), distinct=lib.orc_distinct(h),
               depth=lib.orc_depth(h), levels=[d[i] for i in range(L)], gen_per_level=[g[i] for i in range(L)],
               max_msgs=lib.orc_max_msgs(h), trace_len=lib.orc_trace_len(h), queue_left=lib.orc_queue_left(h))
    if v == 1:
        out["violated"] = invs[lib.orc_violated(h)] if lib.orc_violated(h) < len(invs) else lib.orc_violated(h)
    lib.orc_destroy(h)
    return out


def run_py(n, V, E, Rr, seeded=False, invs=("Inv",), deadlock=False, keep=False):
    cfg = R.Config(n=n, V=V, max_election=E, max_restart=Rr, seeded=seeded, invariants=tuple(invs),
                   check_deadlock=deadlock)
    return cfg, R.bfs(cfg, keep_states=keep)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true")
    args = ap.parse_args()

    # ---------------------------------------------------------------- levels.json
    both = [(3, 1, 1, 3), (3, 2, 1, 3), (2, 1, 2, 3), (4, 1, 1, 3), (3, 1, 2, 3)]
    c_only = [(2, 2, 3, 3), (3, 3, 1, 3), (5, 1, 1, 3), (3, 1, 2, 1), (2, 1, 3, 2)]
    if args.big:
        c_only += [(3, 2, 2, 3), (3, 1, 3, 3)]
    levels = {}
    for (n, V, E, Rr) in both + c_only:
        name = f"n{n}_v{V}_e{E}_r{Rr}"
        c = run_c(n, V, E, Rr)
        src = "c"
        if (n, V, E, Rr) in both:
            _, p = run_py(n, V, E, Rr)
            assert (p.verdict, p.generated, p.distinct, p.depth, p.levels, p.generated_per_level) == (
                c["verdict"], c["generated"], c["distinct"], c["depth"], c["levels"], c["gen_per_level"]), name
            src = "python+c"
        c.update(n=n, V=V, E=E, R=Rr, seeded=False, invariants=["Inv"], check_deadlock=False, source=src)
        levels[name] = c
        print(name, c["distinct"], c["depth"], src, flush=True)
    # seeded commit bug (BASELINE config 5) and debug invariants / deadlock
    extra = [
        ("seeded_n3_v1_e2_r3", dict(n=3, V=1, E=2, Rr=3, seeded=True)),
        ("seeded_n3_v2_e2_r3", dict(n=3, V=2, E=2, Rr=3, seeded=True)),
        ("nosplit_n3_v1_e2_r3", dict(n=3, V=1, E=2, Rr=3, invs=("Inv", "NoSplitVote"))),
        ("deadlock_n3_v1_e1_r3", dict(n=3, V=1, E=1, Rr=3, deadlock=True)),
        ("raftcancommit_n3_v1_e1_r3", dict(n=3, V=1, E=1, Rr=3, invs=("RaftCanCommt",))),
        ("exist_lc_n3_v1_e2_r3", dict(n=3, V=1, E=2, Rr=3, invs=("ExistLeaderAndCandidate",))),
    ]
    for name, kw in extra:
        c = run_c(kw["n"], kw["V"], kw["E"], kw["Rr"], kw.get("seeded", False), kw.get("invs", ("Inv",)),
                  kw.get("deadlock", False))
        _, p = run_py(kw["n"], kw["V"], kw["E"], kw["Rr"], kw.get("seeded", False), kw.get("invs", ("Inv",)),
                      kw.get("deadlock", False))
        assert (p.verdict, p.generated, p.distinct) == (c["verdict"], c["generated"], c["distinct"]), name
        assert (len(p.trace) if p.trace else 0) == c["trace_len"], name
        c.update(n=kw["n"], V=kw["V"], E=kw["E"], R=kw["Rr"], seeded=kw.get("seeded", False),
                 invariants=list(kw.get("invs", ("Inv",))), check_deadlock=kw.get("deadlock", False),
                 source="python+c", queue_left=p.queue_left, violated=p.violated)
        levels[name] = c
        print(name, c["verdict"], c["distinct"], c["trace_len"], flush=True)
    with open(os.path.join(HERE, "levels.json"), "w") as f:
        json.dump(levels, f, indent=1)

    # ---------------------------------------------------------------- traces.json
    traces = {}
    for name, kw in extra:
        cfg, p = run_py(kw["n"], kw["V"], kw["E"], kw["Rr"], kw.get("seeded", False), kw.get("invs", ("Inv",)),
                        kw.get("deadlock", False))
        if p.trace:
            traces[name] = dict(verdict=p.verdict, violated=p.violated,
                                steps=[dict(key=list(k) if k else None, state=R.state_to_json(s)) for k, s in p.trace])
    with open(os.path.join(HERE, "traces.json"), "w") as f:
        json.dump(traces, f)

    # ---------------------------------------------------------------- successors.json
    rng = random.Random(20260101)
    samples = {}
    for (n, V, E, Rr, k) in [(3, 1, 2, 3, 60), (3, 2, 1, 3, 40), (2, 2, 2, 3, 20), (4, 1, 1, 3, 20),
                             (3, 1, 2, 3, 0)]:
        if k == 0:
            continue
        cfg, p = run_py(n, V, E, Rr, keep=True)
        picks = rng.sample(range(len(p.states)), k)
        # bias towards deep states: add the last few states too
        picks += list(range(len(p.states) - 5, len(p.states)))
        items = []
        for i in picks:
            st = p.states[i]
            succ = R.successors(cfg, st)
            perm = list(range(n))
            rng.shuffle(perm)
            pv = R.permute_view(st.view(), perm)
            # rebuild a concrete permuted state (hidden vars permuted too)
            inv = [0] * n
            for a in range(n):
                inv[perm[a]] = a
            pst = R.State(votedFor=pv[0], currentTerm=pv[1], logs=pv[2], matchIndex=pv[3], nextIndex=pv[4],
                          commitIndex=pv[5], msgs=frozenset(pv[6]), role=pv[7], electionCount=st.electionCount,
                          restartCount=st.restartCount,
                          pendingResponse=tuple(tuple(st.pendingResponse[inv[a]][inv[b]] for b in range(n))
                                                for a in range(n)),
                          valSent=st.valSent)
            assert R.canonical(cfg, pst) == R.canonical(cfg, st)
            items.append(dict(level=p.state_levels[i], state=R.state_to_json(st), permuted=R.state_to_json(pst),
                              canon_id=None,
                              successors=[dict(key=list(kk), state=R.state_to_json(t)) for kk, t in succ]))
        # canonical classes among all successors of the samples (fingerprint equivalence)
        canon_ids = {}
        for it in items:
            for sc in it["successors"]:
                c = R.canonical(cfg, R.state_from_json(sc["state"]))
                sc["canon"] = canon_ids.setdefault(c, len(canon_ids))
        samples[f"n{n}_v{V}_e{E}_r{Rr}"] = dict(n=n, V=V, E=E, R=Rr, items=items)
        print("samples", n, V, E, len(items), flush=True)
    with open(os.path.join(HERE, "successors.json"), "w") as f:
        json.dump(samples, f)


if __name__ == "__main__":
    main()
