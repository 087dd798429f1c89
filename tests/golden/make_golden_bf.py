#!/usr/bin/env python3
"""Golden fixtures of the BecomeFollower variant (Raft.tla with Next's `\\/ BecomeFollower(s)`
uncommented, tla:420; RMC_SPEC_BECOME_FOLLOWER) from the oracles, as make_golden.py does for
Raft.tla:

* levels_bf.json      per-level counts, depth, verdict -- small configs by BOTH oracle/raft_ref.py
                      and oracle/raft_oracle.c (must agree), larger ones by the C restatement alone;
* successors_bf.json  sampled reachable states with their successors in TLC order (Python oracle);
* traces_bf.json      counterexamples of debug invariants under the variant (Python oracle).

Usage: python tests/golden/make_golden_bf.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import INV_BIT, R, VERDICTS, c_oracle  # noqa: E402


def run_c(n, V, E, Rr, invs=("Inv",), deadlock=False):
    import ctypes
    lib = c_oracle()
    mask = 0
    for i in invs:
        mask |= 1 << INV_BIT[i]
    h = lib.orc_create(n, V, E, Rr, 2, int(deadlock), mask, 1)  # spec flags: bit 1 = BecomeFollower
    v = lib.orc_run(h, 0)
    d = (ctypes.c_uint64 * 1024)()
    g = (ctypes.c_uint64 * 1024)()
    L = lib.orc_levels(h, d, g, 1024)
    out = dict(verdict=VERDICTS[v], generated=lib.orc_generated(h), distinct=lib.orc_distinct(h),
               depth=lib.orc_depth(h), levels=[d[i] for i in range(L)], gen_per_level=[g[i] for i in range(L)],
               max_msgs=lib.orc_max_msgs(h), trace_len=lib.orc_trace_len(h), queue_left=lib.orc_queue_left(h))
    lib.orc_destroy(h)
    return out


def py_cfg(n, V, E, Rr, invs=("Inv",), deadlock=False):
    return R.Config(n=n, V=V, max_election=E, max_restart=Rr, invariants=tuple(invs), check_deadlock=deadlock,
                    become_follower=True)


def main():
    levels, traces = {}, {}
    runs = [("bf_n3_v1_e1_r3", (3, 1, 1, 3), {}, True), ("bf_n3_v2_e1_r3", (3, 2, 1, 3), {}, True),
            ("bf_n2_v1_e2_r3", (2, 1, 2, 3), {}, True), ("bf_n4_v1_e1_r3", (4, 1, 1, 3), {}, True),
            ("bf_n3_v1_e2_r3", (3, 1, 2, 3), {}, True), ("bf_n5_v1_e1_r3", (5, 1, 1, 3), {}, False),
            ("bf_n2_v2_e3_r3", (2, 2, 3, 3), {}, False),
            ("bf_deadlock_n3_v1_e1_r3", (3, 1, 1, 3), dict(deadlock=True), True),
            ("bf_nosplit_n3_v1_e2_r3", (3, 1, 2, 3), dict(invs=("Inv", "NoSplitVote")), True),
            ("bf_exist_lc_n3_v1_e2_r3", (3, 1, 2, 3), dict(invs=("ExistLeaderAndCandidate",)), True)]
    for name, (n, V, E, Rr), kw, both in runs:
        c = run_c(n, V, E, Rr, **kw)
        src = "c"
        if both:
            cfg = py_cfg(n, V, E, Rr, **kw)
            p = R.bfs(cfg)
            assert (p.verdict, p.generated, p.distinct, p.depth) == (
                c["verdict"], c["generated"], c["distinct"], c["depth"]), name
            if p.verdict == "ok":
                assert (p.levels, p.generated_per_level) == (c["levels"], c["gen_per_level"]), name
            assert (len(p.trace) if p.trace else 0) == c["trace_len"], name
            src = "python+c"
            c.update(queue_left=p.queue_left, violated=p.violated)
            if p.trace:
                traces[name] = dict(verdict=p.verdict, violated=p.violated,
                                    steps=[dict(key=list(k) if k else None, state=R.state_to_json(s))
                                           for k, s in p.trace])
        c.update(n=n, V=V, E=E, R=Rr, seeded=False, become_follower=True,
                 invariants=list(kw.get("invs", ("Inv",))), check_deadlock=kw.get("deadlock", False), source=src)
        levels[name] = c
        print(name, c["verdict"], c["distinct"], c["depth"], src, flush=True)
    with open(os.path.join(HERE, "levels_bf.json"), "w") as f:
        json.dump(levels, f, indent=1)
    with open(os.path.join(HERE, "traces_bf.json"), "w") as f:
        json.dump(traces, f)

    rng = random.Random(20261016)
    samples = {}
    for (n, V, E, Rr, k) in [(3, 1, 2, 3, 40), (3, 2, 1, 3, 20), (4, 1, 1, 3, 15)]:
        cfg = py_cfg(n, V, E, Rr)
        p = R.bfs(cfg, keep_states=True)
        picks = rng.sample(range(len(p.states)), k) + list(range(len(p.states) - 5, len(p.states)))
        items = []
        for i in picks:
            st = p.states[i]
            items.append(dict(level=p.state_levels[i], state=R.state_to_json(st),
                              successors=[dict(key=list(kk), state=R.state_to_json(t))
                                          for kk, t in R.successors(cfg, st)]))
        samples[f"bf_n{n}_v{V}_e{E}_r{Rr}"] = dict(n=n, V=V, E=E, R=Rr, items=items)
        print("samples", n, V, E, len(items), sum(len(it["successors"]) for it in items), flush=True)
    with open(os.path.join(HERE, "successors_bf.json"), "w") as f:
        json.dump(samples, f)


if __name__ == "__main__":
    main()
