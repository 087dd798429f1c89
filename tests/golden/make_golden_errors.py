#!/usr/bin/env python3
"""Golden fixtures of the two test variants that make TLC's non-invariant errors reachable in a BFS
(tools/make_seeded_spec.py --split-brain / --commit-past-log; RMC_SPEC_SPLIT_BRAIN / _COMMIT_PAST_LOG),
from the oracles, as make_golden.py does for Raft.tla:

* levels_errors.json  verdict ("assert" / "eval_error"), TLC's counters at the error (states generated
                      and distinct, queue left), the levels completed before it -- every config by
                      BOTH oracle/raft_ref.py and oracle/raft_oracle.c, which must agree;
* traces_errors.json  the counterexamples (the state whose expansion fails the Assert, or the new state
                      on which Inv's evaluation fails), Python oracle.

The shipped specs reach neither error, so these are the only BFS-level checks of their precedence
(an Assert stops the expansion before its sub-action's batch is counted; an
evaluation error is raised on the new state, as an invariant violation is).  Parity unpinned: there
is no TLC here, and the variants are this build's test specs.

Usage: python tests/golden/make_golden_errors.py
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import INV_BIT, R, VERDICTS, c_oracle  # noqa: E402

FLAGS = {"split_brain": 4, "commit_past_log": 8}  # oracle/raft_oracle.c set_variant bits

CONFIGS = [
    ("sb_n3_v1_e2_r3", "split_brain", (3, 1, 2, 3), ("Inv",)),
    ("sb_n2_v1_e2_r3", "split_brain", (2, 1, 2, 3), ("Inv",)),
    ("sb_n3_v2_e2_r3", "split_brain", (3, 2, 2, 3), ("Inv",)),
    ("sb_n3_v1_e3_r3", "split_brain", (3, 1, 3, 3), ("Inv", "NoSplitVote")),
    ("cpl_n3_v2_e1_r3", "commit_past_log", (3, 2, 1, 3), ("Inv",)),
    ("cpl_n3_v2_e2_r3", "commit_past_log", (3, 2, 2, 3), ("Inv",)),
    ("cpl_n3_v2_e1_r3_nosplit", "commit_past_log", (3, 2, 1, 3), ("NoSplitVote", "Inv")),
]


def run_c(variant, n, V, E, Rr, invs):
    lib = c_oracle()
    mask = 0
    for i in invs:
        mask |= 1 << INV_BIT[i]
    h = lib.orc_create(n, V, E, Rr, FLAGS[variant], 0, mask, 1)
    v = lib.orc_run(h, 0)
    d = (ctypes.c_uint64 * 1024)()
    g = (ctypes.c_uint64 * 1024)()
    L = lib.orc_levels(h, d, g, 1024)
    out = dict(verdict=VERDICTS[v], generated=lib.orc_generated(h), distinct=lib.orc_distinct(h),
               depth=lib.orc_depth(h), levels=[d[i] for i in range(L)], gen_per_level=[g[i] for i in range(L)],
               max_msgs=lib.orc_max_msgs(h), trace_len=lib.orc_trace_len(h), queue_left=lib.orc_queue_left(h))
    lib.orc_destroy(h)
    return out


def main():
    levels, traces = {}, {}
    for name, variant, (n, V, E, Rr), invs in CONFIGS:
        c = run_c(variant, n, V, E, Rr, invs)
        cfg = R.Config(n=n, V=V, max_election=E, max_restart=Rr, invariants=tuple(invs), **{variant: True})
        p = R.bfs(cfg)
        assert (p.verdict, p.generated, p.distinct) == (c["verdict"], c["generated"], c["distinct"]), (name, p, c)
        assert (len(p.trace) if p.trace else 0) == c["trace_len"] and p.queue_left == c["queue_left"], name
        # (mixed INVARIANT lists: whichever error TLC meets first -- e.g. NoSplitVote fails before the Assert)
        c.update(n=n, V=V, E=E, R=Rr, seeded=False, variant=variant, invariants=list(invs), check_deadlock=False,
                 source="python+c", violated=p.violated)
        levels[name] = c
        traces[name] = dict(verdict=p.verdict, violated=p.violated,
                            steps=[dict(key=list(k) if k else None, state=R.state_to_json(s)) for k, s in p.trace])
        print(name, c["verdict"], c["generated"], c["distinct"], c["trace_len"], flush=True)
    with open(os.path.join(HERE, "levels_errors.json"), "w") as f:
        json.dump(levels, f, indent=1)
    with open(os.path.join(HERE, "traces_errors.json"), "w") as f:
        json.dump(traces, f)


if __name__ == "__main__":
    main()
