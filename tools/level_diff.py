#!/usr/bin/env python3
"""First BFS level where a run departs from a golden level list (tests/golden/levels_big.json or
levels.json): the device-driven run (mc.run) and the host-driven one (mc.step per level).

usage: level_diff.py NAME [--file levels_big.json] [--host-only]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-raft_amd"))
import raftmc  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("name")
ap.add_argument("--file", default="levels_big.json")
ap.add_argument("--host-only", action="store_true")
a = ap.parse_args()
g = json.load(open(os.path.join(ROOT, "tests", "golden", a.file)))[a.name]


def cfg():
    return raftmc.ModelConfig(n_servers=g["n"], n_vals=g["V"], max_election=g["E"], max_restart=g["R"],
                              invariants=tuple(g["invariants"]), check_deadlock=g["check_deadlock"])


def report(kind, news, gens):
    want_n, want_g = g["levels"], [None] + g["gen_per_level"]
    for i, (n, gg) in enumerate(zip(news, gens)):
        wn = want_n[i] if i < len(want_n) else None
        wg = want_g[i] if i < len(want_g) else None
        if wn is None and n == 0:  # the empty level after the last
            break
        if n != wn or (wg is not None and gg != wg):
            print(f"{kind}: level {i + 1} departs: new {n} (golden {wn}), generated {gg} (golden {wg})")
            return
    if len([n for n in news if n]) != len(want_n):
        print(f"{kind}: {len([n for n in news if n])} nonempty levels, golden {len(want_n)}")
        return
    print(f"{kind}: all {len(news)} levels match")


if not a.host_only:
    mc = raftmc.ModelChecker(cfg())
    res = mc.run()
    report("device-driven", [ls.new_states for ls in res.levels], [ls.generated for ls in res.levels])
    for i, ls in enumerate(res.levels[:60]):
        print(f"  L{i + 1} F={ls.expanded} G={ls.generated} N={ls.new_states}")
    mc.close()
mc = raftmc.ModelChecker(cfg())
ls = mc.init()
news, gens = [ls.new_states], [ls.generated]
while ls.status == "ok":
    ls = mc.step()
    news.append(ls.new_states)
    gens.append(ls.generated)
report("host-driven", news, gens)
mc.close()
