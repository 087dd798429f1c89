"""Full-size golden levels from the C oracle (oracle/raft_oracle.c, TLC -workers 1 BFS).

Writes levels_big.json: per-level distinct/generated counts, depth and verdict of the
configurations bench.py runs at scale, so the GPU path is pinned at those sizes too.
(3, 2, 2, 3) is bench.py's at-scale workload: ~18.5 M distinct states, a few minutes and a
few GB of host memory for the oracle.

usage: python tests/golden/make_golden_big.py [n V E R ...]
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import run_c  # noqa: E402


def main():
    cfgs = [(3, 2, 2, 3)]
    if len(sys.argv) > 1:
        a = list(map(int, sys.argv[1:]))
        cfgs = [tuple(a[i:i + 4]) for i in range(0, len(a), 4)]
    path = os.environ.get("GOLDEN_BIG_OUT", os.path.join(HERE, "levels_big.json"))
    out = json.load(open(path)) if os.path.exists(path) else {}
    for (n, V, E, Rr) in cfgs:
        t = time.time()
        c = run_c(n, V, E, Rr)
        c.update(n=n, V=V, E=E, R=Rr, seeded=False, invariants=["Inv"], check_deadlock=False, source="c",
                 oracle_seconds=round(time.time() - t, 1))
        out[f"n{n}_v{V}_e{E}_r{Rr}"] = c
        print(n, V, E, Rr, c["verdict"], c["distinct"], c["generated"], c["depth"], c["oracle_seconds"], "s", flush=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
