#!/usr/bin/env python3
"""Sum the per-level HIP-event kernel times of tools/explore.py logs.

Columns: [count, expand, winner count, commit, exchange, other (k_probe, k_insert_winners, appends)] in
seconds, their sum, and the RESULT line's wall seconds.  usage: phase_sums.py LOG [LOG ...]"""
import re
import sys

for path in sys.argv[1:]:
    tot, wall = [0.0] * 6, None
    for ln in open(path):
        m = re.search(r"\[([^\]]*)\]", ln)
        if ln.startswith("L") and m:
            for i, x in enumerate(m.group(1).split()):
                tot[i] += float(x)
        r = re.search(r"^RESULT .* seconds ([\d.]+)", ln)
        if r:
            wall = float(r.group(1))
    print(f"{path}: {[round(x / 1000, 2) for x in tot]} kernels {sum(tot) / 1000:.2f} s, wall {wall} s")
