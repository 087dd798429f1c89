"""Per-level view of a rocprofv3 kernel trace of bench.py (configs[1]).

The device-driven loop enqueues levels in groups, so each exhaustion ends with a few no-op
launches (the loop has stopped; every block returns at once).  bench.py's HIP-event figure
averages only launches that expanded a level; this script gives rocprof's average over the
same set: runs are split at Init's fingerprint launch, and the first `depth` launches of each kernel per run
are the real levels.

usage: python tools/prof_levels.py gpurun_out/prof/bench_kernel_trace.csv [depth=37] [--per-level]

--per-level adds, per BFS level, the median over runs of each kernel's duration and of the idle
gap in front of it, and per run the span from the first launch to the last level's last kernel.
"""
import csv
import sys
from collections import defaultdict


def per_level(runs, depth):
    import statistics
    med = lambda xs: statistics.median(xs) if xs else 0.0
    table = defaultdict(lambda: defaultdict(list))  # level -> kernel -> [dur us]
    gaps = defaultdict(lambda: defaultdict(list))
    spans = []
    for run in runs:
        seen = defaultdict(int)
        prev_end, last_end = None, None
        first = int(run[0]["Start_Timestamp"])
        for r in run:
            k = r["Kernel_Name"].split("(")[0].replace("void rmc::", "").split("<")[0]
            b, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            seen[k] += 1
            lvl = seen[k]
            if k in ("k_expand", "k_wincount", "k_commit") and lvl <= depth:
                table[lvl][k].append((e - b) / 1e3)
                if prev_end is not None:
                    gaps[lvl][k].append((b - prev_end) / 1e3)
                last_end = e
            prev_end = e
        if last_end:
            spans.append((last_end - first) / 1e3)
    print(f"per level (median over {len(runs)} runs, us): kernel duration [idle gap before it]")
    tot = defaultdict(float)
    for lvl in sorted(table):
        cells = []
        for k in ("k_expand", "k_wincount", "k_commit"):
            d, g = med(table[lvl][k]), med(gaps[lvl][k])
            tot[k] += d
            tot[k + " gap"] += g
            cells.append(f"{k[2:]:8s} {d:7.2f} [{g:5.2f}]")
        print(f"L{lvl:3d} " + "  ".join(cells))
    print("sum over levels: " + ", ".join(f"{k} {v:.1f}" for k, v in tot.items()))
    print(f"GPU span per run (first launch -> last level's commit end): median {med(spans):.1f} us")


def main(path, depth=37, levels=False):
    rows = [r for r in csv.DictReader(open(path)) if "rmc::k_" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # every exhaustion starts with Init's level (k_fp_states the first time, k_init_level after): that launch splits the runs
    runs, cur = [], []
    for r in rows:
        if ("k_fp_states" in r["Kernel_Name"] or "k_init_level" in r["Kernel_Name"]) and cur:
            runs.append(cur)
            cur = []
        cur.append(r)
    runs.append(cur)
    tot, cnt, noop, nnoop = defaultdict(int), defaultdict(int), defaultdict(int), defaultdict(int)
    for run in runs:
        seen = defaultdict(int)
        for r in run:
            k = r["Kernel_Name"].split("(")[0].replace("void rmc::", "")
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            seen[k] += 1
            if seen[k] <= depth:
                tot[k] += d
                cnt[k] += 1
            else:
                noop[k] += d
                nnoop[k] += 1
    print(f"{len(runs)} runs, first {depth} launches per kernel per run = levels that ran")
    for k in sorted(tot, key=lambda k: -tot[k]):
        line = f"{k:32s} level launches {cnt[k]:5d} avg {tot[k] / cnt[k] / 1e3:7.2f} us"
        if nnoop[k]:
            line += f" | no-op launches {nnoop[k]:4d} avg {noop[k] / nnoop[k] / 1e3:5.2f} us"
        print(line)
    if levels:
        per_level(runs, depth)


if __name__ == "__main__":
    pos = [a for a in sys.argv[1:] if not a.startswith("--")]
    main(pos[0], int(pos[1]) if len(pos) > 1 else 37, "--per-level" in sys.argv)
