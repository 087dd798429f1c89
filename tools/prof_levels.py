"""Per-level view of a rocprofv3 kernel trace of bench.py (configs[1]).

The device-driven loop enqueues levels in groups, so each exhaustion ends with a few no-op
launches (the loop has stopped; every block returns at once).  bench.py's HIP-event figure
averages only launches that expanded a level; this script gives rocprof's average over the
same set: runs are split at Init's fingerprint launch, and the first `depth` launches of each kernel per run
are the real levels.

usage: python tools/prof_levels.py gpurun_out/prof/bench_kernel_trace.csv [depth=37]
"""
import csv
import sys
from collections import defaultdict


def main(path, depth=37):
    rows = [r for r in csv.DictReader(open(path)) if "rmc::k_" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # every exhaustion starts by fingerprinting Init (k_fp_states): that launch splits the runs
    runs, cur = [], []
    for r in rows:
        if "k_fp_states" in r["Kernel_Name"] and cur:
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


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 37)
