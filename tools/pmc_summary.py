#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) per kernel: averages per dispatch.

HBM bytes follow MI355X_MICROARCH.md's rocprofv3 section: FETCH_SIZE/WRITE_SIZE are KiB;
FETCH_SIZE reads half the bytes of a wide coalesced streaming read on gfx950, so
hbm_read_bytes = 2 * 1024 * FETCH_SIZE (the prescribed correction; our kernels mix scalar
and 16-B loads, so the factor is an upper bound there), hbm_write_bytes = 1024 * WRITE_SIZE.
usage: pmc_summary.py gpurun_out/pmc out.json"""
import collections
import csv
import json
import os
import sys

root, out = sys.argv[1], sys.argv[2]
# per counter: divide by the dispatch count of the pass that collected it
per = collections.defaultdict(dict)
for name in sorted(os.listdir(root)):
    f = os.path.join(root, name, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    ds = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        sums[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
        ds[r["Kernel_Name"]].add(r["Dispatch_Id"])
    for k, cs in sums.items():
        for c, v in cs.items():
            per[k][c] = v / len(ds[k])
        per[k]["dispatches"] = len(ds[k])
summary = {}
for k, cs in per.items():
    e = dict(cs)
    if "FETCH_SIZE" in cs:
        e["hbm_read_bytes"] = 2 * 1024 * cs["FETCH_SIZE"]
    if "WRITE_SIZE" in cs:
        e["hbm_write_bytes"] = 1024 * cs["WRITE_SIZE"]
    if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
        e["hbm_bytes_per_dispatch"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
    if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
        e["l2_hit_rate"] = cs["TCC_HIT_sum"] / max(1.0, cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"])
    summary[k] = e
json.dump(summary, open(out, "w"), indent=1, sort_keys=True)
print(f"{len(summary)} kernels -> {out}")
