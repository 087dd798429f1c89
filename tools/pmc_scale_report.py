#!/usr/bin/env python3
"""At-scale counters of the expansion, probe and commit kernels, per BFS level (tools/pmc_scale.sh output).

tools/pmc_scale.sh runs tools/explore.py once per counter pass: by default 3 servers / 2 values /
MaxElection 2 (18.5 M states), or Raft.cfg's first levels (CFG="3 2 3 3 --levels 44"); either way the
compact seen set is ~140 GB -- far beyond the 256 MB Infinity Cache, so FETCH_SIZE / WRITE_SIZE are
HBM traffic.  explore.py steps level by level on the host-driven path: a level of F parents is
ceil(F / chunk_parents) chunks, one dispatch of each kernel per chunk (k_hash_probe and k_insert_winners
only for chunks of at least --split-min parents), in dispatch order.  The explore log of the same pass gives each level's
parents F, successors G, new states N, average record bytes S and the HIP-event time of each kernel
phase; each dispatch's duration is its own (start / end timestamps of the FETCH_SIZE pass's records).
Per level (dispatches of a level summed) this records:

  alg_bytes    bench.py alg_bytes() -- the algorithmic bytes of the kernel
  hbm_bytes    2 * 1024 * FETCH_SIZE + 1024 * WRITE_SIZE (MI355X_MICROARCH.md rocprofv3 section; the
               x2 is the guide's gfx950 correction for wide streaming reads, an upper bound for the
               8-16 B random accesses that dominate here -- both readings are reported)
  ratio        hbm_bytes / alg_bytes (traffic well above 1 = whole lines moved for a few useful bytes)
  valu_frac    SQ_INSTS_VALU / duration against 256 CUs x 4 SIMDs x 2.4 GHz / 2 wave64 issues per s
               (the SQ pass's own dispatch durations would differ by the pass-to-pass spread)
  alg_GBps     alg_bytes / duration, hbm_GBps = hbm_bytes / duration (peak 8 TB/s)

usage: pmc_scale_report.py gpurun_out/pmcs out.json [--min-parents 500000] [--n 3 --V 2]"""
import argparse
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import HBM_PEAK_GBS, VALU_PEAK, alg_bytes, ctx_bytes  # noqa: E402

LEVEL = re.compile(r"^L\s*(\d+) F=\s*(\d+) G=\s*(\d+) N=\s*(\d+) tot=\s*\d+\s+[\d.]+ms \[([^\]]*)\].*rec=([\d.]+)B"
                   r"(?: self=(\d+))?")
# name -> (kernel name fragment, explore phase column of its HIP-event time, alg_bytes phase)
KERNELS = {"expand": ("k_expand", 1, "expand_hash"), "probe": ("k_hash_probe", 5, "probe"),
           "insert": ("k_insert_winners", 5, "insert"),
           # split chunks commit with k_commit_items<..., false, 64> (+ its one-wave k_commit_finish, not
           # counted; the fused levels' k_commit_items<..., true, 16> is not a split chunk's)
           "commit": ("k_commit_items|, false, 64>", 3, "materialize")}


def levels_of(log):
    out = []
    for ln in open(log):
        m = LEVEL.match(ln)
        if m:
            lv, F, G, N, ph, rec, slf = m.groups()
            out.append(dict(level=int(lv), F=int(F), G=int(G), N=int(N), ms=[float(x) for x in ph.split()],
                            rec=float(rec), self=int(slf or 0)))
    return out


def per_dispatch(csvf, kname):
    """Per dispatch of the kernel, in dispatch order: its counters and its duration in ms (the
    collection record's start / end timestamps)."""
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    frags = kname.split("|")  # every fragment in the kernel's name
    for r in csv.DictReader(open(csvf)):
        if all(f in r["Kernel_Name"] for f in frags):
            d = vals[int(r["Dispatch_Id"])]
            d[r["Counter_Name"]] += float(r["Counter_Value"])
            d["_ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return [vals[k] for k in sorted(vals)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("out")
    ap.add_argument("--min-parents", type=int, default=500000)
    ap.add_argument("--n", type=int, default=3)
    ap.add_argument("--V", type=int, default=2)
    ap.add_argument("--split-min", type=int, default=1 << 16)
    ap.add_argument("--workload", default="")
    a = ap.parse_args()
    maxsucc = 64 + a.n * (4 + a.V + a.n - 1)           # rmc_kernels.hip Spec::MAXS (one message round)
    chunk = min((1 << 28) // maxsucc, 1024 * 4096)     # rmc_engine.hip chunk_parents on one GPU
    report = {"workload": a.workload or "tools/explore.py (see the pass logs)", "hbm_peak_GBps": HBM_PEAK_GBS,
              "valu_peak_insts_per_s": VALU_PEAK, "chunk_parents": chunk,
              "note": "dispatches of a level summed; durations are the explore run's HIP events of the same pass",
              "kernels": {}}
    swb = 48 if a.n >= 4 else 32
    lv_f = levels_of(os.path.join(a.root, "fetch.log"))
    for key, (kname, ph, phase) in KERNELS.items():
        fetch = per_dispatch(os.path.join(a.root, "fetch", "run_counter_collection.csv"), kname)
        write = per_dispatch(os.path.join(a.root, "write", "run_counter_collection.csv"), kname)
        sq = per_dispatch(os.path.join(a.root, "sqa", "run_counter_collection.csv"), kname)
        if not fetch:
            continue
        # dispatches per level
        per = []
        for L in lv_f:
            nch = max(1, -(-L["F"] // chunk))
            if key in ("probe", "insert", "commit"):
                nch = sum(1 for c in range(nch) if min(chunk, L["F"] - c * chunk) >= a.split_min)
            per.append(nch)
        if not (len(fetch) == len(write) == len(sq) == sum(per)):
            sys.exit(f"{kname}: dispatches {len(fetch)}/{len(write)}/{len(sq)} vs {sum(per)} expected from the levels")
        rows, tot, k = [], collections.Counter(), 0
        for L, nch in zip(lv_f, per):
            d0, k = k, k + nch
            if L["F"] < a.min_parents or nch == 0:
                continue
            # duration: the dispatches' own timestamps in the FETCH_SIZE pass (the explore log's
            # HIP-event columns lump k_probe and k_insert_winners together)
            ms = sum(fetch[i]["_ms"] for i in range(d0, k))
            split = L["F"] >= a.split_min  # (every chunk of such a level is split at Raft.cfg's sizes)
            alg = alg_bytes(phase, L["F"], L["G"], L["N"], L["rec"], 0, 8, swb, split=split, CTXB=ctx_bytes(a.n, a.V),
                            Gself=L["self"])
            rd = 1024 * sum(fetch[i]["FETCH_SIZE"] for i in range(d0, k))
            wr = 1024 * sum(write[i]["WRITE_SIZE"] for i in range(d0, k))
            hbm = 2 * rd + wr
            valu = sum(sq[i]["SQ_INSTS_VALU"] for i in range(d0, k))
            rows.append({"level": L["level"], "parents": L["F"], "successors": L["G"], "new": L["N"], "chunks": nch,
                         "ms": ms, "alg_bytes": round(alg), "hbm_bytes": round(hbm), "hbm_bytes_fetch_x1": round(rd + wr),
                         "ratio": round(hbm / alg, 3), "ratio_fetch_x1": round((rd + wr) / alg, 3),
                         "alg_GBps": round(alg / ms / 1e6, 1), "hbm_GBps": round(hbm / ms / 1e6, 1),
                         "valu_insts": round(valu), "valu_per_successor": round(valu / max(1, L["G"]), 1),
                         "valu_frac": round(valu / (ms / 1e3) / VALU_PEAK, 4)})
            for kk, v in (("alg", alg), ("hbm", hbm), ("hbm1", rd + wr), ("ms", ms), ("valu", valu), ("G", L["G"])):
                tot[kk] += v
        if not rows:
            continue
        agg = {"levels": len(rows), "ms": round(tot["ms"], 3), "alg_bytes": round(tot["alg"]),
               "hbm_bytes": round(tot["hbm"]), "ratio": round(tot["hbm"] / tot["alg"], 3),
               "ratio_fetch_x1": round(tot["hbm1"] / tot["alg"], 3),
               "alg_GBps": round(tot["alg"] / tot["ms"] / 1e6, 1), "hbm_GBps": round(tot["hbm"] / tot["ms"] / 1e6, 1),
               "alg_frac": round(tot["alg"] / tot["ms"] / 1e6 / HBM_PEAK_GBS, 5),
               "hbm_frac": round(tot["hbm"] / tot["ms"] / 1e6 / HBM_PEAK_GBS, 5),
               "valu_frac": round(tot["valu"] / (tot["ms"] / 1e3) / VALU_PEAK, 4),
               "valu_per_successor": round(tot["valu"] / max(1, tot["G"]), 1)}
        report["kernels"][key] = {"kernel": kname.replace("|", " "), "levels_with_parents_ge": a.min_parents, "aggregate": agg,
                                  "per_level": rows}
        print(f"{key}: {agg}")
    with open(a.out, "w") as f:
        json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
