#!/usr/bin/env python3
"""Where the GPU timeline goes between kernels: a rocprofv3 --kernel-trace (+ --memory-copy-trace)
of a run, cut into windows of `--window` ms; per window, the time inside each kernel, inside
copies (by direction), and idle (no kernel or copy running).  Idle time is host round trips and
launch latency -- the per-chunk overhead of a host-driven level.

usage: python tools/gaps.py kernel_trace.csv [memory_copy_trace.csv] [--window MS] [--last K]"""
import argparse
import csv
from collections import defaultdict


def load(path, kind):
    out = []
    for r in csv.DictReader(open(path)):
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"] if kind == "k" else r["Direction"].replace("MEMORY_COPY_", "copy ")
        if kind == "k":
            name = name.split("(")[0].replace("void ", "")
        out.append((a, b, name))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernels")
    ap.add_argument("copies", nargs="?")
    ap.add_argument("--window", type=float, default=1000.0)
    ap.add_argument("--last", type=int, default=8)
    a = ap.parse_args()
    ev = load(a.kernels, "k") + (load(a.copies, "c") if a.copies else [])
    ev.sort()
    t0, t1 = ev[0][0], max(e[1] for e in ev)
    W = int(a.window * 1e6)
    wins = defaultdict(lambda: defaultdict(float))
    busy = defaultdict(float)
    # union of busy intervals per window
    cur_a, cur_b = ev[0][0], ev[0][1]
    merged = []
    for s, e, n in ev:
        if s > cur_b:
            merged.append((cur_a, cur_b))
            cur_a, cur_b = s, e
        else:
            cur_b = max(cur_b, e)
        w = (s - t0) // W
        wins[w][n] += (e - s) / 1e6
        wins[w]["#" + n] += 1
    merged.append((cur_a, cur_b))
    for s, e in merged:
        ws, we = (s - t0) // W, (e - t0) // W
        for w in range(ws, we + 1):
            lo, hi = max(s, t0 + w * W), min(e, t0 + (w + 1) * W)
            if hi > lo:
                busy[w] += (hi - lo) / 1e6
    nw = (t1 - t0) // W + 1
    print(f"span {(t1 - t0) / 1e9:.2f} s, {len(ev)} events, window {a.window:.0f} ms")
    for w in range(max(0, nw - a.last), nw):
        tot = min(W, t1 - t0 - w * W) / 1e6
        d = wins[w]
        parts = ", ".join(f"{k} {v:.1f} ms/{int(d['#' + k])}" for k, v in sorted(d.items(), key=lambda x: -x[1])
                          if not k.startswith("#") and v > 0.05 * tot)
        print(f"[{w * a.window / 1000:7.1f} s] busy {busy[w]:7.1f} of {tot:7.1f} ms ({100 * busy[w] / tot:5.1f} %)  {parts}")


if __name__ == "__main__":
    main()
