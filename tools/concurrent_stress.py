"""Repeats small golden configurations on one GPU for a fixed time and counts runs whose counters,
levels or counterexample differ from the golden ones (tests/golden).  Started as two or more
processes at once, it checks the single-GPU path while other processes share the card -- the
condition under which the multi-rank tests' rare mismatch appeared.

usage: python tools/concurrent_stress.py SECONDS [device_levels] [name ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-raft_amd"))
import raftmc  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
LEVELS = json.load(open(os.path.join(GOLD, "levels.json")))
TRACES = json.load(open(os.path.join(GOLD, "traces.json")))


def main():
    secs = float(sys.argv[1])
    dl = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    names = sys.argv[3:] or ["deadlock_n3_v1_e1_r3", "n3_v1_e2_r3", "seeded_n3_v2_e2_r3"]
    t_end = time.time() + secs
    runs = bad = 0
    last = time.time()
    while time.time() < t_end:
        for name in names:
            g = LEVELS[name]
            mc = raftmc.ModelChecker(raftmc.ModelConfig(
                n_servers=g["n"], n_vals=g["V"], max_election=g["E"], max_restart=g["R"],
                invariants=tuple(g["invariants"]), check_deadlock=g["check_deadlock"],
                spec_variant=1 if g["seeded"] else 0, chunk_successors=3000, device_levels=dl))
            res = mc.run()
            got = (res.generated, res.distinct)
            lv = [ls.new_states for ls in res.levels if ls.new_states]
            ok = got == (g["generated"], g["distinct"])
            if g["verdict"] == "ok":
                ok = ok and lv == g["levels"]
            if ok and name in TRACES:
                ok = [st for _, st in mc.trace()] == [e["state"] for e in TRACES[name]["steps"]]
            mc.close()
            runs += 1
            if not ok:
                bad += 1
                print(f"MISMATCH {name}: {got} vs {(g['generated'], g['distinct'])} levels {lv}", flush=True)
        if time.time() - last > 30:
            print(f"pid {os.getpid()}: {runs} runs, {bad} mismatches", flush=True)
            last = time.time()
    print(f"pid {os.getpid()} device_levels={dl}: {runs} runs, {bad} mismatches", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
