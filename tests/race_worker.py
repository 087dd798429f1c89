"""Runs golden configurations through the race-probe build of librmc.so (test helper).

usage: RMC_LIBRARY=tla-raft_amd/build_race/librmc.so python race_worker.py SPEC_JSON
SPEC = {"single": 0|1 (rmc_debug_race: one control block per device-loop level, the logic before the
pair), "runs": [{"name", "cfg": ModelConfig keywords, "env": {...}}], "out": result path}.  Every
in-launch hand-off of that build runs its forced worst-case schedule (rmc_kernels.hip, race probe);
each run's counters, levels and trace go to `out` as JSON for the caller to compare with the goldens."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-raft_amd"))

import raftmc  # noqa: E402


def main():
    spec = json.loads(sys.argv[1])
    lib = raftmc.load_library()
    if not hasattr(lib, "rmc_debug_race"):
        sys.exit("this librmc.so was not built with -DRMC_RACE_PROBE")
    out = []
    for run in spec["runs"]:
        for k, v in run.get("env", {}).items():
            os.environ[k] = str(v)
        if lib.rmc_debug_race(int(spec["single"])) != 0:
            sys.exit("rmc_debug_race failed")
        r = {"name": run["name"]}
        try:
            with raftmc.ModelChecker(raftmc.ModelConfig(device=0, **run["cfg"])) as mc:
                res = mc.run()
                r.update(status=res.status, generated=res.generated, distinct=res.distinct, depth=res.depth,
                         queue=res.queue, violated=res.violated, trace_len=res.trace_len,
                         levels=[ls.new_states for ls in res.levels if ls.new_states],
                         gen_per_level=[ls.generated for ls in res.levels[1:]],
                         trace=[[list(k) if k else None, st] for k, st in mc.trace()] if res.trace_len else [])
        except raftmc.RmcError as e:
            r.update(status="error", error=str(e))
        for k in run.get("env", {}):
            os.environ.pop(k, None)
        out.append(r)
    with open(spec["out"], "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
