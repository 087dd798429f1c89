"""Forced worst-case schedules at every in-launch hand-off (the race-probe build, -DRMC_RACE_PROBE).

Round 4 found a race in the device loop only statistically: a commit block with no parent that the
busy GPU started late read the control block after the launch's last arriver had advanced it to the
next level.  The probe build makes that schedule happen on every level, and the
others that could hide a similar fault: block 0 arrives last at k_wincount's and k_commit's counters,
and claimers of an election slot hold their y word back (elect_slot, owner_bid).  With the control-
block pair every golden run still matches -- device loop, host-driven split chunks, sharded rounds;
with the pre-pair logic (rmc_debug_race(1): one block read and written in place) configs[1] must come
out wrong in a single run.  Parity unpinned, as every golden here (tests/golden, the oracles)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RACE_LIB = os.path.join(ROOT, "tla-raft_amd", "build_race", "librmc.so")
LEVELS = json.load(open(os.path.join(GOLDEN, "levels.json")))
TRACES = json.load(open(os.path.join(GOLDEN, "traces.json")))
def cfg_of(g, **kw):
    c = dict(n_servers=g["n"], n_vals=g["V"], max_election=g["E"], max_restart=g["R"],
             invariants=list(g["invariants"]), check_deadlock=g["check_deadlock"],
             spec_variant=1 if g.get("seeded") else 0)
    c.update(kw)
    return c


def run_worker(single, runs, tmp_path, **extra_env):
    if not os.path.exists(RACE_LIB):
        pytest.fail(f"{RACE_LIB} missing: make -C tla-raft_amd (__graft_entry__.build) builds it")
    out = tmp_path / "race.json"
    env = dict(os.environ, RMC_LIBRARY=RACE_LIB, **extra_env)
    spec = {"single": single, "runs": runs, "out": str(out)}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "race_worker.py"), json.dumps(spec)], env=env,
                       capture_output=True, text=True, timeout=150)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    return json.load(open(out))


def matches(g, r, name):
    if r["status"] != {"ok": "done"}.get(g["verdict"], g["verdict"]):
        return False
    if (r["generated"], r["distinct"]) != (g["generated"], g["distinct"]):
        return False
    if g["verdict"] == "ok":
        return r["depth"] == g["depth"] and r["levels"] == g["levels"] and r["gen_per_level"] == g["gen_per_level"]
    ok = r["trace_len"] == g["trace_len"] and r["queue"] == g["queue_left"]
    if name in TRACES:
        ok = ok and r["trace"] == [[e["key"], e["state"]] for e in TRACES[name]["steps"]]
    return ok


NAMES = ["n3_v1_e2_r3", "seeded_n3_v2_e2_r3", "deadlock_n3_v1_e1_r3", "n4_v1_e1_r3", "exist_lc_n3_v1_e2_r3"]


def test_forced_schedules_keep_golden_results(tmp_path):
    """The probe build with the control-block pair: every golden run is exact on the device loop, on
    host-driven split chunks and on 2 / 3 virtual shards (split rounds: the owner elections too)."""
    runs = []
    for n in NAMES:
        g = LEVELS[n]
        runs.append({"name": n, "cfg": cfg_of(g)})
        runs.append({"name": n, "cfg": cfg_of(g, device_levels=1), "env": {"RMC_SPLIT_MIN": 1}})
        runs.append({"name": n, "cfg": cfg_of(g, virtual_shards=2, chunk_successors=3000, shard_min_states=40),
                     "env": {"RMC_SPLIT_MIN": 1}})
        runs.append({"name": n, "cfg": cfg_of(g, virtual_shards=3, chunk_successors=3000, shard_min_states=1)})
    res = run_worker(0, runs, tmp_path)
    bad = [(r["name"], i % 4, r.get("error") or (r["generated"], r["distinct"])) for i, r in enumerate(res)
           if not matches(LEVELS[r["name"]], r, r["name"])]
    assert not bad, bad


def test_single_control_block_fails_under_the_forced_late_block(tmp_path):
    """The logic before the pair (one control block per level, read and advanced in place) with the
    late commit block forced: configs[1] (3 servers, 1 value, MaxElection 2) must fail -- the late block
    takes the next level's parent count, arrives at the next level's counters and leaves them off by
    one (the probe build checks that every counter has re-armed itself when a level finishes; a
    violation found at that level could otherwise go to the wrong level's summary, round 4's symptom).
    With the item-parallel commit (16 parents a block) the late block's extra arrival can also fire a
    level's finish before that level's blocks are all in, and the run ends early with wrong counts
    before any re-arm check: either way the run is not the golden one."""
    g = LEVELS["n3_v1_e2_r3"]
    res = run_worker(1, [{"name": "n3_v1_e2_r3", "cfg": cfg_of(g)}], tmp_path)
    assert not matches(g, res[0], "n3_v1_e2_r3"), "the forced late block went unnoticed"
    r = res[0]
    assert "arrival counters" in r.get("error", "") or (r.get("distinct"), r.get("depth")) != (g["distinct"], g["depth"]), r

