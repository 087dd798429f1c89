"""The multi-rank sharded path with real process separation (myrun.sh:3 -workers).

RCCL refuses two ranks on one device, so on a one-GPU box the ranks exchange through the
host-staged transport (include/rmc.h rmc_transport; raftmc.HostTransport over a gloo group):
W processes, each its own context on device 0, each holding one fingerprint-owner shard of the
block-cyclic level, every collective of step_sharded (level sizes, gathered count matrices, the
successor / verdict / winner all-to-all-v, failure agreement) between separate processes.  The
runs must give the golden levels, counters at the error and counterexamples of the single GPU
(tests/golden/), and an allocation failure injected on one rank must stop every rank with
RMC_E_MEMORY in the same round -- no rank left waiting in a collective."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(GOLDEN, "levels.json")) as _f:
    LEVELS = json.load(_f)
with open(os.path.join(GOLDEN, "traces.json")) as _f:
    TRACES = json.load(_f)
with open(os.path.join(GOLDEN, "levels_bf.json")) as _f:
    LEVELS.update(json.load(_f))  # the BecomeFollower variant (Raft.tla:420): keys bf_*
SPEC = {False: 0, True: 1}


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(tmp_path, W, cfg, inject=None, inject_rank=None, trace=False, timeout=240):
    port = _port()
    procs, outs = [], []
    for r in range(W):
        out = str(tmp_path / f"rank{r}.json")
        spec = dict(rank=r, world=W, port=port, cfg=cfg, out=out, trace=trace,
                    inject=inject if (inject_rank is None or inject_rank == r) else None)
        # RMC_COLL_CHECK: the ranks compare every collective's sequence number, call site and size
        # first, so a rank off the common path fails with both sites named instead of hanging
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "hostx_worker.py"), json.dumps(spec)],
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                                      env=dict(os.environ, RMC_COLL_CHECK="1")))
        outs.append(out)
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=timeout)[0])
    except subprocess.TimeoutExpired:
        for p in procs:
            p.kill()
        raise AssertionError("a rank did not finish (left in a collective?)")
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    rs = [json.load(open(o)) for o in outs]
    for r, log in zip(rs, logs):
        r["_log"] = log[-2000:]
    return rs


def golden_cfg(g, **kw):
    spec = 2 if g.get("become_follower") else (1 if g["seeded"] else 0)
    return dict(n_servers=g["n"], n_vals=g["V"], max_election=g["E"], max_restart=g["R"],
                invariants=list(g["invariants"]), check_deadlock=g["check_deadlock"], spec_variant=spec, **kw)


def check(g, r):
    assert "error" not in r, r.get("error")
    assert r["status"] == {"ok": "done"}.get(g["verdict"], g["verdict"])
    assert (r["generated"], r["distinct"]) == (g["generated"], g["distinct"])
    if g["verdict"] == "ok":
        assert r["depth"] == g["depth"] and r["queue"] == 0
        assert [lv[3] for lv in r["levels"] if lv[3]] == g["levels"]
        assert [lv[2] for lv in r["levels"][1:]] == g["gen_per_level"]
    else:
        assert r["trace_len"] == g["trace_len"] and r["queue"] == g["queue_left"]
        if g["verdict"] == "invariant":
            assert r["violated"] == g["violated"]


@pytest.mark.parametrize("W,shard_min", [(2, 1), (2, 40), (3, 1)])
@pytest.mark.parametrize("name", ["n3_v1_e2_r3", "seeded_n3_v2_e2_r3", "deadlock_n3_v1_e1_r3", "n4_v1_e1_r3",
                                  "exist_lc_n3_v1_e2_r3", "bf_n4_v1_e1_r3"])
def test_ranks_identical_to_single(name, W, shard_min, tmp_path):
    """Golden levels, counters and counterexample at W ranks; every rank reports the same run."""
    g = LEVELS[name]
    rs = run_ranks(tmp_path, W, golden_cfg(g, chunk_successors=3000, shard_min_states=shard_min),
                   trace=name in TRACES)
    errs = [r.get("error") for r in rs]
    assert not any(errs), "\n".join(f"rank {i}: {e}\n{r['_log']}" for i, (e, r) in enumerate(zip(errs, rs)))
    got = [[lv[3] for lv in r["levels"] if lv[3]] for r in rs]
    if g["verdict"] == "ok":  # the first level that differs, on every rank (before the totals)
        for i, lv in enumerate(got):
            bad = next((k for k, (a, b) in enumerate(zip(lv, g["levels"])) if a != b), None)
            assert bad is None and len(lv) == len(g["levels"]), \
                f"rank {i}: level {bad}: {lv[bad - 1:bad + 2] if bad else lv[-3:]} vs golden " \
                f"{g['levels'][bad - 1:bad + 2] if bad else g['levels'][-3:]}; all ranks: {got}"
    for r in rs:
        check(g, r)
        assert r["levels"] == rs[0]["levels"]
    if name in TRACES:
        exp = [[e["key"], e["state"]] for e in TRACES[name]["steps"]]
        for r in rs:
            assert r["trace"] == exp


@pytest.mark.parametrize("site", [1, 2, 3, 4, 6, 7])
def test_ranks_agree_on_allocation_failure(site, tmp_path):
    """The allocation at `site` fails on rank 1 only, in round 1 of level 14 of configs[1]: both
    processes must raise RMC_E_MEMORY (none left in a collective), within the test timeout."""
    g = LEVELS["n3_v1_e2_r3"]
    cfg = golden_cfg(g, chunk_successors=3000, shard_min_states=1)
    rs = run_ranks(tmp_path, 2, cfg, inject=f"{site},1,1,14", inject_rank=1, timeout=180)
    for r in rs:
        assert "error" in r and "RMC_E_MEMORY" in r["error"], (site, r)
    assert "injected" in rs[1]["error"]
