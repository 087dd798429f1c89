"""GPU parity tests: the HIP path (through the C-ABI) against the oracle fixtures.

Bit-exact bar: identical successor lists (TLC order, keys and concrete states), identical
symmetry classes, identical invariant values, identical per-level distinct/generated
counts, depth, verdict and counterexample traces (tests/golden/, from oracle/)."""
import dataclasses
import functools
import gzip
import json
import os

import pytest

import raft_ref as R
import raftmc
from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


LEVELS = load("levels.json")
LEVELS_BIG = load("levels_big.json") if os.path.exists(os.path.join(GOLDEN, "levels_big.json")) else {}
PREFIX = load("levels_prefix.json") if os.path.exists(os.path.join(GOLDEN, "levels_prefix.json")) else {}
SAMPLES = load("successors.json")
TRACES = load("traces.json")
# the BecomeFollower variant (Raft.tla:420 uncommented; tests/golden/make_golden_bf.py)
LEVELS_BF = load("levels_bf.json")
SAMPLES_BF = load("successors_bf.json")
TRACES_BF = load("traces_bf.json")
# the test variants in which the Assert / the evaluation error are reachable in a BFS
# (tools/make_seeded_spec.py --split-brain / --commit-past-log; tests/golden/make_golden_errors.py)
LEVELS_ERR = load("levels_errors.json")
TRACES_ERR = load("traces_errors.json")

_cache = {}


def checker(n, V, E, Rr, **kw):
    key = (n, V, E, Rr, tuple(sorted(kw.items())))
    if key not in _cache:
        _cache[key] = raftmc.ModelChecker(raftmc.ModelConfig(n_servers=n, n_vals=V, max_election=E,
                                                             max_restart=Rr, **kw))
    return _cache[key]


@pytest.mark.parametrize("name", sorted(SAMPLES))
def test_successors_match_oracle(name):
    g = SAMPLES[name]
    mc = checker(g["n"], g["V"], g["E"], g["R"])
    for it in g["items"]:
        got = mc.successors(it["state"])
        exp = it["successors"]
        assert [list(k) for k, _, _ in got] == [e["key"] for e in exp]
        for (k, st, _), e in zip(got, exp):
            assert st == e["state"], (k, it["state"])


@pytest.mark.parametrize("name", sorted(SAMPLES))
def test_fingerprint_classes_match_oracle(name):
    g = SAMPLES[name]
    mc = checker(g["n"], g["V"], g["E"], g["R"])
    fp_of_canon = {}
    canon_of_fp = {}
    for it in g["items"]:
        assert mc.fingerprint(it["state"]) == mc.fingerprint(it["permuted"])
        for (k, st, fp), e in zip(mc.successors(it["state"]), it["successors"]):
            assert mc.fingerprint(st) == fp
            c = e["canon"]
            assert fp_of_canon.setdefault(c, fp) == fp
            assert canon_of_fp.setdefault(fp, c) == c


@pytest.mark.parametrize("name", sorted(SAMPLES))
def test_invariants_match_oracle(name):
    g = SAMPLES[name]
    cfg = R.Config(n=g["n"], V=g["V"], max_election=g["E"], max_restart=g["R"])
    mc = checker(g["n"], g["V"], g["E"], g["R"])
    names = ["Inv", "NoSplitVote", "RaftCanCommt", "FollowerCanCommit", "CommitAll", "NoAllCommit",
             "ExistLeaderAndCandidate"]
    for it in g["items"]:
        for sc in [it] + it["successors"][:4]:
            st = R.state_from_json(sc["state"])
            for nm in names:
                try:
                    exp = R.INV_FUNCS[nm](cfg, st)
                except R.EvalError:
                    exp = None
                assert mc.eval_invariant(sc["state"], nm) == exp, nm


# Deep states (tests/golden/make_golden_deep.py): guided walks from Init to depth 60-86 -- Raft.cfg
# states with up to 41 messages, configs[3] up to 63 -- plus synthetic states past them, up to the
# layout's message cap (64 at 3 servers; 122-126 at 4-5 servers: the second message round, MR = 2).
with gzip.open(os.path.join(GOLDEN, "successors_deep.json.gz"), "rt") as _f:
    DEEP = json.load(_f)
INV_NAMES = ["Inv", "NoSplitVote", "RaftCanCommt", "FollowerCanCommit", "CommitAll", "NoAllCommit",
             "ExistLeaderAndCandidate"]


@pytest.mark.parametrize("name", sorted(DEEP))
def test_deep_successors_match_oracle(name):
    """Successor lists (TLC order, keys and concrete states) of message-heavy states, and the Assert
    (tla:185) exactly where both oracles raise it."""
    g = DEEP[name]
    mc = checker(g["n"], g["V"], g["E"], g["R"])
    n_assert = 0
    for it in g["items"]:
        if it["assert_fails"]:
            with pytest.raises(AssertionError, match="split brain"):
                mc.successors(it["state"])
            n_assert += 1
            continue
        got = mc.successors(it["state"])
        exp = it["successors"]
        assert [list(k) for k, _, _ in got] == [e["key"] for e in exp], it["nmsgs"]
        for (k, st, _), e in zip(got, exp):
            assert st == e["state"], (k, it["nmsgs"])
    assert n_assert == g["coverage"]["assert_states"]


@pytest.mark.parametrize("name", sorted(DEEP))
def test_deep_fingerprint_classes_match_oracle(name):
    """The 128-bit symmetry fingerprint induces the oracles' exact canonical partition on every
    successor of the deep states (and a permuted copy has its state's fingerprint)."""
    g = DEEP[name]
    mc = checker(g["n"], g["V"], g["E"], g["R"])
    fp_of_canon, canon_of_fp = {}, {}
    for it in g["items"]:
        if it["assert_fails"]:
            continue
        assert mc.fingerprint(it["state"]) == mc.fingerprint(it["permuted"])
        for (k, st, fp), e in zip(mc.successors(it["state"]), it["successors"]):
            assert mc.fingerprint(st) == fp
            assert fp_of_canon.setdefault(e["canon"], fp) == fp
            assert canon_of_fp.setdefault(fp, e["canon"]) == e["canon"]
    assert len(fp_of_canon) == len({e["canon"] for it in g["items"] for e in it.get("successors", [])})


@pytest.mark.parametrize("name", sorted(DEEP))
def test_deep_invariants_match_oracle(name):
    """Every invariant (tla:434-499; None = TLC evaluation error) on the deep states and their first
    successors, as both oracles evaluate them."""
    g = DEEP[name]
    mc = checker(g["n"], g["V"], g["E"], g["R"])
    for it in g["items"]:
        if it["assert_fails"]:
            continue
        for tag, vals in it["invariants"].items():
            st = it["state"] if tag == "state" else it["successors"][int(tag[4:])]["state"]
            assert [mc.eval_invariant(st, nm) for nm in INV_NAMES] == vals, (tag, it["nmsgs"])


def _no_all_commit_state(msgs):
    """n3 V1: s1 leads at term 1 with commitIndex 2, s2 committed, s3 not yet (tla:451-466)."""
    e = (1, 0)
    return R.State(votedFor=(0, 0, 0), currentTerm=(1, 1, 1), logs=(((0, -1), e),) * 3,
                   matchIndex=((2, 2, 2), (1, 1, 1), (1, 1, 1)), nextIndex=((3, 3, 3), (2, 2, 2), (2, 2, 2)),
                   commitIndex=(2, 2, 1), msgs=frozenset(msgs), role=(R.LEADER, R.FOLLOWER, R.FOLLOWER),
                   electionCount=1, restartCount=0, pendingResponse=((False,) * 3,) * 3, valSent=(0,))


def test_no_all_commit_reads_msgs():
    """NoAllCommit (tla:451-481), the one invariant over msgs: TRUE with its three messages,
    FALSE as soon as any one is missing or differs in a field the formula tests."""
    cfg = R.Config(n=3, V=1, max_election=2, max_restart=3)
    mc = checker(3, 1, 2, 3)
    req1 = R.append_req(0, 2, 1, 1, 0, ((1, 0),), 1)
    resp1 = R.append_resp(2, 0, 1, 1, True)
    req2 = R.append_req(0, 2, 1, 2, 1, (), 2)
    noise = [R.append_req(0, 1, 1, 1, 0, ((1, 0),), 1), R.append_resp(1, 0, 1, 2, True)]
    cases = [
        [req1, resp1, req2], [req1, resp1, req2] + noise, [resp1, req2], [req1, req2], [req1, resp1],
        [R.append_req(0, 2, 2, 1, 0, ((1, 0),), 1), resp1, req2],   # term # currentTerm[s3]
        [req1, R.append_resp(2, 0, 1, 1, False), req2],               # succ FALSE
        [req1, R.append_resp(1, 0, 1, 1, True), req2],                # wrong src
        [req1, resp1, R.append_req(0, 1, 1, 2, 1, (), 2)],            # wrong dst
    ]
    seen = set()
    for msgs in cases:
        st = _no_all_commit_state(msgs)
        exp = R.INV_FUNCS["NoAllCommit"](cfg, st)
        seen.add(exp)
        assert mc.eval_invariant(R.state_to_json(st), "NoAllCommit") == exp, msgs
    assert seen == {True, False}
    # the state conjuncts: commitIndex of s3 must be 1
    st = dataclasses.replace(_no_all_commit_state([req1, resp1, req2]), commitIndex=(2, 2, 2))
    assert R.INV_FUNCS["NoAllCommit"](cfg, st) is False
    assert mc.eval_invariant(R.state_to_json(st), "NoAllCommit") is False


def test_no_all_commit_run_matches_oracle():
    """INVARIANT NoAllCommit: FALSE at Init, so TLC stops there with a 1-state trace."""
    cfg = R.Config(n=3, V=1, max_election=1, max_restart=3, invariants=("NoAllCommit",))
    p = R.bfs(cfg)
    mc = raftmc.ModelChecker(raftmc.ModelConfig(n_servers=3, n_vals=1, max_election=1, max_restart=3,
                                                invariants=("NoAllCommit",)))
    res = mc.run()
    assert (res.status, res.generated, res.distinct) == (p.verdict, p.generated, p.distinct)
    assert res.violated == p.violated == "NoAllCommit"
    assert res.trace_len == len(p.trace) == 1
    mc.close()


@pytest.mark.parametrize("order", [("NoAllCommit", "RaftCanCommt"), ("RaftCanCommt", "NoAllCommit"),
                                   ("Inv", "CommitAll", "RaftCanCommt")])
def test_invariants_checked_in_cfg_order(order):
    """Both invariants are FALSE at Init: TLC reports the one the cfg lists first (Raft.cfg:33-34),
    as the oracle does -- not the lower invariant bit."""
    cfg = R.Config(n=3, V=1, max_election=1, max_restart=3, invariants=order)
    p = R.bfs(cfg)
    with raftmc.ModelChecker(raftmc.ModelConfig(n_servers=3, n_vals=1, max_election=1, max_restart=3,
                                                invariants=order)) as mc:
        res = mc.run()
    assert res.status == p.verdict == "invariant"
    assert res.violated == p.violated == [i for i in order if i != "Inv"][0]


def test_eval_error_state():
    mc = checker(3, 2, 3, 3)
    s = R.state_to_json(R.State((-1, -1, -1), (1, 1, 1), (((0, -1), (1, 0), (1, 1)), ((0, -1), (1, 0)), ((0, -1),)),
                                ((1, 1, 1),) * 3, ((2, 2, 2),) * 3, (1, 3, 1), frozenset(), (2, 0, 0), 0, 0,
                                ((False,) * 3,) * 3, (0, 0)))
    assert mc.eval_invariant(s, "Inv") is None


def spec_of(g):
    if g.get("become_follower"):
        return raftmc.SPEC_BECOME_FOLLOWER
    if g.get("variant"):
        return {"split_brain": raftmc.SPEC_SPLIT_BRAIN, "commit_past_log": raftmc.SPEC_COMMIT_PAST_LOG}[g["variant"]]
    return raftmc.SPEC_SEEDED if g["seeded"] else raftmc.SPEC_RAFT


def run_cfg(g, **kw):
    mc = raftmc.ModelChecker(raftmc.ModelConfig(
        n_servers=g["n"], n_vals=g["V"], max_election=g["E"], max_restart=g["R"],
        invariants=tuple(g["invariants"]), check_deadlock=g["check_deadlock"],
        spec_variant=spec_of(g), **kw))
    res = mc.run()
    return mc, res


def check_levels(g, res):
    assert res.status == {"ok": "done"}.get(g["verdict"], g["verdict"])
    assert res.generated == g["generated"] and res.distinct == g["distinct"]
    if g["verdict"] == "ok":
        assert res.depth == g["depth"]
        assert [ls.new_states for ls in res.levels if ls.new_states] == g["levels"]
        assert [ls.generated for ls in res.levels[1:]] == g["gen_per_level"]
        assert res.queue == 0
    else:
        assert res.trace_len == g["trace_len"]
        assert res.queue == g["queue_left"]
        if g["verdict"] == "invariant":
            assert res.violated == g["violated"]


@pytest.mark.parametrize("name", sorted(LEVELS))
def test_bfs_matches_golden_levels(name):
    g = LEVELS[name]
    mc, res = run_cfg(g)
    check_levels(g, res)
    mc.close()


@pytest.mark.parametrize("name", sorted(LEVELS))
def test_split_probe_chunks_match_golden_levels(name, monkeypatch):
    """Every chunk split (RMC_SPLIT_MIN=1, host-driven levels): k_probe elects, k_insert_winners inserts
    and leaves its verdicts for the commit -- levels, counters at an error and traces as the golden run."""
    monkeypatch.setenv("RMC_SPLIT_MIN", "1")
    g = LEVELS[name]
    mc, res = run_cfg(g, device_levels=1)
    check_levels(g, res)
    if name in TRACES:
        assert [(list(k) if k else None, st) for k, st in mc.trace()] == \
               [(e["key"], e["state"]) for e in TRACES[name]["steps"]]
    mc.close()


@pytest.mark.parametrize("mode", ["virtual2", "rccl1", "virtual3_rebid"])
@pytest.mark.parametrize("name", sorted(LEVELS))
def test_sharded_commit_list_matches_golden_levels(name, mode, monkeypatch):
    """Split sharded rounds (RMC_SPLIT_MIN=1 makes every round one): the fingerprint pass bids each
    shard's own successors in its election table, the commit visits only the parents with winners
    (k_nzlist) -- levels, counters at an error and traces as the golden run.  virtual3_rebid: the
    bids are always redone in the owner table (RMC_OWNER_LXY=2, the fallback for received items
    that do not fit beside them)."""
    monkeypatch.setenv("RMC_SPLIT_MIN", "1")
    g = LEVELS[name]
    if mode == "virtual3_rebid":
        monkeypatch.setenv("RMC_OWNER_LXY", "2")
        kw = dict(virtual_shards=3, chunk_successors=3000, shard_min_states=1)
    elif mode == "virtual2":
        kw = dict(virtual_shards=2, chunk_successors=3000, shard_min_states=1)
    else:
        kw = dict(world_size=1, rank=0, comm_unique_id=raftmc.comm_unique_id(), chunk_successors=3000,
                  shard_min_states=1)
    mc, res = run_cfg(g, **kw)
    check_levels(g, res)
    if name in TRACES:
        assert [(list(k) if k else None, st) for k, st in mc.trace()] == \
               [(e["key"], e["state"]) for e in TRACES[name]["steps"]]
    mc.close()


@pytest.mark.parametrize("mode", ["virtual2", "rccl1"])
@pytest.mark.parametrize("name", ["n3_v1_e2_r3", "seeded_n3_v2_e2_r3", "n4_v1_e1_r3"])
def test_sharded_run_then_reset_reruns_golden(name, mode, monkeypatch):
    """A sharded run whose split rounds used the fused election table (ET) as their owner table,
    then rmc_reset, then a second run whose first levels are replicated (the fused election again):
    both runs give the golden levels, counters and traces (the owner keys a sharded round leaves in L
    are smaller than any fused election word; reset must clear them)."""
    if name not in LEVELS:
        pytest.skip("no such golden configuration")
    monkeypatch.setenv("RMC_SPLIT_MIN", "1")
    g = LEVELS[name]
    if mode == "virtual2":
        kw = dict(virtual_shards=2, chunk_successors=3000, shard_min_states=40)
    else:
        kw = dict(world_size=1, rank=0, comm_unique_id=raftmc.comm_unique_id(), chunk_successors=3000,
                  shard_min_states=40)
    mc, res = run_cfg(g, **kw)
    check_levels(g, res)
    for _ in range(2):
        mc.reset()
        res = mc.run()
        check_levels(g, res)
        if name in TRACES:
            assert [(list(k) if k else None, st) for k, st in mc.trace()] == \
                   [(e["key"], e["state"]) for e in TRACES[name]["steps"]]
    mc.close()


@pytest.mark.parametrize("name", sorted(LEVELS_BIG))
def test_bfs_matches_golden_levels_at_scale(name):
    """bench.py's at-scale workload (10^7 states) against the C oracle's full BFS, level by level."""
    g = LEVELS_BIG[name]
    mc, res = run_cfg(g)
    check_levels(g, res)
    mc.close()


# Raft.cfg as shipped (Raft.cfg:1-34 under myrun.sh:3): the exhaustion recorded on MI355X
# (profiles/r02_explore_raftcfg_levels.txt, profiles/r02_myrun_raftcfg_raft.txt).  Beyond the C
# oracle's prefix these totals are this checker's own (TLC cannot run here: parity unpinned).
RAFT_CFG_TOTALS = dict(distinct=10946499503, generated=56936653204, depth=72)


def test_raft_cfg_exhausted_and_prefix_matches_c_oracle():
    """configs[0]/[2]: Raft.cfg as shipped (3 servers, 2 values, MaxElection 3, MaxRestart 3) exhausted
    on one GPU -- the large-run storage (compact seen set, frontier ring, host trace) end to end.  The
    first 34 levels (743.6 M states, 2.47 G generated; oracle/raft_prefix.c) equal the C oracle's level
    by level, distinct and generated."""
    g = PREFIX["n3_v2_e3_r3"]
    for mc in _cache.values():  # the run takes most of the device's memory
        mc.close()
    _cache.clear()
    with raftmc.ModelChecker(raftmc.ModelConfig(n_servers=3, n_vals=2, max_election=3, max_restart=3)) as mc:
        res = mc.run()
    got = [ls.new_states for ls in res.levels]
    assert got[:len(g["levels"])] == g["levels"]
    assert [ls.generated for ls in res.levels[1:len(g["gen_per_level"]) + 1]] == g["gen_per_level"]
    assert res.status == "done" and res.queue == 0
    assert (res.distinct, res.generated, res.depth) == (RAFT_CFG_TOTALS["distinct"], RAFT_CFG_TOTALS["generated"],
                                                        RAFT_CFG_TOTALS["depth"])
    assert res.seen_slot_bytes == 8


@pytest.mark.skipif("n5_v1_e3_r3" not in PREFIX, reason="no configs[3] prefix fixture")
def test_configs3_prefix_matches_c_oracle():
    """configs[3] (5 servers, 1 value, MaxElection 3, MaxRestart 3; Raft.cfg:16-18 with s4, s5 in
    Servers): the levels the C oracle completes (tests/golden/make_golden_prefix.py --mt, exact
    canonical forms over all 120 permutations) equal the GPU's level by level -- the signature
    pre-sort symmetry minimum against the exact orbit count."""
    g = PREFIX["n5_v1_e3_r3"]
    for mc in _cache.values():
        mc.close()
    _cache.clear()
    with raftmc.ModelChecker(raftmc.ModelConfig(n_servers=5, n_vals=1, max_election=3, max_restart=3)) as mc:
        mc.init()
        while len(mc.levels) < len(g["levels"]) + 1:
            mc.step()
        got = [ls.new_states for ls in mc.levels]
        assert got[:len(g["levels"])] == g["levels"]
        assert [ls.generated for ls in mc.levels[1:len(g["gen_per_level"]) + 1]] == g["gen_per_level"]


@pytest.mark.parametrize("name", sorted(TRACES))
def test_counterexample_trace_matches_oracle(name):
    g = LEVELS[name]
    t = TRACES[name]
    mc, res = run_cfg(g)
    tr = mc.trace()
    assert len(tr) == len(t["steps"])
    for (key, st), e in zip(tr, t["steps"]):
        assert (list(key) if key else None) == e["key"]
        assert st == e["state"]
    mc.close()


def test_results_independent_of_chunking_and_seen_growth():
    """Chunk boundaries and seen-set rehashing must not change TLC's discovery order."""
    g = LEVELS["n3_v1_e2_r3"]
    for kw in (dict(chunk_successors=6000, seen_log2=10), dict(chunk_successors=40000, seen_log2=12)):
        mc, res = run_cfg(g, **kw)
        check_levels(g, res)
        mc.close()


@pytest.mark.parametrize("device_levels", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("name", sorted(LEVELS))
def test_device_level_loop_matches_golden(name, device_levels):
    """Host-driven levels (1) and device-driven batches of 2 / 3 levels (odd and even
    frontier-buffer swaps, a batch boundary every few levels) give TLC's results."""
    g = LEVELS[name]
    mc, res = run_cfg(g, device_levels=device_levels)
    check_levels(g, res)
    if name in TRACES:
        tr = mc.trace()
        assert [st for _, st in tr] == [e["state"] for e in TRACES[name]["steps"]]
    mc.close()


def test_steps_api_batches_levels():
    """rmc_steps hands back several levels per host round trip on one GPU, and the
    per-level statistics equal the host-driven ones."""
    g = LEVELS["n3_v1_e2_r3"]
    mk = lambda **kw: raftmc.ModelChecker(raftmc.ModelConfig(n_servers=3, n_vals=1, max_election=2, max_restart=3,
                                                             **kw))
    a, b = mk(), mk(device_levels=1)
    a.init(); b.init()
    la, calls = [], 0
    while True:
        got = a.steps()
        calls += 1
        la += got
        if got[-1].status != "ok":
            break
    lb = [b.step() for _ in range(len(la))]
    assert calls < len(la)
    assert [(x.level, x.expanded, x.generated, x.new_states, x.queue) for x in la] == \
           [(x.level, x.expanded, x.generated, x.new_states, x.queue) for x in lb]
    assert a.result().distinct == g["distinct"]
    a.close(); b.close()


# ---- large-run storage: compact seen set, frontier ring at a fixed budget --------------------
LARGE_MODE = ["n3_v1_e2_r3", "n3_v2_e1_r3", "n4_v1_e1_r3", "n5_v1_e1_r3", "n3_v3_e1_r3", "seeded_n3_v2_e2_r3",
              "deadlock_n3_v1_e1_r3", "nosplit_n3_v1_e2_r3", "seeded_n3_v1_e2_r3"]


@pytest.mark.parametrize("device_levels", [0, 1])
@pytest.mark.parametrize("name", LARGE_MODE)
def test_compact_seen_set_and_fixed_ring_match_golden(name, device_levels):
    """The storage a large run switches to -- 8-B seen-set slots (migrated from the 16-B table after
    2^10 slots, sized to the run) and a frontier ring pinned at ~60 % of the live frontier's peak,
    so that the next level reuses the space of chunks already expanded and wraps around the ring --
    gives TLC's results: per-level counts, depth, verdict, queue and the counterexample."""
    g = LEVELS[name]
    probe, res0 = run_cfg(g, chunk_successors=6000, device_levels=1)
    peak = res0.frontier_peak_bytes
    probe.close()
    slots = 1 << max(12, (int(g["distinct"] / 0.6)).bit_length())
    ring = int(0.6 * peak) + 4 * 6000 * 36 + 4096
    mc, res = run_cfg(g, chunk_successors=6000, device_levels=device_levels, compact_log2=10, seen_log2=8,
                      seen_mem_bytes=8 * slots, frontier_mem_bytes=ring)
    check_levels(g, res)
    if g["distinct"] > 2048:  # the run outgrew the 2^10-slot full table
        assert res.seen_slot_bytes == 8 and res.seen_slots == slots
        assert res.frontier_ring_bytes <= max(ring, 4 * 6000 * 36 * 2)
    if name in TRACES:
        tr = mc.trace()
        assert [st for _, st in tr] == [e["state"] for e in TRACES[name]["steps"]]
    mc.close()


def test_compact_seen_set_at_scale():
    """bench's at-scale configuration (18.5M states) on the compact seen set and a ring at ~60 % of
    its peak frontier: the C oracle's per-level counts."""
    g = LEVELS_BIG["n3_v2_e2_r3"]
    mc, res = run_cfg(g, compact_log2=20, seen_log2=12, seen_mem_bytes=8 << 25, frontier_mem_bytes=600 << 20)
    check_levels(g, res)
    assert res.seen_slot_bytes == 8
    mc.close()


def test_seeded_trace_independent_of_chunking():
    g = LEVELS["seeded_n3_v1_e2_r3"]
    mc, res = run_cfg(g, chunk_successors=6000, seen_log2=10)
    check_levels(g, res)
    mc.close()


# ---- sharded BFS, run as virtual shards on one GPU -------------------------------
# Block-cyclic levels, fingerprint-owner election by global key (rmc_engine.hip step_sharded): the
# level order is TLC's at any shard count, so every golden config -- invariant, deadlock and
# seeded runs included -- must give W = 1's per-level sizes, counters at the error, queue and
# counterexample.  Small rounds (chunk_successors) make many rounds per level, blocks of a few
# dozen parents, and winners of one shard spread over several owners (the grouped exchange).
@pytest.mark.parametrize("shard_min", [1, 40])
@pytest.mark.parametrize("shards", [2, 4, 8])
@pytest.mark.parametrize("name", sorted(LEVELS))
def test_sharded_bfs_identical_to_one_shard(name, shards, shard_min):
    """Sharded from Init (shard_min 1), or replicated until a level reaches 40 states and sharded after."""
    g = LEVELS[name]
    mc, res = run_cfg(g, virtual_shards=shards, chunk_successors=3000, shard_min_states=shard_min)
    check_levels(g, res)
    if name in TRACES:
        tr = mc.trace()
        assert len(tr) == len(TRACES[name]["steps"])
        for (key, st), e in zip(tr, TRACES[name]["steps"]):
            assert (list(key) if key else None) == e["key"]
            assert st == e["state"]
    mc.close()


@pytest.mark.parametrize("clear_rounds", ["1", "2", "5"])
@pytest.mark.parametrize("name", ["n3_v1_e2_r3", "seeded_n3_v2_e2_r3", "n4_v1_e1_r3"])
def test_sharded_owner_table_tags_across_clears(name, clear_rounds, monkeypatch):
    """The owner's election table is cleared only every RMC_OT_CLEAR_ROUNDS rounds (owner_table): slots
    and keys of earlier rounds must read as free / larger however many rounds lie between clears."""
    monkeypatch.setenv("RMC_OT_CLEAR_ROUNDS", clear_rounds)
    g = LEVELS[name]
    mc, res = run_cfg(g, virtual_shards=4, chunk_successors=3000, shard_min_states=1)
    check_levels(g, res)
    mc.close()


# The same protocol through the RCCL transport: world_size 1 with a unique id is a one-rank
# communicator, so every collective of step_sharded (all-reduce of the level size, the gathered
# count matrices, the round's failure table) runs through RCCL on the stream.  A rank's part for
# itself is a device copy (its successor items placed in the receive buffer directly); with
# RMC_SELF_VIA_RCCL=1 it goes through the grouped ncclSend/ncclRecv of successors, verdicts and
# winner records like any peer's.  A one-GPU box cannot hold two ranks (RCCL refuses two ranks on
# one device); this is the RCCL code path short of the xGMI hop.
@pytest.mark.parametrize("self_rccl", ["0", "1"])
@pytest.mark.parametrize("shard_min", [1, 40])
@pytest.mark.parametrize("name", ["n3_v1_e2_r3", "n4_v1_e1_r3", "seeded_n3_v2_e2_r3", "deadlock_n3_v1_e1_r3",
                                  "n2_v2_e3_r3", "exist_lc_n3_v1_e2_r3"])
def test_rccl_one_rank_identical_to_single(name, shard_min, self_rccl, monkeypatch):
    monkeypatch.setenv("RMC_SELF_VIA_RCCL", self_rccl)
    g = LEVELS[name]
    mc, res = run_cfg(g, world_size=1, rank=0, comm_unique_id=raftmc.comm_unique_id(), chunk_successors=3000,
                      shard_min_states=shard_min)
    check_levels(g, res)
    if name in TRACES:
        assert [(list(k) if k else None, st) for k, st in mc.trace()] == \
               [(e["key"], e["state"]) for e in TRACES[name]["steps"]]
    mc.close()


@pytest.mark.parametrize("shards", [2, 3, 8])
@pytest.mark.parametrize("name", ["seeded_n3_v2_e2_r3", "deadlock_n3_v1_e1_r3", "n3_v2_e1_r3"])
def test_sharded_level_stats_equal_single(name, shards):
    """Every level's statistics (expanded, generated, new states, queue, running totals) at W shards
    equal the single-GPU run's, up to and including the level of the error."""
    g = LEVELS[name]
    one, r1 = run_cfg(g, device_levels=1)
    many, rw = run_cfg(g, virtual_shards=shards, chunk_successors=3000, shard_min_states=1)
    key = lambda ls: (ls.level, ls.expanded, ls.generated, ls.new_states, ls.queue, ls.total_generated,
                      ls.total_distinct, ls.status, ls.self_loops)
    assert [key(x) for x in rw.levels] == [key(x) for x in r1.levels]
    assert (rw.status, rw.distinct, rw.generated, rw.queue, rw.depth) == (r1.status, r1.distinct, r1.generated,
                                                                          r1.queue, r1.depth)
    assert many.trace() == one.trace()
    one.close()
    many.close()


# ---- checkpoint / resume (TLC's states/ metadir + -recover) ----------
@pytest.mark.parametrize("name", ["n3_v1_e2_r3", "n3_v2_e1_r3", "seeded_n3_v1_e2_r3", "deadlock_n3_v1_e1_r3"])
def test_checkpoint_resume_matches_uninterrupted(name, tmp_path):
    """Stop after a few levels, checkpoint, and finish the run twice: in the same checker and in
    a fresh one resumed from the file.  Both must give the golden counts, the golden per-level
    sizes of the remaining levels and the identical counterexample."""
    g = LEVELS[name]
    cfg = dict(n_servers=g["n"], n_vals=g["V"], max_election=g["E"], max_restart=g["R"],
               invariants=tuple(g["invariants"]), check_deadlock=g["check_deadlock"],
               spec_variant=raftmc.SPEC_SEEDED if g["seeded"] else raftmc.SPEC_RAFT)
    path = str(tmp_path / "run.ckpt")
    a = raftmc.ModelChecker(raftmc.ModelConfig(**cfg))
    a.init()
    k = 0
    while k < 6 and a.step().status == "ok":
        k += 1
    assert k == 6, "the configuration must run past the checkpoint level"
    a.checkpoint(path)
    done = len(a.levels)
    res_a = a.run()
    b = raftmc.ModelChecker(raftmc.ModelConfig(**cfg))
    b.resume(path)
    res_b = b.run()
    check_levels(g, res_a)
    for f in ("status", "generated", "distinct", "depth", "queue", "violated", "trace_len"):
        assert getattr(res_b, f) == getattr(res_a, f), f
    assert [ls.new_states for ls in res_b.levels] == [ls.new_states for ls in res_a.levels[done:]]
    assert b.trace() == a.trace()
    a.close()
    b.close()


@pytest.mark.parametrize("mode", ["virtual2", "virtual4", "rccl1"])
@pytest.mark.parametrize("name,shard_min", [("n3_v1_e2_r3", 1), ("seeded_n3_v2_e2_r3", 40),
                                            ("deadlock_n3_v1_e1_r3", 1), ("n4_v1_e1_r3", 40)])
def test_sharded_checkpoint_resume_matches_uninterrupted(name, shard_min, mode, tmp_path):
    """Checkpoint of a sharded run (virtual shards, or the RCCL transport on a one-rank
    communicator) after six levels -- sharded from Init, or still replicated / just sharded with
    shard_min 40 -- resumed in a fresh checker with the same layout: the golden counts, the
    remaining levels and the counterexample of the uninterrupted run."""
    g = LEVELS[name]
    cfg = dict(n_servers=g["n"], n_vals=g["V"], max_election=g["E"], max_restart=g["R"],
               invariants=tuple(g["invariants"]), check_deadlock=g["check_deadlock"],
               spec_variant=raftmc.SPEC_SEEDED if g["seeded"] else raftmc.SPEC_RAFT,
               chunk_successors=3000, shard_min_states=shard_min)
    if mode.startswith("virtual"):
        cfg["virtual_shards"] = int(mode[7:])
    path = str(tmp_path / "run.ckpt")

    def make():
        extra = dict(world_size=1, rank=0, comm_unique_id=raftmc.comm_unique_id()) if mode == "rccl1" else {}
        return raftmc.ModelChecker(raftmc.ModelConfig(**cfg, **extra))

    a = make()
    a.init()
    k = 0
    while k < 6 and a.step().status == "ok":
        k += 1
    assert k == 6, "the configuration must run past the checkpoint level"
    a.checkpoint(path)
    done = len(a.levels)
    res_a = a.run()
    b = make()
    b.resume(path)
    res_b = b.run()
    check_levels(g, res_a)
    for f in ("status", "generated", "distinct", "depth", "queue", "violated", "trace_len"):
        assert getattr(res_b, f) == getattr(res_a, f), f
    assert [ls.new_states for ls in res_b.levels] == [ls.new_states for ls in res_a.levels[done:]]
    assert b.trace() == a.trace()
    a.close()
    b.close()


def test_sharded_checkpoint_resume_at_scale(tmp_path):
    """18.5 M states over 2 virtual shards, sharded from the first level of 2^20 states, compact
    seen-set shards and rings at their budget: checkpointed after 30 levels (sharded by then),
    resumed in a fresh checker, finished with the C oracle's counts."""
    g = LEVELS_BIG["n3_v2_e2_r3"]
    cfg = raftmc.ModelConfig(n_servers=3, n_vals=2, max_election=2, max_restart=3, virtual_shards=2,
                             compact_log2=20, seen_log2=12, seen_mem_bytes=8 << 25, frontier_mem_bytes=1 << 30)
    path = str(tmp_path / "big.ckpt")
    with raftmc.ModelChecker(cfg) as a:
        a.init()
        while len(a.levels) < 31:
            assert a.step().status == "ok"
        assert max(ls.expanded for ls in a.levels) >= 1 << 20, "the run must be sharded at the checkpoint"
        a.checkpoint(path)
        done = len(a.levels)
    with raftmc.ModelChecker(cfg) as b:
        b.resume(path)
        res = b.run()
    assert (res.status, res.distinct, res.generated, res.depth) == ("done", g["distinct"], g["generated"], g["depth"])
    assert [ls.new_states for ls in res.levels if ls.new_states] == g["levels"][done:]
    assert [ls.generated for ls in res.levels] == g["gen_per_level"][done - 1:]
    assert res.seen_slot_bytes == 8


def test_sharded_resume_rejects_another_layout(tmp_path):
    path = str(tmp_path / "run.ckpt")
    base = dict(n_servers=3, n_vals=1, max_election=2, max_restart=3, chunk_successors=3000, shard_min_states=1)
    with raftmc.ModelChecker(raftmc.ModelConfig(**base, virtual_shards=2)) as a:
        a.init()
        a.step()
        a.checkpoint(path)
    with raftmc.ModelChecker(raftmc.ModelConfig(**base, virtual_shards=4)) as b:
        with pytest.raises(raftmc.RmcError, match="another shard layout"):
            b.resume(path)
    with raftmc.ModelChecker(raftmc.ModelConfig(**base)) as c:
        with pytest.raises(raftmc.RmcError, match="another shard layout"):
            c.resume(path)


def test_sharded_resume_adopts_a_smaller_stored_chunk(tmp_path):
    """A sharded checkpoint written with a smaller chunk size (chunk_successors) than the resuming context's
    is adopted -- the block-cyclic layout needs the writer's size and the larger buffers hold it -- and the
    run finishes with the golden counts; a larger stored chunk is refused, and the refusing context still
    runs from Init with its own chunk size (the adoption is undone when a resume fails)."""
    g = LEVELS["n3_v1_e2_r3"]
    small, large = str(tmp_path / "small.ckpt"), str(tmp_path / "large.ckpt")
    base = dict(n_servers=3, n_vals=1, max_election=2, max_restart=3, shard_min_states=1, virtual_shards=2)
    for path, cs in ((small, 3000), (large, 12000)):
        with raftmc.ModelChecker(raftmc.ModelConfig(**base, chunk_successors=cs)) as a:
            a.init()
            for _ in range(6):
                a.step()
            a.checkpoint(path)
    with raftmc.ModelChecker(raftmc.ModelConfig(**base, chunk_successors=6000)) as b:
        b.resume(small)
        res = b.run()
        assert (res.status, res.distinct, res.generated, res.depth) == ("done", g["distinct"], g["generated"],
                                                                        g["depth"])
        assert [ls.new_states for ls in res.levels if ls.new_states] == g["levels"][7:]
    with raftmc.ModelChecker(raftmc.ModelConfig(**base, chunk_successors=6000)) as c:
        with pytest.raises(raftmc.RmcError, match="another shard layout"):
            c.resume(large)
        check_levels(g, c.run())
    # adopted, then refused further on (a corrupt data section): the context keeps its own chunk size
    data = bytearray(open(small, "rb").read())
    data[-20] ^= 0xFF
    bad = str(tmp_path / "bad.ckpt")
    open(bad, "wb").write(bytes(data))
    with raftmc.ModelChecker(raftmc.ModelConfig(**base, chunk_successors=6000)) as d:
        with pytest.raises(raftmc.RmcError):
            d.resume(bad)
        check_levels(g, d.run())


def test_resume_rejects_another_configuration(tmp_path):
    path = str(tmp_path / "run.ckpt")
    with raftmc.ModelChecker(raftmc.ModelConfig(n_servers=3, n_vals=1, max_election=1, max_restart=3)) as a:
        a.init()
        a.step()
        a.checkpoint(path)
    with raftmc.ModelChecker(raftmc.ModelConfig(n_servers=3, n_vals=1, max_election=2, max_restart=3)) as b:
        with pytest.raises(raftmc.RmcError, match="not a checkpoint of this configuration"):
            b.resume(path)


def test_launcher_checkpoint_and_recover(tmp_path):
    """raftmc -checkpoint / -metadir / -recover (TLC's flags): a run checkpointed after its first
    batch of levels, recovered in a second process, ends with the uninterrupted run's counts."""
    import subprocess
    from test_host import LAUNCHER, cfg_text
    g = LEVELS["n3_v1_e2_r3"]
    (tmp_path / "Raft.cfg").write_text(cfg_text(E=2, R=3, vals="v1"))
    env = dict(os.environ, RMC_SKIP_SPEC_CHECK="1")
    # a small initial seen set makes the device loop hand back to the host every few levels
    base = [LAUNCHER, "-deadlock", "-seenlog2", "10", "-config", str(tmp_path / "Raft.cfg")]
    meta = str(tmp_path / "states")
    r1 = subprocess.run(base + ["-checkpoint", "0.000001", "-metadir", meta, str(tmp_path / "Raft.tla")],
                        capture_output=True, text=True, env=env, timeout=120)
    assert r1.returncode == 0, r1.stdout + r1.stderr
    assert "Checkpointing completed" in r1.stdout and os.path.exists(os.path.join(meta, "raftmc.ckpt"))
    want = f"{g['generated']} states generated, {g['distinct']} distinct states found, 0 states left on queue."
    assert want in r1.stdout
    r2 = subprocess.run(base + ["-checkpoint", "0", "-recover", meta, str(tmp_path / "Raft.tla")],
                        capture_output=True, text=True, env=env, timeout=120)
    assert r2.returncode == 0, r2.stdout + r2.stderr
    assert "Recovery completed" in r2.stdout and want in r2.stdout
    assert f"The depth of the complete state graph search is {g['depth']}." in r2.stdout


# ---- error paths and the TLC-style output ----------------------------------------------------
def _leader_with_same_term_append_req():
    """s1 leads at term 1 while s2 (also at term 1) has sent it an AppendReq: UpdateTerm(s1)'s
    second disjunct evaluates Assert(role[s1] # Leader, "split brain") (Raft.tla:183-185)."""
    req = R.append_req(1, 0, 1, 1, 0, (), 1)
    return R.State(votedFor=(0, 1, -1), currentTerm=(1, 1, 1), logs=(((0, -1),),) * 3,
                   matchIndex=((1, 1, 1),) * 3, nextIndex=((2, 2, 2),) * 3, commitIndex=(1, 1, 1),
                   msgs=frozenset([req]), role=(R.LEADER, R.LEADER, R.FOLLOWER), electionCount=2, restartCount=0,
                   pendingResponse=((False,) * 3,) * 3, valSent=(-1,))


def test_assert_split_brain_through_the_kernels():
    """The HIP expansion reports the Assert of Raft.tla:185 exactly where the oracle raises it."""
    cfg = R.Config(n=3, V=1, max_election=2, max_restart=3)
    st = _leader_with_same_term_append_req()
    with pytest.raises(R.AssertionFailure):
        R.successors(cfg, st)
    mc = checker(3, 1, 2, 3)
    with pytest.raises(AssertionError, match="split brain"):
        mc.successors(R.state_to_json(st))
    # the same message at a higher term takes UpdateTerm's first disjunct: no Assert, same successors
    st2 = dataclasses.replace(st, msgs=frozenset([R.append_req(1, 0, 2, 1, 0, (), 1)]), currentTerm=(1, 2, 1))
    exp = R.successors(cfg, st2)
    got = mc.successors(R.state_to_json(st2))
    assert [list(k) for k, _, _ in got] == [list(k) for k, _ in exp]
    assert [g[1] for g in got] == [R.state_to_json(t) for _, t in exp]


def test_eval_error_through_successor_invariants():
    """A state whose Inv evaluation leaves logs[p]'s domain (Raft.tla:499) gives the TLC evaluation
    error through the kernels' invariant code, and a leader-free state does not."""
    mc = checker(3, 2, 3, 3)
    bad = R.State((-1, -1, -1), (1, 1, 1), (((0, -1), (1, 0), (1, 1)), ((0, -1), (1, 0)), ((0, -1),)),
                  ((1, 1, 1),) * 3, ((2, 2, 2),) * 3, (1, 3, 1), frozenset(), (2, 0, 0), 0, 0,
                  ((False,) * 3,) * 3, (0, 0))
    cfg = R.Config(n=3, V=2, max_election=3, max_restart=3)
    with pytest.raises(R.EvalError):
        R.INV_FUNCS["Inv"](cfg, bad)
    assert mc.eval_invariant(R.state_to_json(bad), "Inv") is None
    ok = dataclasses.replace(bad, role=(0, 0, 0))
    assert mc.eval_invariant(R.state_to_json(ok), "Inv") is True


def test_launcher_prints_tlc_counterexample(tmp_path):
    """raftmc on the seeded spec: TLC's error line, then every State k block -- the action and all 12
    variables in TLA+ syntax -- equal to the oracle's counterexample rendered the same way."""
    import subprocess
    from test_host import LAUNCHER, cfg_text
    from tla_render import render_state
    g, t = LEVELS["seeded_n3_v1_e2_r3"], TRACES["seeded_n3_v1_e2_r3"]
    (tmp_path / "RaftSeeded.cfg").write_text(cfg_text(E=2, R=3, vals="v1"))
    env = dict(os.environ, RMC_SKIP_SPEC_CHECK="1")
    r = subprocess.run([LAUNCHER, "-deadlock", "-workers", "4", "-config", str(tmp_path / "RaftSeeded.cfg"),
                        str(tmp_path / "RaftSeeded.tla")], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 12, r.stdout + r.stderr
    out = r.stdout.splitlines()
    assert "Error: Invariant Inv is violated." in out
    assert "Error: The behavior up to this point is:" in out
    # State blocks; msgs continuation lines ("   [..]") belong to the msgs line
    blocks, cur = [], None
    for line in out:
        if line.startswith("State "):
            cur = [line]
            blocks.append(cur)
        elif cur is not None and line.startswith("/\\ "):
            cur.append(line)
        elif cur is not None and line.startswith("   ["):
            cur[-1] += " " + line.strip()
        elif cur is not None and not line.strip():
            cur = None
    assert len(blocks) == len(t["steps"]) == g["trace_len"]
    actions = raftmc.ACTIONS
    for k, (blk, step) in enumerate(zip(blocks, t["steps"])):
        if step["key"] is None:
            assert blk[0] == f"State {k + 1}: <Initial predicate>"
        else:
            srv, act, _ = step["key"]
            assert blk[0] == f"State {k + 1}: <{actions[act]}(s{srv + 1})>", blk[0]
        want = render_state(step["state"], ["s1", "s2", "s3"], ["v1"])
        assert [l.replace(",  [", ", [") for l in blk[1:]] == want, (k, blk[1:], want)
    assert f"{g['generated']} states generated, {g['distinct']} distinct states found, " \
           f"{g['queue_left']} states left on queue." in out


@pytest.mark.parametrize("spec", ["seeded", "raft_e2"])
def test_launcher_gpus_one_rank_prints_the_single_path_lines(spec, tmp_path):
    """raftmc -gpus 1 -onerank: a rank process forked by the launcher, its RCCL id handed down a pipe,
    the sharded protocol through a one-rank communicator from Init's level -- TLC's lines (counters,
    depth or the violation and every State block) equal the single-GPU run's."""
    import subprocess
    from test_host import LAUNCHER, cfg_text
    name = "RaftSeeded" if spec == "seeded" else "Raft"
    (tmp_path / f"{name}.cfg").write_text(cfg_text(E=2, R=3, vals="v1"))
    env = dict(os.environ, RMC_SKIP_SPEC_CHECK="1")
    base = [LAUNCHER, "-deadlock", "-config", str(tmp_path / f"{name}.cfg"), str(tmp_path / f"{name}.tla")]
    import re
    stamp = re.compile(r"\d{4}-\d\d-\d\d \d\d:\d\d:\d\d")
    keep = lambda out: [stamp.sub("T", ln) for ln in out.splitlines()
                        if not ln.startswith(("Starting", "Finished in", "Progress(", "GPU:", "Running", "vm:",
                                              "RCCL version", "HIP version", "ROCm version", "Hostname",
                                              "Librccl path"))]
    one = subprocess.run(base, capture_output=True, text=True, env=env, timeout=180)
    rk = subprocess.run(base[:1] + ["-gpus", "1", "-onerank", "-shardmin", "1"] + base[1:], capture_output=True,
                        text=True, env=env, timeout=180)
    assert one.returncode == rk.returncode == (12 if spec == "seeded" else 0), rk.stdout + rk.stderr
    assert keep(rk.stdout) == keep(one.stdout)
    assert "Running breadth-first search Model-Checking on 1 GPU" in rk.stdout


# ---- the BecomeFollower variant (Raft.tla:190-231, 420) ---------------------
# Next with `\/ BecomeFollower(s)` uncommented: FollowerUpdateTerm / CandidateToFollower /
# LeaderToFollower right after UpdateTerm, a second candidate per message lane (k_expand<..., BFV>).
@pytest.mark.parametrize("name", sorted(SAMPLES_BF))
def test_become_follower_successors_match_oracle(name):
    g = SAMPLES_BF[name]
    mc = checker(g["n"], g["V"], g["E"], g["R"], spec_variant=raftmc.SPEC_BECOME_FOLLOWER)
    n_bf = 0
    for it in g["items"]:
        got = mc.successors(it["state"])
        exp = it["successors"]
        assert [list(k) for k, _, _ in got] == [e["key"] for e in exp]
        for (k, st, _), e in zip(got, exp):
            assert st == e["state"], (k, it["state"])
        n_bf += sum(1 for e in exp if e["key"][1] == R.A_BF)
    assert n_bf > 0  # the samples reach BecomeFollower steps


@pytest.mark.parametrize("name", sorted(LEVELS_BF))
def test_become_follower_bfs_matches_golden_levels(name):
    g = LEVELS_BF[name]
    mc, res = run_cfg(g)
    check_levels(g, res)
    if name in TRACES_BF:
        tr = mc.trace()
        assert [(list(k) if k else None, st) for k, st in tr] == [(e["key"], e["state"]) for e in TRACES_BF[name]["steps"]]
    mc.close()


def _trace_matches(mc, t):
    assert [(list(k) if k else None, st) for k, st in mc.trace()] == [(e["key"], e["state"]) for e in t["steps"]]


@pytest.mark.parametrize("mode", ["default", "host_levels", "split", "virtual2", "virtual4", "rccl1"])
@pytest.mark.parametrize("name", sorted(LEVELS_ERR))
def test_bfs_error_precedence_matches_golden(name, mode, monkeypatch):
    """The Assert (Raft.tla:185) and Inv's evaluation error (Raft.tla:499) met inside a BFS -- the test
    variants RaftSplitBrain / RaftCommitPastLog -- stop the run where both oracles stop it: the same
    verdict, TLC's counters at the error (states generated and distinct, queue left), the levels before
    it and the counterexample, on the device loop, host-driven levels, split chunks, 2/4 virtual shards
    and the one-rank RCCL communicator."""
    g = LEVELS_ERR[name]
    kw = {}
    if mode == "host_levels":
        kw = dict(device_levels=1)
    elif mode == "split":
        monkeypatch.setenv("RMC_SPLIT_MIN", "1")
        kw = dict(device_levels=1)
    elif mode.startswith("virtual"):
        kw = dict(virtual_shards=int(mode[-1]), chunk_successors=3000, shard_min_states=1)
    elif mode == "rccl1":
        kw = dict(world_size=1, rank=0, comm_unique_id=raftmc.comm_unique_id(), chunk_successors=3000,
                  shard_min_states=1)
    mc, res = run_cfg(g, **kw)
    check_levels(g, res)
    assert [ls.new_states for ls in res.levels if ls.new_states][:len(g["levels"]) - 1] == g["levels"][:-1]
    _trace_matches(mc, TRACES_ERR[name])
    mc.close()


@pytest.mark.parametrize("name,code,line", [("sb_n3_v1_e2_r3", 14, "Error: The first argument of Assert evaluated to FALSE"),
                                            ("cpl_n3_v2_e1_r3", 75, "Error: Evaluating invariant Inv failed.")])
def test_launcher_reports_bfs_errors(name, code, line, tmp_path):
    """raftmc on the test variants (named as tools/make_seeded_spec.py writes them): TLC's error lines
    and exit codes for the Assert and the evaluation error, the counterexample's length and TLC's
    counters at the error."""
    import subprocess
    from test_host import LAUNCHER, cfg_text
    g = LEVELS_ERR[name]
    mod = {"split_brain": "RaftSplitBrain", "commit_past_log": "RaftCommitPastLog"}[g["variant"]]
    (tmp_path / f"{mod}.cfg").write_text(cfg_text(E=g["E"], R=g["R"], vals=", ".join(f"v{i + 1}" for i in range(g["V"]))))
    env = dict(os.environ, RMC_SKIP_SPEC_CHECK="1")
    r = subprocess.run([LAUNCHER, "-deadlock", "-config", str(tmp_path / f"{mod}.cfg"), str(tmp_path / f"{mod}.tla")],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == code, r.stdout + r.stderr
    assert any(ln.startswith(line) for ln in r.stdout.splitlines()), r.stdout
    assert sum(1 for ln in r.stdout.splitlines() if ln.startswith("State ")) == g["trace_len"]
    assert (f"{g['generated']} states generated, {g['distinct']} distinct states found, {g['queue_left']} states "
            f"left on queue.") in r.stdout


@pytest.mark.parametrize("shards", [2, 4])
@pytest.mark.parametrize("name", ["bf_n3_v1_e2_r3", "bf_n4_v1_e1_r3", "bf_n5_v1_e1_r3"])
def test_become_follower_sharded_identical(name, shards):
    """The BecomeFollower variant sharded; at 4 and 5 servers a state has 288 / 301 successor slots
    (msg_cap 128 + the BecomeFollower candidates), past 8 bits: the sharded election key's 10-bit rank."""
    g = LEVELS_BF[name]
    mc, res = run_cfg(g, virtual_shards=shards, chunk_successors=6000, shard_min_states=1)
    check_levels(g, res)
    mc.close()



SELF_LOOP_CASES = ["n3_v1_e1_r3", "n2_v1_e2_r3", "n3_v2_e1_r3"]


@functools.lru_cache(maxsize=None)
def _oracle_self_loops(name):
    """Per expanded level, the oracle's successors identical to their parent (n3 V2 E1: ~11 s)."""
    g = LEVELS[name]
    cfg = R.Config(n=g["n"], V=g["V"], max_election=g["E"], max_restart=g["R"])
    ref = R.bfs(cfg, keep_states=True)
    want = [0] * max(ref.state_levels)
    for st, lv in zip(ref.states, ref.state_levels):
        want[lv - 1] += sum(1 for _, t in R.successors(cfg, st) if t == st)
    return want


SHARDED_SELF_MODES = {
    "virtual2": dict(virtual_shards=2, chunk_successors=3000, shard_min_states=1),
    "virtual3": dict(virtual_shards=3, chunk_successors=3000, shard_min_states=1),
    "rccl1": dict(world_size=1, rank=0, chunk_successors=3000, shard_min_states=1),
}


@pytest.mark.parametrize("mode", ["device_loop", "host_fused", "split", "virtual2", "virtual3", "rccl1",
                                  "virtual2_split", "rccl1_split"])
@pytest.mark.parametrize("name", SELF_LOOP_CASES)
def test_self_loops_per_level_match_oracle(name, mode, monkeypatch):
    """rmc_level_stats.self_loops (ABI 5): per expanded level, the successors equal to their parent
    (FollowerAcceptEntry changing nothing, tla:275-300) -- counted by the item-parallel fused expansion
    (device loop and host-driven chunks), by a split chunk's winner count, and on the sharded path (2 / 3
    virtual shards, a one-rank RCCL communicator; rounds below the split size count them in the routed
    expansion, split rounds in the winner count) -- equal the oracle's count of successors identical to
    their parent (oracle/raft_ref.py successors, exact state equality)."""
    g = LEVELS[name]
    want = _oracle_self_loops(name)
    if mode.endswith("split"):
        monkeypatch.setenv("RMC_SPLIT_MIN", "1")
    base = mode[:-len("_split")] if mode.endswith("_split") else mode
    kw = dict(SHARDED_SELF_MODES.get(base, {}))
    if base == "rccl1":
        kw["comm_unique_id"] = raftmc.comm_unique_id()
    if base in ("host_fused", "split"):
        kw["device_levels"] = 1
    mc, res = run_cfg(g, **kw)
    check_levels(g, res)
    got = [ls.self_loops for ls in res.levels[1:]]
    assert got == want[:len(got)] and sum(got) == sum(want), (got, want)
    assert sum(want) > 0
    mc.close()
