"""CPU tests of the parity oracle itself (oracle/ is test infrastructure).

Pins the restatement the only ways available: SURVEY.md Appendix C's hand-derived
answers, agreement between the independent Python and C restatements, and the
committed golden fixtures (tests/golden/make_golden.py)."""
import ctypes
import json
import os
import subprocess

import pytest

import raft_ref as R
from conftest import GOLDEN, ROOT

ORC_DIR = os.path.join(ROOT, "oracle")
ORC_SO = os.path.join(ORC_DIR, "build", "libraft_oracle.so")


@pytest.fixture(scope="module")
def levels():
    with open(os.path.join(GOLDEN, "levels.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def corc():
    if not os.path.exists(ORC_SO):
        subprocess.check_call(["make", "-s", "-C", ORC_DIR])
    import importlib.util
    spec = importlib.util.spec_from_file_location("mg", os.path.join(GOLDEN, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg


def test_appendix_c_known_answers():
    # n=3, E>=3: levels 1,1,3,9 with 3,5,17 generated
    cfg = R.Config(n=3, V=1, max_election=3, max_restart=3)
    seen_levels, gen = _first_levels(cfg, 4)
    assert seen_levels == [1, 1, 3, 9]
    assert gen == [3, 5, 17]
    cfg2 = R.Config(n=3, V=1, max_election=2, max_restart=3)
    assert _first_levels(cfg2, 4) == ([1, 1, 3, 6], [3, 5, 11])
    cfg5 = R.Config(n=5, V=1, max_election=2, max_restart=3)
    assert _first_levels(cfg5, 3) == ([1, 1, 3], [5, 9])


def _first_levels(cfg, L):
    """BFS truncated after L levels (Python oracle)."""
    s0 = R.init_state(cfg)
    seen = {R.canonical(cfg, s0)}
    frontier = [s0]
    levels, gens = [1], []
    for _ in range(L - 1):
        nxt, g = [], 0
        for st in frontier:
            for _, t in R.successors(cfg, st):
                g += 1
                c = R.canonical(cfg, t)
                if c not in seen:
                    seen.add(c)
                    nxt.append(t)
        levels.append(len(nxt))
        gens.append(g)
        frontier = nxt
    return levels, gens


def test_init_state_matches_spec():
    cfg = R.Config(n=3, V=2)
    s = R.init_state(cfg)
    assert s.votedFor == (R.NONE,) * 3 and s.currentTerm == (0, 0, 0)
    assert s.logs[0] == ((0, R.NONE),) and s.matchIndex[1] == (1, 1, 1) and s.nextIndex[2] == (2, 2, 2)
    assert s.msgs == frozenset() and s.valSent == (R.NONE, R.NONE)
    assert R.inv_leader_has_all_committed(cfg, s)


def test_message_order_is_tlc_record_order():
    # 4-field VoteResp < 6-field records < 8-field AppendReq; VoteReq < AppendResp at equal dst
    vp = R.vote_resp(2, 0, 3)
    vq = R.vote_req(0, 1, 1, 1, 0)
    ap = R.append_resp(0, 1, 1, 1, True)
    aq = R.append_req(1, 0, 1, 1, 0, (), 1)
    assert vp < vq < ap < aq
    assert R.vote_req(2, 0, 1, 1, 0) < R.append_resp(2, 0, 1, 1, False)
    assert R.append_req(0, 1, 1, 1, 0, (), 1) < R.append_req(0, 1, 1, 1, 0, ((1, 0),), 1)


def test_median_is_kth_smallest():
    cfg = R.Config(n=3)
    assert R.median(cfg, (1, 3, 2)) == 2
    assert R.median(cfg, (3, 3, 1)) == 3
    cfg5 = R.Config(n=5)
    assert R.median(cfg5, (1, 2, 3, 4, 5)) == 3
    seeded = R.Config(n=3, seeded=True)
    assert R.median(seeded, (1, 3, 2)) == 3  # threshold n: the maximum, i.e. the leader alone


def test_inv_eval_error_is_detected():
    cfg = R.Config(n=3, V=2)
    s = R.init_state(cfg)
    # leader s1 with a 3-entry log; s2 committed 3 but holds only 2 entries
    logs = (((0, -1), (1, 0), (1, 1)), ((0, -1), (1, 0)), ((0, -1),))
    s = R.State(s.votedFor, (1, 1, 1), logs, s.matchIndex, s.nextIndex, (1, 3, 1), s.msgs, (R.LEADER, 0, 0),
                0, 0, s.pendingResponse, s.valSent)
    with pytest.raises(R.EvalError):
        R.inv_leader_has_all_committed(cfg, s)


def test_python_and_c_oracles_agree_small(corc):
    for (n, V, E, Rr) in [(3, 1, 1, 3), (2, 2, 2, 2)]:
        c = corc.run_c(n, V, E, Rr)
        _, p = corc.run_py(n, V, E, Rr)
        assert (p.generated, p.distinct, p.depth, p.levels, p.generated_per_level) == (
            c["generated"], c["distinct"], c["depth"], c["levels"], c["gen_per_level"])


def test_c_oracle_reproduces_golden_levels(corc, levels):
    for name, g in levels.items():
        if g["distinct"] > 500_000:
            continue
        c = corc.run_c(g["n"], g["V"], g["E"], g["R"], g["seeded"], tuple(g["invariants"]), g["check_deadlock"])
        for k in ("verdict", "generated", "distinct", "depth", "levels", "gen_per_level", "trace_len"):
            assert c[k] == g[k], (name, k)


def test_golden_levels_are_self_consistent(levels):
    for name, g in levels.items():
        if g["verdict"] == "ok":
            assert sum(g["levels"]) == g["distinct"], name
            assert 1 + sum(g["gen_per_level"]) == g["generated"], name
            assert len(g["levels"]) == g["depth"], name
            assert g["levels"][:2] == [1, 1], name


def test_shuffled_order_gives_same_counts_small():
    """SURVEY App. D.2 order-sensitivity probe: shuffled successor order, same partition sizes."""
    cfg = R.Config(n=3, V=2, max_election=1, max_restart=3)
    a = R.bfs(cfg)
    b = R.bfs(cfg, order="shuffle", seed=7)
    assert (a.distinct, a.levels) == (b.distinct, b.levels)


ORDER_PROBE = os.path.join(GOLDEN, "order_probe.json")


def test_order_probe_fixtures_order_insensitive(levels):
    """SURVEY App. D.2 / VERDICT r1 item 7: the C oracle explored each configuration in TLC order (0),
    with every level and every parent's successors reversed (1), and with a seeded shuffle of every
    level (2) -- tests/golden/make_order_probe.py.  Identical per-level distinct and generated counts
    (up to the violation, and its depth, for the seeded runs) say which representative of a VIEW class
    is kept (Raft.tla:34-38) does not change what is reachable: the [TLC-ext] enumeration order and a
    multi-GPU order could not move the counts.  Order 0 is the golden TLC-order run."""
    probe = json.load(open(ORDER_PROBE))
    for k in ("n3_v1_e2_r3", "n3_v2_e2_r3", "seeded_n3_v1_e2_r3", "seeded_n3_v2_e2_r3"):
        assert k in probe, k
    for name, rec in probe.items():
        runs = rec["orders"]
        assert set(runs) == {"0", "1", "2"}, name
        assert rec["order_insensitive"], name
        base = runs["0"]
        for o in ("1", "2"):
            r = runs[o]
            assert (r["verdict"], r["depth"]) == (base["verdict"], base["depth"]), (name, o)
            k = len(base["levels"]) if base["verdict"] == 0 else base["depth"] - 1
            assert r["levels"][:k] == base["levels"][:k], (name, o)
            assert r["gen_per_level"][:k - 1] == base["gen_per_level"][:k - 1], (name, o)
        if name in levels and base["verdict"] == 0:
            g = levels[name]
            assert base["levels"] == g["levels"] and base["distinct"] == g["distinct"], name


def test_no_all_commit_c_and_python_agree(corc):
    """NoAllCommit (tla:451-481) reads msgs: both restatements agree on a state that satisfies
    it and on each variant that drops or alters one of its three messages."""
    import raftmc
    lib = ctypes.CDLL(ORC_SO)
    lib.orc_inv.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int32), ctypes.c_int]
    cfg = R.Config(n=3, V=1, max_election=2, max_restart=3)
    e = (1, 0)
    req1 = R.append_req(0, 2, 1, 1, 0, (e,), 1)
    resp1 = R.append_resp(2, 0, 1, 1, True)
    req2 = R.append_req(0, 2, 1, 2, 1, (), 2)
    got = []
    for msgs in ([req1, resp1, req2], [resp1, req2], [req1, req2], [req1, resp1],
                 [req1, R.append_resp(2, 0, 1, 1, False), req2], [req1, resp1, R.append_req(0, 1, 1, 2, 1, (), 2)]):
        st = R.State(votedFor=(0, 0, 0), currentTerm=(1, 1, 1), logs=(((0, -1), e),) * 3,
                     matchIndex=((2, 2, 2), (1, 1, 1), (1, 1, 1)), nextIndex=((3, 3, 3), (2, 2, 2), (2, 2, 2)),
                     commitIndex=(2, 2, 1), msgs=frozenset(msgs), role=(R.LEADER, R.FOLLOWER, R.FOLLOWER),
                     electionCount=1, restartCount=0, pendingResponse=((False,) * 3,) * 3, valSent=(0,))
        u = raftmc.state_to_unpacked(R.state_to_json(st), 3, 1)
        arr = (ctypes.c_int32 * len(u))(*u)
        exp = R.INV_FUNCS["NoAllCommit"](cfg, st)
        assert lib.orc_inv(3, 1, arr, 5) == int(exp), msgs
        got.append(exp)
    assert got == [True, False, False, False, False, False]


@pytest.mark.parametrize("n,V,E,Rr", [(3, 1, 1, 3), (2, 1, 2, 3), (3, 2, 1, 2)])
def test_follower_append_entry_variant_is_raft(n, V, E, Rr):
    """Uncommenting `\\/ FollowerAppendEntry(s)` in Next (tla:425): restated as TLC evaluates
    it, the action's closing UNCHANGED (tla:371) tests msgs' = msgs and commitIndex' =
    commitIndex after its own SendMsg, so it is never enabled -- the variant explores exactly
    Raft.tla's state graph.  The 371 check is reached (not vacuous) and never passes."""
    base = R.bfs(R.Config(n=n, V=V, max_election=E, max_restart=Rr))
    R.FAPP_STATS.update(reached_unchanged=0, enabled=0)
    var = R.bfs(R.Config(n=n, V=V, max_election=E, max_restart=Rr, follower_append_entry=True))
    assert R.FAPP_STATS["reached_unchanged"] > 0 and R.FAPP_STATS["enabled"] == 0
    assert (var.verdict, var.generated, var.distinct, var.depth, var.levels, var.generated_per_level) == (
        base.verdict, base.generated, base.distinct, base.depth, base.levels, base.generated_per_level)


def test_multithreaded_cpu_baseline_matches_golden():
    """oracle/raft_mt.c (bench.py's cpu_baseline: the same restatement on all host cores, level-
    synchronous with first-wins election) reaches the single-threaded oracle's counts."""
    import ctypes
    so = os.path.join(ROOT, "oracle", "build", "libraft_mt.so")
    if not os.path.exists(so):
        pytest.skip("oracle/build/libraft_mt.so not built")
    lib = ctypes.CDLL(so)
    lib.orc_mt_run.argtypes = [ctypes.c_int] * 5 + [ctypes.POINTER(ctypes.c_uint64)] * 2 + [ctypes.POINTER(ctypes.c_int)]
    levels = json.load(open(os.path.join(GOLDEN, "levels.json")))
    for name in ("n3_v1_e1_r3", "n3_v2_e1_r3", "n2_v2_e3_r3", "n4_v1_e1_r3", "n3_v1_e2_r1"):
        g = levels[name]
        for threads in (1, 3, 8):
            d, gen, dep = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
            rc = lib.orc_mt_run(g["n"], g["V"], g["E"], g["R"], threads, ctypes.byref(d), ctypes.byref(gen),
                                ctypes.byref(dep))
            assert rc == 0
            assert (d.value, gen.value, dep.value) == (g["distinct"], g["generated"], g["depth"]), (name, threads)


def test_mt_oracle_levels_match_golden_and_prefix():
    """orc_mt_levels (the --mt prefix generator behind the configs[3] fixture) reports the same
    per-level distinct/generated counts as the single-threaded oracle's golden levels, and a run
    stopped at max_states ends on a complete level that is a prefix of them."""
    import ctypes
    so = os.path.join(ROOT, "oracle", "build", "libraft_mt.so")
    if not os.path.exists(so):
        pytest.skip("oracle/build/libraft_mt.so not built")
    lib = ctypes.CDLL(so)
    P64 = ctypes.POINTER(ctypes.c_uint64)
    lib.orc_mt_levels.argtypes = [ctypes.c_int] * 5 + [ctypes.c_uint64, P64, P64, ctypes.c_int, P64, P64,
                                                       ctypes.POINTER(ctypes.c_int)]
    levels = json.load(open(os.path.join(GOLDEN, "levels.json")))
    for name, max_states, threads in (("n3_v1_e2_r3", 0, 4), ("n4_v1_e1_r3", 0, 3), ("n3_v1_e2_r3", 5000, 8)):
        g = levels[name]
        d, gen = (ctypes.c_uint64 * 256)(), (ctypes.c_uint64 * 256)()
        dist, tot, dep = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
        rc = lib.orc_mt_levels(g["n"], g["V"], g["E"], g["R"], threads, max_states, d, gen, 256,
                               ctypes.byref(dist), ctypes.byref(tot), ctypes.byref(dep))
        D = dep.value
        if max_states == 0:
            assert rc == 0 and D == g["depth"] and list(d[:D]) == g["levels"]
            assert list(gen[:D]) == g["gen_per_level"]
        else:
            assert rc == 2 and D < g["depth"] and sum(d[:D]) == dist.value >= max_states
            assert list(d[:D]) == g["levels"][:D] and list(gen[:D - 1]) == g["gen_per_level"][:D - 1]


def test_deep_fixture_coverage_and_python_recheck():
    """successors_deep.json.gz (tests/golden/make_golden_deep.py) covers the message-heavy states
    the BFS prefixes cannot reach -- Raft.cfg states with more than 30 messages, and 4/5-server
    states past 64 (the kernels' second message round) -- and every 7th item's successors, classes
    and invariants still come out of the Python restatement unchanged."""
    import gzip
    with gzip.open(os.path.join(GOLDEN, "successors_deep.json.gz"), "rt") as f:
        deep = json.load(f)
    cov = {k: v["coverage"] for k, v in deep.items()}
    assert cov["raftcfg_n3_v2_e3_r3"]["states_over_30_msgs"] >= 50
    assert cov["raftcfg_n3_v2_e3_r3"]["max_msgs"] >= 40 and cov["raftcfg_n3_v2_e3_r3"]["max_depth"] >= 60
    assert cov["c4_n5_v1_e3_r3"]["max_msgs"] >= 60
    assert cov["c4_n5_v1_e3_r3"]["synthetic_states_over_64_msgs"] >= 10
    names = ["Inv", "NoSplitVote", "RaftCanCommt", "FollowerCanCommit", "CommitAll", "NoAllCommit",
             "ExistLeaderAndCandidate"]
    for g in deep.values():
        cfg = R.Config(n=g["n"], V=g["V"], max_election=g["E"], max_restart=g["R"])
        canon = {}
        for it in g["items"][::7]:
            st = R.state_from_json(it["state"])
            if it["assert_fails"]:
                with pytest.raises(R.AssertionFailure):
                    R.successors(cfg, st)
                continue
            succ = R.successors(cfg, st)
            assert [list(k) for k, _ in succ] == [e["key"] for e in it["successors"]]
            assert [R.state_to_json(t) for _, t in succ] == [e["state"] for e in it["successors"]]
            for (_, t), e in zip(succ, it["successors"]):
                c = R.canonical(cfg, t)
                assert canon.setdefault(c, e["canon"]) == e["canon"]
            for nm, v in zip(names, it["invariants"]["state"]):
                try:
                    got = R.INV_FUNCS[nm](cfg, st)
                except R.EvalError:
                    got = None
                assert got == v, nm


@pytest.mark.parametrize("name", ["sb_n3_v1_e2_r3", "sb_n2_v1_e2_r3", "cpl_n3_v2_e1_r3", "sb_n3_v1_e3_r3"])
def test_error_variant_fixtures_recheck(name):
    """The test variants that reach the Assert / Inv's evaluation error in a BFS (RaftSplitBrain,
    RaftCommitPastLog): the Python restatement reproduces the committed fixture (generated by both
    oracles, tests/golden/make_golden_errors.py) -- verdict, TLC's counters, trace length."""
    g = json.load(open(os.path.join(GOLDEN, "levels_errors.json")))[name]
    cfg = R.Config(n=g["n"], V=g["V"], max_election=g["E"], max_restart=g["R"], invariants=tuple(g["invariants"]),
                   **{g["variant"]: True})
    p = R.bfs(cfg)
    assert (p.verdict, p.generated, p.distinct, p.queue_left, len(p.trace)) == \
        (g["verdict"], g["generated"], g["distinct"], g["queue_left"], g["trace_len"])
    assert p.levels[:-1] == g["levels"][:-1]
