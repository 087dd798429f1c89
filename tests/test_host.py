"""CPU tests of the product's host side: C-ABI exports, cfg parsing, spec identification,
launcher argument handling.  No compute call is made here (no GPU in this container)."""
import ctypes
import json
import os
import re
import subprocess

import pytest

import raftmc
from conftest import ROOT, has_gpu

HEADER = os.path.join(ROOT, "include", "rmc.h")
LAUNCHER = os.path.join(ROOT, "tla-raft_amd", "build", "raftmc")
REF_TLA = "/root/reference/Raft.tla"

# A model config equivalent to the shipped Raft.cfg (Raft.cfg:1-34), written for these tests.
CFG = """CONSTANTS
    MaxTerm = 3
    MaxRestart = {R}
    MaxElection = {E}
    Follower = Follower
    Candidate = Candidate
    Leader = Leader
    None = None
    VoteReq = VoteReq
    VoteResp = VoteResp
    AppendReq = AppendReq
    AppendResp = AppendResp
    s1 = s1
    s2 = s2
    s3 = s3
    s4 = s4
    s5 = s5
    Servers = {{{servers}}}
    v1 = v1
    v2 = v2
    Vals = {{{vals}}}
\\* a comment
SYMMETRY symmServers
VIEW view
INIT Init
NEXT Next
INVARIANT
{inv}
"""


def cfg_text(E=3, R=3, servers="s1, s2, s3", vals="v1, v2", inv="Inv"):
    return CFG.format(E=E, R=R, servers=servers, vals=vals, inv=inv)


def test_library_exports_every_declared_symbol():
    lib = raftmc.load_library()
    decl = re.findall(r"^\s*(?:int|void|const char \*)\s*\**\s*(rmc_\w+)\s*\(", open(HEADER).read(), re.M)
    assert len(decl) >= 14
    for name in decl:
        assert hasattr(lib, name), name
    assert lib.rmc_abi_version() == raftmc.ABI_VERSION == 5


def test_load_library_refuses_another_abi(tmp_path, monkeypatch):
    """A librmc.so of another ABI is refused, not decoded with the wrong struct strides (round 5's r05i
    failure: an ABI-4 race-probe build read through the ABI-5 rmc_level_stats)."""
    src = tmp_path / "old.c"
    src.write_text("int rmc_abi_version(void) { return 4; }\n")
    so = tmp_path / "librmc_old.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    monkeypatch.setattr(raftmc, "_lib", None)
    with pytest.raises(raftmc.RmcError, match="ABI 4"):
        raftmc.load_library(str(so))
    assert raftmc._lib is None


def test_parse_shipped_config_equivalent():
    c = raftmc.parse_config(cfg_text())
    assert (c.n_servers, c.n_vals, c.max_election, c.max_restart) == (3, 2, 3, 3)
    assert c.invariants == ("Inv",) and c.symmetry


def test_parse_verbatim_reference_pair():
    """The reference's own Raft.cfg + Raft.tla (myrun.sh:3 inputs), read in place."""
    cfg_path, tla_path = "/root/reference/Raft.cfg", REF_TLA
    if not (os.path.exists(cfg_path) and os.path.exists(REF_TLA)):
        pytest.skip("reference files not present on this machine")
    c = raftmc.parse_config(open(cfg_path).read(), open(tla_path).read())
    assert (c.n_servers, c.n_vals, c.max_election, c.max_restart) == (3, 2, 3, 3)
    assert c.invariants == ("Inv",) and c.symmetry and c.spec_variant == raftmc.SPEC_RAFT


def test_parse_keeps_invariant_order():
    """TLC checks INVARIANTs in the order the cfg lists them (Raft.cfg:33-34)."""
    c = raftmc.parse_config(cfg_text(inv="NoAllCommit\nRaftCanCommt\nInv"))
    assert c.invariants == ("NoAllCommit", "RaftCanCommt", "Inv")
    assert c.to_c().invariant_order == (6 | 3 << 4 | 1 << 8)
    c = raftmc.parse_config(cfg_text(inv="Inv\nNoAllCommit\nInv"))  # listed twice: checked once
    assert c.invariants == ("Inv", "NoAllCommit")


def test_parse_variants():
    c = raftmc.parse_config(cfg_text(E=2, servers="s1, s2, s3, s4, s5", vals="v1", inv="Inv\nNoSplitVote"))
    assert (c.n_servers, c.n_vals, c.max_election) == (5, 1, 2)
    assert c.invariants == ("Inv", "NoSplitVote")
    c = raftmc.parse_config(cfg_text().replace("SYMMETRY symmServers", ""))
    assert not c.symmetry


@pytest.mark.parametrize("bad,msg", [
    (cfg_text().replace("VIEW view", ""), "VIEW"),
    (cfg_text().replace("MaxElection = 3", "MaxElection = 9"), "MaxElection"),
    (cfg_text().replace("Leader = Leader", "Leader = 1"), "Leader"),
    (cfg_text(inv="Bogus"), "Bogus"),
    (cfg_text(servers=""), "Servers"),
    (cfg_text() + "PROPERTY Liveness\n", "PROPERTY"),
    (cfg_text().replace("INIT Init", "INIT Foo"), "INIT"),
])
def test_parse_errors_are_loud(bad, msg):
    with pytest.raises(raftmc.RmcError, match=msg):
        raftmc.parse_config(bad)


def test_spec_identification():
    if not os.path.exists(REF_TLA):
        pytest.skip("reference Raft.tla not present on this machine")
    tla = open(REF_TLA).read()
    assert raftmc.parse_config(cfg_text(), tla).spec_variant == raftmc.SPEC_RAFT
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_seeded_spec
    assert raftmc.parse_config(cfg_text(), make_seeded_spec.seeded(tla)).spec_variant == raftmc.SPEC_SEEDED
    import make_variant_spec  # Next with FollowerAppendEntry (tla:425): never enabled, Raft.tla's model
    assert raftmc.parse_config(cfg_text(), make_variant_spec.follower_append_entry(tla)).spec_variant == \
        raftmc.SPEC_RAFT
    with pytest.raises(raftmc.RmcError, match="not kikimo"):
        raftmc.parse_config(cfg_text(), tla.replace("MaxElection", "MaxElections"))


def test_create_fails_loudly_without_gpu():
    if has_gpu():
        pytest.skip("GPU present")
    with pytest.raises(raftmc.RmcError, match="RMC_E_DEVICE"):
        raftmc.ModelChecker(raftmc.ModelConfig())


def test_unpacked_roundtrip():
    import raft_ref as R
    cfg = R.Config(n=3, V=2)
    st = R.init_state(cfg)
    for _, t in R.successors(cfg, st):
        for _, u in R.successors(cfg, t):
            d = R.state_to_json(u)
            assert raftmc.unpacked_to_state(raftmc.state_to_unpacked(d, 3, 2), 3, 2) == d


def test_launcher_rejects_unknown_flags(tmp_path):
    r = subprocess.run([LAUNCHER, "-bogus", "Raft.tla"], capture_output=True, text=True)
    assert r.returncode == 150 and "unsupported option" in r.stderr


def test_launcher_gpus_argument(tmp_path):
    """-gpus N (one rank process per GPU, myrun.sh:3's -workers on the node): the count is checked;
    without a GPU every rank fails to start, and the launcher still ends (no rank left waiting for
    the RCCL id) with TLC's header and the error once, from rank 0."""
    r = subprocess.run([LAUNCHER, "-gpus", "0", "Raft.tla"], capture_output=True, text=True)
    assert r.returncode == 150 and "-gpus" in r.stderr
    if has_gpu():
        pytest.skip("the no-device path needs a machine without a GPU")
    (tmp_path / "Raft.cfg").write_text(cfg_text(E=2, R=3, vals="v1"))
    env = dict(os.environ, RMC_SKIP_SPEC_CHECK="1")
    r = subprocess.run([LAUNCHER, "-gpus", "3", "-deadlock", "-config", str(tmp_path / "Raft.cfg"),
                        str(tmp_path / "Raft.tla")], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 75, r.stdout + r.stderr
    out = r.stdout.splitlines()
    assert sum(1 for ln in out if ln.startswith("Running breadth-first search Model-Checking on 3 GPUs")) == 1
    assert sum(1 for ln in out if ln.startswith("Error: could not start the GPU model checker")) == 1


def test_launcher_reports_cfg_errors(tmp_path):
    (tmp_path / "Raft.cfg").write_text(cfg_text().replace("VIEW view", ""))
    env = dict(os.environ, RMC_SKIP_SPEC_CHECK="1")
    r = subprocess.run([LAUNCHER, "-deadlock", "-workers", "4", "-config", str(tmp_path / "Raft.cfg"),
                        str(tmp_path / "Raft.tla")], capture_output=True, text=True, env=env)
    assert r.returncode == 151 and "VIEW" in r.stdout


def _locations(tla_path):
    out = subprocess.check_output([LAUNCHER, "-print-locations", str(tla_path)], text=True)
    return {ln.split()[0]: tuple(map(int, ln.split()[1:])) for ln in out.splitlines()}


def test_action_locations_rules(tmp_path):
    """The trace header's range (raftmc.cpp action_locations): from the first token after "==" to the
    last token before the next column-1 line, skipping blank lines, comment-only lines and a trailing
    line comment."""
    spec = ("---- MODULE M ----\n"
            "Restart(s) ==\n"
            "  /\\ role[s] = Leader   \\* trailing comment\n"
            "  /\\ UNCHANGED x\n"
            "  \\* /\\ Print(x, TRUE)\n"
            "\n"
            "ClientReq(s) == /\\ y' = 1\n"
            "====\n")
    (tmp_path / "M.tla").write_text(spec)
    loc = _locations(tmp_path / "M.tla")
    assert loc["Restart"] == (3, 3, 4, 16)
    assert loc["ClientReq"] == (7, 17, 7, 25)
    assert loc["BecomeLeader"] == (0, 0, 0, 0)  # absent: the launcher falls back to <Action(s)>


def test_action_locations_on_reference_spec():
    """The ranges on the verbatim Raft.tla (skipped where the reference is absent, as on the GPU box).
    Hand-checked against the text: BecomeCandidate's body runs from tla:108 col 3 to the UNCHANGED
    conjunct ending tla:130 col 79; BecomeLeader's ends at tla:172, not at the commented-out Print on
    tla:173; BecomeFollower is the three-line disjunction tla:229-231."""
    src = "/root/reference/Raft.tla"
    if not os.path.exists(src):
        pytest.skip("reference Raft.tla not present")
    loc = _locations(src)
    assert loc["BecomeCandidate"] == (108, 3, 130, 79)
    assert loc["BecomeLeader"][:3] == (158, 3, 172)
    assert loc["UpdateTerm"][:3] == (176, 3, 188)
    assert loc["ResponseVote"][:3] == (133, 3, 155)
    assert loc["Restart"][:3] == (410, 3, 414)
    assert loc["BecomeFollower"] == (229, 3, 231, 24)
    lines = open(src).read().split("\n")
    for name, (l0, c0, l1, c1) in loc.items():
        assert l0 > 1 and lines[l0 - 2].startswith(name + "(s) ==") or lines[l0 - 1].startswith(name), name
        assert lines[l0 - 1][c0 - 1] in "/\\", name          # every body is a conjunction / disjunction list
        last = lines[l1 - 1].split("\\*")[0].rstrip()
        assert len(last) == c1 and last.lstrip(), name         # ends on the last code column of its line


def test_become_follower_variant_spec_recognised():
    """tools/make_variant_spec.py --become-follower on Raft.tla (skipped where the reference is absent, as on
    the GPU box): the launcher's parser maps the text to RMC_SPEC_BECOME_FOLLOWER."""
    src = "/root/reference/Raft.tla"
    if not os.path.exists(src):
        pytest.skip("reference Raft.tla not present")
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    text = subprocess.check_output([sys.executable, os.path.join(root, "tools", "make_variant_spec.py"),
                                    "--become-follower", src]).decode()
    cfg = raftmc.parse_config(open("/root/reference/Raft.cfg").read(), tla_text=text)
    assert cfg.spec_variant == raftmc.SPEC_BECOME_FOLLOWER


def test_bench_xgmi_model():
    """bench.py's modelled xGMI bytes: nothing below the first sharded level, (W-1)/W
    of 28 B per successor + the winners' records and sidecars from it on, zero on one GPU."""
    import importlib.util
    from types import SimpleNamespace as L
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    levels = [L(expanded=10, generated=50, new_bytes=400, new_states=10, self_loops=5),
              L(expanded=2 ** 20, generated=130, new_bytes=800, new_states=20, self_loops=30),
              L(expanded=100, generated=10, new_bytes=0, new_states=0, self_loops=0)]
    assert bench.xgmi_model(levels, 1) == 0
    # (self-loops of a split round are set apart, never routed)
    per = 100 * 28 + 800 + 16 * 20 + 10 * 28
    assert bench.xgmi_model(levels, 2) == per // 2
    assert bench.xgmi_model(levels, 8) == int(per * 7 / 8)


def _bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench


def test_bench_split_bytes_account_for_the_probe_pass():
    """A split chunk's expansion + k_hash_probe move the fused expansion's algorithmic bytes plus what
    the split adds: each parent's hash context written and read back (2 x 112 B for 3 servers and 2
    values) and its count read (4 B), and each successor's staged row read back (32 B)."""
    bench = _bench()
    F, G, N, S = 1000, 5200, 1000, 69.5
    ctxb = bench.ctx_bytes(3, 2)
    assert ctxb == 112
    fused = bench.alg_bytes("expand_hash", F, G, N, S, 16, 8, 32)
    split = bench.alg_bytes("expand_hash", F, G, N, S, 16, 8, 32, split=True, CTXB=ctxb) + \
        bench.alg_bytes("probe", F, G, N, S, 16, 8, 32, CTXB=ctxb)
    assert split == fused + F * (4 + 2 * ctxb) + G * 32


def test_bench_split_roofline_levels_and_bytes():
    """The headline roofline counts the levels whose every chunk is split (>= 2^16 parents; a level whose tail
    chunk is smaller runs that chunk on the fused kernel and is left out), their chunks' algorithmic bytes
    (alg_bytes split=True with the level's successors spread by parents) over their HIP-event expansion time."""
    from types import SimpleNamespace as L
    bench = _bench()
    cfg = L(n_servers=3, n_vals=2, chunk_successors=0)
    cp = bench.chunk_parents(3, 2)
    assert cp == 3050402

    def lv(F, G, N, slf, ms, k):
        ph = [0.0] * 6
        ph[bench.PH_EXPAND] = ms
        la = [0] * 6
        la[bench.PH_EXPAND] = k
        return L(expanded=F, generated=G, new_states=N, self_loops=slf, kernel_ms=ph, kernel_launches=la)
    levels = [lv(1, 3, 1, 0, 0.0, 1),                    # Init's level (skipped)
              lv(1000, 5000, 2000, 100, 0.05, 1),        # fused: below the split size
              lv(2 * cp, 10 * cp, 3 * cp, cp, 80.0, 2),  # two whole split chunks
              lv(cp + 1000, 5 * cp, cp, 0, 50.0, 2),     # a fused tail chunk: left out
              lv(cp + 70000, 5 * cp, cp, 0, 60.0, 2)]    # a split tail chunk
    r = bench.split_roofline([levels], 69.5, cfg)
    assert r["launches"] == 4 and r["levels"] == 2
    want = 0.0
    for F, G, N, slf in ((2 * cp, 10 * cp, 3 * cp, cp), (cp + 70000, 5 * cp, cp, 0)):
        for c0 in range(0, F, cp):
            f = min(cp, F - c0)
            want += bench.alg_bytes("expand_hash", f, G * f / F, N * f / F, 69.5, 16, SWB=32, split=True, CTXB=112,
                                    Gself=slf * f / F)
    assert r["algorithmic_bytes_per_launch"] == round(want / 4)
    assert abs(r["achieved"] - want / 0.140 / 1e9) < 0.01
    assert r["frac"] == round(r["achieved"] / bench.HBM_PEAK_GBS, 5)
    # at N > 1 a rank expands 1/N of every level
    r2 = bench.split_roofline([levels], 69.5, cfg, world=2)
    assert abs(r2["algorithmic_bytes_per_launch"] - round(want / 8)) <= 1


def test_bench_counters_at_scale_read_from_profiles():
    """bench.py's at-scale counters come from the newest committed per-level PMC report, and every
    aggregate is recomputable from its per-level rows."""
    bench = _bench()
    c = bench.counters_at_scale()
    if c is None:
        pytest.skip("no at-scale PMC report committed")
    d = json.load(open(os.path.join(ROOT, c["source"])))
    for k, v in d["kernels"].items():
        rows = v["per_level"]
        alg = sum(r["alg_bytes"] for r in rows)
        hbm = sum(r["hbm_bytes"] for r in rows)
        ms = sum(r["ms"] for r in rows)
        assert abs(hbm / alg - v["aggregate"]["ratio"]) < 2e-3
        assert abs(alg / ms / 1e6 / bench.HBM_PEAK_GBS - v["aggregate"]["alg_frac"]) < 2e-5
        assert c[k]["ratio"] == v["aggregate"]["ratio"]


def test_error_variant_specs_recognised():
    """tools/make_seeded_spec.py --split-brain / --commit-past-log on Raft.tla (skipped where the
    reference is absent): the parser maps each text to its variant by content hash."""
    if not os.path.exists(REF_TLA):
        pytest.skip("reference Raft.tla not present")
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_seeded_spec as M
    tla = open(REF_TLA).read()
    assert raftmc.parse_config(cfg_text(), M.split_brain(tla)).spec_variant == raftmc.SPEC_SPLIT_BRAIN
    assert raftmc.parse_config(cfg_text(), M.commit_past_log(tla)).spec_variant == raftmc.SPEC_COMMIT_PAST_LOG
    with pytest.raises(raftmc.RmcError, match="not kikimo"):
        raftmc.parse_config(cfg_text(), M.split_brain(tla).replace(">= 1 ", ">= 2 "))
