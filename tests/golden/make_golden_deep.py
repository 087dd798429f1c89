#!/usr/bin/env python3
"""Deep-state fixtures: guided random walks from Init into the message-heavy part of the state space.

The BFS prefixes (levels_prefix.json) pin the GPU's counts only where the C oracle can finish
(Raft.cfg: 30 of 72 levels, states with at most 22 messages).  msgs only grows (Raft.tla:43-45),
so the deep levels hold the states with the most messages -- up to 44 at Raft.cfg, and past 64 at
5 servers, where the kernels take a second message round (MR = 2, ids 64-127).  This script walks
from Init (tla:93-105) through Next (tla:416-430) with a bias towards successors that add
messages (go-with-the-winners: walks branched from the paths that reached the most messages), and
commits, per configuration, sampled walk states with:

* their successors in TLC order (keys + concrete states), computed by BOTH oracle/raft_ref.py and
  oracle/raft_oracle.c (orc_successors) and required to agree;
* a server-permuted copy (same symmetry class, tla:21);
* the exact canonical class of every successor (raft_ref.canonical: lexicographic minimum of the
  permuted view over all |Servers|! permutations, tla:21,38), cross-checked against the C
  oracle's exact-canonical hash (orc_canon_hash) -- the two must induce the same partition;
* every invariant's value (tla:434-499; None = TLC evaluation error), Python and C agreeing.

Walk states are reachable (each lies on a path from Init); a few `synthetic` states add random
universe messages to the heaviest walk states up to the GPU layout's message cap (past 64 at 4-5
servers), because the walks top out just below it.  The per-state bar is successors.json's:
bit-exact successor lists, equal classes, equal invariant values.  The fixture records the |msgs|
range it covers per configuration.

Usage: python tests/golden/make_golden_deep.py   (a few minutes on 8 cores; writes successors_deep.json.gz)
"""
import ctypes
import gzip
import json
import os
import random
import sys
import time
import zlib
from concurrent.futures import ProcessPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tla-raft_amd"))

import raft_ref as R  # noqa: E402
from raftmc import state_to_unpacked, unpacked_to_state, unpacked_len  # noqa: E402  (pure-Python converters)

ORC = os.path.join(ROOT, "oracle", "build", "libraft_oracle.so")
INV_NAMES = ["Inv", "NoSplitVote", "RaftCanCommt", "FollowerCanCommit", "CommitAll", "NoAllCommit",
             "ExistLeaderAndCandidate"]

# (name, n, V, E, R, search rounds, synthetic states, walk states kept, message cap of the GPU layout)
CONFIGS = [
    ("raftcfg_n3_v2_e3_r3", 3, 2, 3, 3, 3000, 10, 120, 64),  # Raft.cfg as shipped (configs[0]/[2])
    ("c4_n5_v1_e3_r3", 5, 1, 3, 3, 1500, 16, 72, 128),       # configs[3]: 5 servers (MR = 2 past 64)
    ("n4_v1_e3_r3", 4, 1, 3, 3, 600, 8, 30, 128),            # 4 servers: the signature-coset minimum at n = 4
]


def c_lib():
    lib = ctypes.CDLL(ORC)
    lib.orc_successors.argtypes = [ctypes.c_int] * 5 + [ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                                        ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32)]
    lib.orc_canon_hash.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int32),
                                   ctypes.POINTER(ctypes.c_uint64)]
    lib.orc_inv.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int32), ctypes.c_int]
    return lib


def c_successors(lib, cfg, d, cap_msgs=160):
    u = state_to_unpacked(d, cfg.n, cfg.V)
    inp = (ctypes.c_int32 * len(u))(*u)
    stride = unpacked_len(cfg.n, cfg.V, cap_msgs)
    cap = 1024
    out = (ctypes.c_int32 * (stride * cap))()
    keys = (ctypes.c_uint32 * cap)()
    cnt = lib.orc_successors(cfg.n, cfg.V, cfg.max_election, cfg.max_restart, 0, inp, out, stride, cap, keys)
    if cnt < 0:
        return cnt, []
    res = []
    for i in range(cnt):
        k = keys[i]
        res.append(([k >> 24, (k >> 16) & 0xFF, k & 0xFFFF], unpacked_to_state(out[i * stride:(i + 1) * stride],
                                                                               cfg.n, cfg.V)))
    return cnt, res


def c_canon(lib, cfg, d):
    u = state_to_unpacked(d, cfg.n, cfg.V)
    inp = (ctypes.c_int32 * len(u))(*u)
    h = (ctypes.c_uint64 * 2)()
    assert lib.orc_canon_hash(cfg.n, cfg.V, inp, h) == 0
    return (h[0], h[1])


def c_inv(lib, cfg, d, i):
    u = state_to_unpacked(d, cfg.n, cfg.V)
    inp = (ctypes.c_int32 * len(u))(*u)
    r = lib.orc_inv(cfg.n, cfg.V, inp, i)
    return None if r not in (0, 1) else bool(r)


def walk(lib, cfg, rng, prefix, steps, w_elect, mcap):
    """Continue a path from Init: at every step one successor (C oracle, orc_successors) whose exact
    canonical class (orc_canon_hash) the path has not visited, drawn with weight 3 if it adds a
    message, 1 if not, `w_elect` for BecomeCandidate / Restart (elections and restarts are bounded,
    tla:108,411: spending them late leaves room for more replication traffic per term)."""
    path = list(prefix)
    seen = {c_canon(lib, cfg, d) for d in path}
    st = path[-1]
    for _ in range(steps):
        cnt, succ = c_successors(lib, cfg, st)
        if cnt <= 0:
            break
        cand, wts = [], []
        for (s, a, w), t in succ:
            if len(t["msgs"]) > mcap:
                continue
            h = c_canon(lib, cfg, t)
            if h in seen:
                continue
            cand.append((t, h))
            wts.append(w_elect if a in (R.A_BC, R.A_RS) else (3.0 if len(t["msgs"]) > len(st["msgs"]) else 1.0))
        if not cand:
            break
        st, h = rng.choices(cand, weights=wts)[0]
        seen.add(h)
        path.append(st)
    return path


def search(lib, cfg, rng, rounds, mcap):
    """Go-with-the-winners over walks: 40 walks from Init, then `rounds` times a walk branched at a
    random point of one of the 20 paths that reached the most messages.  Returns every path."""
    elect = (0.02, 0.05, 0.1, 0.3)
    init = [R.state_to_json(R.init_state(cfg))]
    pool = []
    for i in range(40):
        p = walk(lib, cfg, rng, init, 400, elect[i % 4], mcap)
        pool.append((max(len(d["msgs"]) for d in p), p))
    for it in range(rounds):
        pool.sort(key=lambda x: -x[0])
        _, p = rng.choice(pool[:20])
        lo = 1 if it % 2 else max(1, len(p) // 2)  # every other branch from the path's second half
        q = walk(lib, cfg, rng, p[:rng.randrange(lo, len(p) + 1)], 400, elect[it % 4], mcap)
        pool.append((max(len(d["msgs"]) for d in q), q))
    return [p for _, p in pool]


def random_msg(cfg, rng):
    """A message of the static universe (rmc_spec.h Dims; tla:117-125,149,254-263,283-290,310-317)."""
    n, V, E = cfg.n, cfg.V, cfg.max_election
    src = rng.randrange(n)
    dst = rng.choice([x for x in range(n) if x != src])
    term = rng.randint(1, E)
    t = rng.randrange(4)
    if t == 0:
        return R.vote_req(src, dst, term, rng.randint(1, V + 1), rng.randint(0, E))
    if t == 1:
        return R.vote_resp(src, dst, term)
    if t == 2:  # an entry only after index <= V: Len(logs) <= V + 1 (tla:236-237)
        ent = () if V == 0 or rng.random() < 0.4 else ((rng.randint(1, E), rng.randrange(V)),)
        pli = rng.randint(1, V if ent else V + 1)
        return R.append_req(src, dst, term, pli, rng.randint(0, E), ent, rng.randint(1, V + 1))
    return R.append_resp(src, dst, term, rng.randint(1, V + 1), rng.random() < 0.5)


def augment(cfg, rng, st, total):
    """st with random universe messages added until |msgs| = total.  Not reachable in general, but
    every action and invariant is defined on it (the oracles and the kernels evaluate any state
    whose fields lie in their domains): it drives the message lanes past what the walks reach --
    for 5 servers past 64, the kernels' second message round (MR = 2)."""
    msgs = set(st.msgs)
    while len(msgs) < total:
        msgs.add(random_msg(cfg, rng))
    return R.State(**{**st.__dict__, "msgs": frozenset(msgs)})


def one_config(spec):
    name, n, V, E, Rr, walks, n_synth, keep, mcap = spec
    cfg = R.Config(n=n, V=V, max_election=E, max_restart=Rr)
    rng = random.Random(zlib.crc32(name.encode()) ^ 20261017)
    lib = c_lib()
    t0 = time.time()
    pool = [(k, R.state_from_json(d)) for p in search(lib, cfg, rng, walks, mcap) for k, d in enumerate(p) if k]
    # keep states spread over |msgs|, the heaviest third of the range weighted double
    by_m = {}
    for k, st in pool:
        by_m.setdefault(len(st.msgs), []).append((k, st))
    mmax = max(by_m)
    ms = sorted(by_m)
    picked, seen = [], set()
    heavy = [m for m in ms if m >= mmax * 2 // 3]
    order = heavy * 2 + ms
    i = 0
    while len(picked) < keep and i < 50 * keep:
        m = order[i % len(order)]
        i += 1
        k, st = rng.choice(by_m[m])
        key = R.canonical(cfg, st)
        if key in seen:
            continue
        seen.add(key)
        picked.append((k, st))
    # message-heavy synthetic states on top of the heaviest walk states: up to the layout's cap
    heavy_pool = [x for x in pool if len(x[1].msgs) >= mmax - 4]
    synth = []
    for j in range(n_synth):
        k, st = rng.choice(heavy_pool)
        synth.append((k, augment(cfg, rng, st, rng.randint(mmax + 1, mcap))))
    items, canon_ids, c_of_py = [], {}, {}
    for k, st in [(k, st) for k, st in picked] + [(-k, st) for k, st in synth]:
        d = R.state_to_json(st)
        try:
            succ = R.successors(cfg, st)
        except R.AssertionFailure:  # UpdateTerm's Assert (tla:185): a leader with a same-term AppendReq
            assert c_successors(lib, cfg, d)[0] == -1, (name, "C oracle misses the Assert")
            items.append(dict(depth=abs(k), synthetic=k < 0, nmsgs=len(st.msgs), state=d, assert_fails=True))
            continue
        assert all(len(log) <= V + 1 for _, t in succ for log in t.logs), (name, "log past V + 1")
        cnt, csucc = c_successors(lib, cfg, d)
        assert cnt == len(succ), (name, cnt, len(succ))
        for (kk, t), (ck, cd) in zip(succ, csucc):
            assert list(kk) == ck and R.state_to_json(t) == cd, (name, kk, ck)
        perm = list(range(n))
        rng.shuffle(perm)
        pv = R.permute_view(st.view(), perm)
        inv = [0] * n
        for a in range(n):
            inv[perm[a]] = a
        pst = R.State(votedFor=pv[0], currentTerm=pv[1], logs=pv[2], matchIndex=pv[3], nextIndex=pv[4],
                      commitIndex=pv[5], msgs=frozenset(pv[6]), role=pv[7], electionCount=st.electionCount,
                      restartCount=st.restartCount,
                      pendingResponse=tuple(tuple(st.pendingResponse[inv[a]][inv[b]] for b in range(n))
                                            for a in range(n)),
                      valSent=st.valSent)
        assert R.canonical(cfg, pst) == R.canonical(cfg, st)
        sjs = []
        for kk, t in succ:
            tj = R.state_to_json(t)
            c = R.canonical(cfg, t)
            cid = canon_ids.setdefault(c, len(canon_ids))
            ch = c_canon(lib, cfg, tj)
            assert c_of_py.setdefault(ch, cid) == cid, (name, "C/Python canonical partitions differ")
            sjs.append(dict(key=list(kk), state=tj, canon=cid))
        invs = {}
        for sc_st, sc_d, tag in [(st, d, "state")] + [(t, R.state_to_json(t), f"succ{j}")
                                                     for j, (_, t) in enumerate(succ[:4])]:
            vals = []
            for ii, nm in enumerate(INV_NAMES):
                try:
                    pyv = R.INV_FUNCS[nm](cfg, sc_st)
                except R.EvalError:
                    pyv = None
                assert c_inv(lib, cfg, sc_d, ii) == pyv, (name, nm, tag)
                vals.append(pyv)
            invs[tag] = vals
        items.append(dict(depth=abs(k), synthetic=k < 0, nmsgs=len(st.msgs), assert_fails=False, state=d, permuted=R.state_to_json(pst),
                          successors=sjs, invariants=invs))
    nm = [it["nmsgs"] for it in items if not it["synthetic"]]
    succ_nm = [len(s["state"]["msgs"]) for it in items for s in it.get("successors", [])]
    out = dict(n=n, V=V, E=E, R=Rr, items=items,
               coverage=dict(states=len(items), successors=sum(len(it.get("successors", [])) for it in items),
                             assert_states=sum(1 for it in items if it["assert_fails"]),
                             min_msgs=min(nm), max_msgs=max(nm), max_successor_msgs=max(succ_nm),
                             states_over_30_msgs=sum(1 for x in nm if x > 30),
                             synthetic_states=len(synth),
                             synthetic_max_msgs=max(len(st.msgs) for _, st in synth),
                             synthetic_states_over_64_msgs=sum(1 for _, st in synth if len(st.msgs) > 64),
                             max_depth=max(it["depth"] for it in items),
                             pool_max_msgs=mmax,
                             generator="tests/golden/make_golden_deep.py (raft_ref.py + raft_oracle.c agree)"))
    print(name, json.dumps(out["coverage"]), f"{time.time() - t0:.0f}s", flush=True)
    return name, out


def main():
    with ProcessPoolExecutor(max_workers=len(CONFIGS)) as ex:
        res = dict(ex.map(one_config, CONFIGS))
    with gzip.open(os.path.join(HERE, "successors_deep.json.gz"), "wt") as f:
        json.dump(res, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
