"""Raft.cfg's deep levels (35-72) checked state by state against the C oracle.

The per-level counts of levels 1-34 equal the C oracle's BFS (levels_prefix.json); the oracle
cannot exhaust levels 35-72 (10.2 G of the 10.95 G states).  Here the GPU's finished run is sampled
instead: >= 10^4 states spread evenly over levels 35-72 (seeded), and for each, with
oracle/raft_oracle.c as the checker:
  (i)   its path -- TLC's parent pointers and slot keys, rmc_state_path -- has exactly L - 1 steps
        through states of levels 1 .. L - 1 and replays from Init through the oracle's successors in
        TLC key order (orc_replay): the state is a real state of level L under Raft.tla's semantics;
  (ii)  every oracle successor of it (Next, Raft.tla:416-430) has its fingerprint in the GPU's seen
        set: the exploration is closed under Next at the deep levels;
  (iii) first discovery wins inside its parent: no successor of its parent with a smaller key (TLC
        order) is in its exact symmetry class (orc_canon_hash);
  (iv)  distinct sampled states are distinct exact classes (the seen set kept one state per class);
  (v)   its whole-state fingerprint (k_fp_states) is in the seen set: the split chunks' lane-per-
        successor fingerprints (k_hash_probe) and the single-state path agree at depth;
  (vi)  its five server-permuted images (SYMMETRY symmServers, Raft.cfg:24) and a copy with every variable
        outside the VIEW changed (Raft.tla:38, Raft.cfg:26) have its fingerprint: the fingerprint is a function
        of the symmetry class at the deep levels, so no class is split in two -- which (iv) alone, on a
        sample, could only see if both halves were drawn.
Parity is still unpinned by TLC (no TLC anywhere here); this pins the deep levels to the restatement."""
import ctypes
import itertools
import os
import random

import numpy as np
import pytest

import raft_ref as R
import raftmc

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORC_SO = os.path.join(ROOT, "oracle", "build", "libraft_oracle.so")
N, V, E, RR = 3, 2, 3, 3
SAMPLES = 10_000
LO, HI = 35, 72


def _images(u):
    """(vi): the state's server-permuted images and a copy with its non-VIEW variables changed (unpacked)."""
    st = R.state_from_json(raftmc.unpacked_to_state(list(u), N, V))
    out = []
    for pi in itertools.permutations(range(N)):
        if list(pi) == list(range(N)):
            continue
        vf, ct, logs, mi, ni, ci, msgs, role = R.permute_view(st.view(), pi)
        img = R.State(votedFor=vf, currentTerm=ct, logs=logs, matchIndex=mi, nextIndex=ni, commitIndex=ci,
                      msgs=frozenset(msgs), role=role, electionCount=st.electionCount,
                      restartCount=st.restartCount, pendingResponse=st.pendingResponse, valSent=st.valSent)
        out.append(img)
    # outside the VIEW: electionCount, restartCount, pendingResponse, valSent (Raft.tla:29, 34)
    out.append(R.State(votedFor=st.votedFor, currentTerm=st.currentTerm, logs=st.logs, matchIndex=st.matchIndex,
                       nextIndex=st.nextIndex, commitIndex=st.commitIndex, msgs=st.msgs, role=st.role,
                       electionCount=(st.electionCount + 1) % (E + 1), restartCount=(st.restartCount + 1) % (RR + 1),
                       pendingResponse=tuple(tuple(not x for x in r) for r in st.pendingResponse),
                       valSent=tuple(0 if x == R.NONE else R.NONE for x in st.valSent)))
    return [raftmc.state_to_unpacked(R.state_to_json(x), N, V) for x in out]


def _orc():
    lib = ctypes.CDLL(ORC_SO)
    i32p, u32p, u64p = ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64)
    lib.orc_replay.argtypes = [ctypes.c_int] * 5 + [i32p, u32p, ctypes.c_int, i32p, ctypes.c_int]
    lib.orc_successors.argtypes = [ctypes.c_int] * 5 + [i32p, i32p, ctypes.c_int, ctypes.c_int, u32p]
    lib.orc_canon_hash.argtypes = [ctypes.c_int, ctypes.c_int, i32p, u64p]
    return lib


def test_raft_cfg_deep_levels_sampled():
    lib = _orc()
    stride = raftmc.unpacked_len(N, V, 64)
    cfg = raftmc.ModelConfig(n_servers=N, n_vals=V, max_election=E, max_restart=RR)
    init_u = raftmc.state_to_unpacked(R.state_to_json(R.init_state(R.Config(n=N, V=V, max_election=E,
                                                                             max_restart=RR))), N, V)
    init_arr = (ctypes.c_int32 * stride)(*init_u)
    with raftmc.ModelChecker(cfg) as mc:
        res = mc.run()
        assert res.status == "done" and res.depth == HI
        size = {1: 1}
        for ls in res.levels:
            if ls.new_states:
                size[ls.level + 1] = ls.new_states
        start, at = {}, 0
        for L in sorted(size):
            start[L] = at
            at += size[L]
        assert at == res.distinct
        # an even share per level; what the last, small levels cannot take goes to the widest ones
        per = -(-SAMPLES // (HI - LO + 1))
        quota = {L: min(per, size[L]) for L in range(LO, HI + 1)}
        short = SAMPLES - sum(quota.values())
        for L in sorted(quota, key=lambda x: -size[x]):
            add = min(short, size[L] - quota[L])
            quota[L] += add
            short -= add
        rng = random.Random(20261017)
        picks = sorted((L, start[L] + i) for L in quota for i in rng.sample(range(size[L]), quota[L]))
        out = (ctypes.c_int32 * stride)()
        par = (ctypes.c_int32 * stride)()
        succ = (ctypes.c_int32 * (stride * 512))()
        skeys = (ctypes.c_uint32 * 512)()
        h = (ctypes.c_uint64 * 2)()
        batch, classes, n_succ = [], set(), 0
        images, owner = [], []  # (vi): each image and the batch index of its state
        for L, gid in picks:
            keys, gids = mc.state_path(gid)
            # (i) L - 1 steps, through the levels in order
            assert len(keys) == L - 1 and gids[-1] == gid, (L, gid)
            for k, g in enumerate(gids):
                assert start[k + 1] <= g < start[k + 1] + size[k + 1], (L, gid, k, g)
            ck = (ctypes.c_uint32 * len(keys))(*[(s << 24) | (a << 16) | w for s, a, w in keys])
            r = lib.orc_replay(N, V, E, RR, 0, init_arr, ck, len(keys), out, stride)
            assert r > 0, f"level {L} state {gid}: step {-r} of its path is not enabled in the oracle"
            # (iii) first discovery wins among its parent's successors
            assert lib.orc_replay(N, V, E, RR, 0, init_arr, ck, len(keys) - 1, par, stride) > 0
            ns = lib.orc_successors(N, V, E, RR, 0, par, succ, stride, 512, skeys)
            assert ns > 0
            j = next(i for i in range(ns) if skeys[i] == ck[len(keys) - 1])
            assert list(succ[j * stride:j * stride + r]) == list(out[:r])
            assert lib.orc_canon_hash(N, V, out, h) == 0
            mine = (h[0], h[1])
            for i in range(j):
                assert lib.orc_canon_hash(N, V, ctypes.cast(ctypes.addressof(succ) + 4 * i * stride,
                                                            ctypes.POINTER(ctypes.c_int32)), h) == 0
                assert (h[0], h[1]) != mine, f"level {L} state {gid}: an earlier successor of its parent is in its class"
            # (iv) one state per class
            assert mine not in classes, f"level {L} state {gid}: a second state of one symmetry class"
            classes.add(mine)
            # (ii) + (v): the state and every oracle successor of it
            for img in _images(out[:r]):
                images.append(np.asarray(img + [0] * (stride - len(img)), dtype=np.int32))
                owner.append(len(batch))
            batch.append(np.frombuffer(out, dtype=np.int32, count=stride).copy())
            ns = lib.orc_successors(N, V, E, RR, 0, out, succ, stride, 512, skeys)
            assert ns >= 0
            n_succ += ns
            for i in range(ns):
                batch.append(np.frombuffer(succ, dtype=np.int32, count=stride, offset=4 * i * stride).copy())
        arr = np.ascontiguousarray(np.stack(batch))
        fps = mc.fingerprints_unpacked(arr, stride, len(batch))
        present = mc.seen_contains(fps)
        missing = sum(1 for p in present if not p)
        assert missing == 0, f"{missing} of {len(batch)} sampled states / oracle successors not in the seen set"
        # (vi) the images' fingerprints are their states'
        ifp = mc.fingerprints_unpacked(np.ascontiguousarray(np.stack(images)), stride, len(images))
        split = sum(1 for k, f in enumerate(ifp) if tuple(f) != tuple(fps[owner[k]]))
        assert split == 0, f"{split} of {len(images)} symmetric / non-VIEW images fingerprint apart from their states"
    print(f"deep check: {len(picks)} states over levels {LO}-{HI}, {n_succ} oracle successors, all in the seen set; "
          f"{len(images)} images, each with its state's fingerprint")
    assert len(picks) == SAMPLES
