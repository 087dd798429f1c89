"""raftmc -- Python binding of librmc.so, the MI355X-native model checker for kikimo/tla-raft.

This is the host-side mirror of the reference's only interface, the TLC run in
``myrun.sh:3`` (``-deadlock -workers 4 -config Raft.cfg Raft.tla``): parse the
model config, exhaust ``Raft.tla``'s state space breadth-first and report TLC's
numbers (states generated, distinct states, depth, counterexample).  Everything
runs in the HIP kernels behind the C-ABI declared in ``include/rmc.h``; there is
no CPU fallback -- ``ModelChecker`` raises if the library or the GPU is missing.
"""
from __future__ import annotations

import ctypes
from collections.abc import Sequence as _SeqABC
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RMC_LIBRARY") or os.path.join(os.path.dirname(_HERE), "build", "librmc.so")

RMC_OK, RMC_DONE, RMC_VIOLATION, RMC_ASSERT, RMC_EVAL_ERROR, RMC_DEADLOCK = 0, 1, 2, 3, 4, 5
STATUS_NAMES = {RMC_OK: "ok", RMC_DONE: "done", RMC_VIOLATION: "invariant", RMC_ASSERT: "assert",
                RMC_EVAL_ERROR: "eval_error", RMC_DEADLOCK: "deadlock"}
ERRORS = {-1: "RMC_E_ARG", -2: "RMC_E_DEVICE", -3: "RMC_E_MEMORY", -4: "RMC_E_CAPACITY",
          -5: "RMC_E_STATE", -6: "RMC_E_PARSE", -7: "RMC_E_COMM"}

# invariant bits (include/rmc.h), Raft.tla:434-503
INVARIANT_BITS = {
    "Inv": 1 << 0, "LeaderHasAllCommittedEntries": 1 << 0, "NoSplitVote": 1 << 1, "RaftCanCommt": 1 << 2,
    "FollowerCanCommit": 1 << 3, "CommitAll": 1 << 4, "NoAllCommit": 1 << 5, "ExistLeaderAndCandidate": 1 << 6,
}
INVARIANT_BY_BIT = ["Inv", "NoSplitVote", "RaftCanCommt", "FollowerCanCommit", "CommitAll", "NoAllCommit",
                    "ExistLeaderAndCandidate"]
ACTIONS = ("BecomeCandidate", "UpdateTerm", "ResponseVote", "BecomeLeader", "ClientReq", "LeaderAppendEntry",
           "FollowerAcceptEntry", "FollowerRejectEntry", "HandleAppendResp", "LeaderCanCommit", "Restart",
           "FollowerAppendEntry", "BecomeFollower")  # 11: never enabled (tla:425 variant); 12: tla:420 variant
SPEC_RAFT, SPEC_SEEDED, SPEC_BECOME_FOLLOWER = 0, 1, 2
SPEC_SPLIT_BRAIN, SPEC_COMMIT_PAST_LOG = 3, 4  # test variants: Assert / evaluation error reachable in a BFS
# include/rmc.h RMC_ABI_VERSION: the struct layouts below (_Config, _LevelStats, _Result) follow this ABI; a
# library of another ABI would be decoded with the wrong strides, so load_library refuses it
ABI_VERSION = 5


class RmcError(RuntimeError):
    pass


class _Config(ctypes.Structure):
    _fields_ = [
        ("n_servers", ctypes.c_int32), ("n_vals", ctypes.c_int32), ("max_election", ctypes.c_int32),
        ("max_restart", ctypes.c_int32), ("invariants", ctypes.c_uint32), ("check_deadlock", ctypes.c_int32),
        ("spec_variant", ctypes.c_int32), ("device", ctypes.c_int32), ("msg_cap", ctypes.c_int32),
        ("seen_log2", ctypes.c_int32), ("no_symmetry", ctypes.c_int32), ("chunk_successors", ctypes.c_uint64),
        ("rank", ctypes.c_int32), ("world_size", ctypes.c_int32), ("comm_unique_id", ctypes.c_void_p),
        ("virtual_shards", ctypes.c_int32), ("timing_phases", ctypes.c_uint32),
        ("device_levels", ctypes.c_uint32), ("shard_min_states", ctypes.c_uint64),
        ("invariant_order", ctypes.c_uint32), ("compact_log2", ctypes.c_uint32),
        ("seen_mem_bytes", ctypes.c_uint64), ("frontier_mem_bytes", ctypes.c_uint64),
    ]


class _LevelStats(ctypes.Structure):
    _fields_ = [
        ("level", ctypes.c_int32), ("status", ctypes.c_int32), ("expanded", ctypes.c_uint64),
        ("generated", ctypes.c_uint64), ("new_states", ctypes.c_uint64), ("total_generated", ctypes.c_uint64),
        ("total_distinct", ctypes.c_uint64), ("queue", ctypes.c_uint64), ("seconds", ctypes.c_double),
        ("kernel_ms", ctypes.c_double * 6), ("kernel_launches", ctypes.c_uint64 * 6),
        ("new_bytes", ctypes.c_uint64), ("self_loops", ctypes.c_uint64),
    ]


class _Result(ctypes.Structure):
    _fields_ = [
        ("status", ctypes.c_int32), ("depth", ctypes.c_int32), ("generated", ctypes.c_uint64),
        ("distinct", ctypes.c_uint64), ("queue", ctypes.c_uint64), ("violated", ctypes.c_int32),
        ("trace_len", ctypes.c_uint32), ("seconds", ctypes.c_double),
        ("seen_slots", ctypes.c_uint64), ("seen_slot_bytes", ctypes.c_int32), ("pad_", ctypes.c_int32),
        ("frontier_ring_bytes", ctypes.c_uint64), ("frontier_peak_bytes", ctypes.c_uint64),
    ]


_U64P = ctypes.POINTER(ctypes.c_uint64)
_ALLREDUCE = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, _U64P, ctypes.c_int32, ctypes.c_int32)
_ALLGATHER = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, _U64P, ctypes.c_int32, _U64P)
_ALLTOALLV = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, _U64P, _U64P, ctypes.c_void_p,
                              _U64P, _U64P)


class _Transport(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("allreduce_u64", _ALLREDUCE), ("allgather_u64", _ALLGATHER),
                ("alltoallv", _ALLTOALLV)]


_lib = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load librmc.so; raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RmcError(f"librmc.so not found at {path}: run __graft_entry__.build() (make -C tla-raft_amd)")
    lib = ctypes.CDLL(path)
    vp, i32, u32, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64
    P = ctypes.POINTER
    lib.rmc_abi_version.restype = ctypes.c_int
    abi = lib.rmc_abi_version()
    if abi != ABI_VERSION:
        raise RmcError(f"{path} has ABI {abi}, this binding decodes ABI {ABI_VERSION}: rebuild it "
                       f"(make -C tla-raft_amd)")
    lib.rmc_parse_config.argtypes = [ctypes.c_char_p, ctypes.c_char_p, P(_Config), ctypes.c_char_p, ctypes.c_size_t]
    lib.rmc_create.argtypes = [P(_Config), P(vp)]
    lib.rmc_init.argtypes = [vp, P(_LevelStats)]
    lib.rmc_step.argtypes = [vp, P(_LevelStats)]
    lib.rmc_steps.argtypes = [vp, P(_LevelStats), u32, P(u32)]
    lib.rmc_set_timing.argtypes = [vp, u32]
    lib.rmc_probe_peak.argtypes = [i32, u32, u64, P(ctypes.c_double), P(ctypes.c_double)]
    lib.rmc_run.argtypes = [vp, P(_Result)]
    lib.rmc_reset.argtypes = [vp]
    lib.rmc_checkpoint.argtypes = [vp, ctypes.c_char_p]
    lib.rmc_resume.argtypes = [vp, ctypes.c_char_p]
    lib.rmc_run_levels.argtypes = [vp, P(_LevelStats), u32, P(u32), P(_Result)]
    lib.rmc_comm_unique_id.argtypes = [vp]
    lib.rmc_get_result.argtypes = [vp, P(_Result)]
    lib.rmc_trace_len.argtypes = [vp, P(u32)]
    lib.rmc_trace_state.argtypes = [vp, u32, P(i32), ctypes.c_size_t, P(i32), P(i32), P(i32)]
    lib.rmc_last_error.argtypes = [vp]
    lib.rmc_last_error.restype = ctypes.c_char_p
    lib.rmc_destroy.argtypes = [vp]
    lib.rmc_destroy.restype = None
    lib.rmc_successors.argtypes = [vp, P(i32), P(i32), ctypes.c_size_t, u32, P(u32), P(u64), P(u32)]
    lib.rmc_fingerprint.argtypes = [vp, P(i32), P(u64)]
    lib.rmc_eval_invariant.argtypes = [vp, P(i32), u32, P(i32)]
    lib.rmc_set_transport.argtypes = [P(_Transport)]
    lib.rmc_state_path.argtypes = [vp, u64, P(u32), P(u64), u32, P(u32)]
    lib.rmc_fingerprints.argtypes = [vp, P(i32), ctypes.c_size_t, u64, P(u64)]
    lib.rmc_seen_contains.argtypes = [vp, P(u64), u64, P(ctypes.c_uint8)]
    _lib = lib
    return lib


# ------------------------------------------------------------------------------ config
@dataclass
class ModelConfig:
    """What Raft.cfg binds (Raft.cfg:1-34) plus TLC's -deadlock flag (myrun.sh:3)."""
    n_servers: int = 3
    n_vals: int = 2
    max_election: int = 3
    max_restart: int = 3
    invariants: Tuple[str, ...] = ("Inv",)
    check_deadlock: bool = False
    spec_variant: int = SPEC_RAFT
    symmetry: bool = True
    device: int = -1
    msg_cap: int = 0
    seen_log2: int = 0
    chunk_successors: int = 0
    virtual_shards: int = 0          # >1: that many fingerprint-owner shards on one device
    rank: int = 0                    # multi-GPU: this process's rank
    world_size: int = 1              # multi-GPU: ranks (one process per GPU)
    comm_unique_id: Optional[bytes] = None  # 128 bytes from comm_unique_id() on rank 0
    timing_phases: int = 0           # bit i: time phase i with HIP events (0 = all phases)
    device_levels: int = 0           # levels per host round trip in run() (0 = auto, 1 = host-driven)
    shard_min_states: int = 0        # >1 shards: replicate levels below this size (0 = auto 2^20, 1 = always shard)
    compact_log2: int = 0            # seen set: 16-B slots up to 2^compact_log2 slots, then 8-B slots (0 = auto 27)
    seen_mem_bytes: int = 0          # compact seen-set budget (0 = auto: half the free device memory)
    frontier_mem_bytes: int = 0      # frontier ring budget once the seen set is compact (0 = auto)

    def to_c(self) -> _Config:
        c = _Config()
        c.n_servers, c.n_vals = self.n_servers, self.n_vals
        c.max_election, c.max_restart = self.max_election, self.max_restart
        mask, order, k = 0, 0, 0
        for name in self.invariants:  # cfg order: TLC checks the invariants in that order
            bit = INVARIANT_BITS[name]
            if not mask & bit:
                order |= (bit.bit_length()) << (4 * k)
                k += 1
            mask |= bit
        c.invariants = mask
        c.invariant_order = order
        c.check_deadlock = int(self.check_deadlock)
        c.spec_variant = self.spec_variant
        c.device = self.device
        c.msg_cap = self.msg_cap
        c.seen_log2 = self.seen_log2
        c.no_symmetry = 0 if self.symmetry else 1
        c.chunk_successors = self.chunk_successors
        c.rank, c.world_size = self.rank, self.world_size
        c.virtual_shards = self.virtual_shards
        c.timing_phases = self.timing_phases
        c.device_levels = self.device_levels
        c.shard_min_states = self.shard_min_states
        c.compact_log2 = self.compact_log2
        c.seen_mem_bytes = self.seen_mem_bytes
        c.frontier_mem_bytes = self.frontier_mem_bytes
        if self.comm_unique_id is not None:
            self._idbuf = ctypes.create_string_buffer(bytes(self.comm_unique_id), 128)
            c.comm_unique_id = ctypes.cast(self._idbuf, ctypes.c_void_p)
        return c


def probe_peak(device: int = -1, table_log2: int = 28, probes: int = 1 << 28) -> float:
    """Random one-slot probes/s of a seen-set-shaped table (16-B slots) on the GPU."""
    lib = load_library()
    r, t = ctypes.c_double(), ctypes.c_double()
    rc = lib.rmc_probe_peak(device, table_log2, probes, ctypes.byref(r), ctypes.byref(t))
    if rc != RMC_OK:
        raise RmcError(f"rmc_probe_peak failed: {ERRORS.get(rc, rc)}")
    return r.value


def parse_config(cfg_text: str, tla_text: Optional[str] = None) -> ModelConfig:
    """Parse Raft.cfg text (and identify Raft.tla by content) through the library's parser."""
    lib = load_library()
    c = _Config()
    err = ctypes.create_string_buffer(512)
    rc = lib.rmc_parse_config(cfg_text.encode(), tla_text.encode() if tla_text is not None else None,
                              ctypes.byref(c), err, 512)
    if rc != RMC_OK:
        raise RmcError(err.value.decode())
    invs, o = [], c.invariant_order
    while o:
        invs.append(INVARIANT_BY_BIT[(o & 15) - 1])
        o >>= 4
    invs = tuple(invs) or tuple(name for bit, name in enumerate(INVARIANT_BY_BIT) if c.invariants & (1 << bit))
    return ModelConfig(n_servers=c.n_servers, n_vals=c.n_vals, max_election=c.max_election,
                       max_restart=c.max_restart, invariants=invs, check_deadlock=bool(c.check_deadlock),
                       spec_variant=c.spec_variant, symmetry=not c.no_symmetry)


def comm_unique_id() -> bytes:
    """RCCL unique id for a multi-GPU run (rank 0 creates it, every rank passes it in)."""
    lib = load_library()
    buf = ctypes.create_string_buffer(128)
    rc = lib.rmc_comm_unique_id(buf)
    if rc != RMC_OK:
        raise RmcError(f"rmc_comm_unique_id failed: {ERRORS.get(rc, rc)}")
    return buf.raw


class HostTransport:
    """The sharded protocol's collectives through host memory and a torch.distributed process group
    (include/rmc.h rmc_transport) instead of RCCL: every rank of a world_size > 1 run installs one
    before creating its ModelChecker (without comm_unique_id).  With a gloo group the ranks may share
    one device -- the multi-rank path of SURVEY 8(e) as separate processes on a one-GPU box (tests) --
    since RCCL refuses two ranks on one device.  A callback that raises fails the step (RMC_E_COMM)."""

    def __init__(self, group=None):
        import numpy as np
        import torch
        import torch.distributed as dist
        self._np, self._torch, self._dist, self._group = np, torch, dist, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self._c = _Transport(None, _ALLREDUCE(self._allreduce), _ALLGATHER(self._allgather),
                             _ALLTOALLV(self._alltoallv))

    @staticmethod
    def _failed():
        import sys
        import traceback
        traceback.print_exc(file=sys.stderr)
        return 1

    def _u64(self, ptr, n):
        return self._np.ctypeslib.as_array(ptr, shape=(n,))

    def _allreduce(self, _user, v, n, is_max):
        try:
            a = self._u64(v, n)
            t = self._torch.from_numpy(a.astype(self._np.int64))  # values < 2^63 (counts, keys, codes)
            self._dist.all_reduce(t, op=self._dist.ReduceOp.MAX if is_max else self._dist.ReduceOp.SUM,
                                  group=self._group)
            a[:] = t.numpy().astype(self._np.uint64)
            return 0
        except Exception:  # noqa: BLE001 -- the library raises RMC_E_COMM
            return self._failed()

    def _allgather(self, _user, row, k, out):
        try:
            t = self._torch.from_numpy(self._u64(row, k).astype(self._np.int64))
            parts = [self._torch.empty_like(t) for _ in range(self.world)]
            self._dist.all_gather(parts, t, group=self._group)
            self._u64(out, self.world * k)[:] = self._torch.cat(parts).numpy().astype(self._np.uint64)
            return 0
        except Exception:  # noqa: BLE001
            return self._failed()

    def _alltoallv(self, _user, send, send_off, send_bytes, recv, recv_off, recv_bytes):
        try:
            W = self.world
            sb, rb = self._u64(send_bytes, W).tolist(), self._u64(recv_bytes, W).tolist()
            so, ro = self._u64(send_off, W).tolist(), self._u64(recv_off, W).tolist()
            send_end = max([int(o + b) for o, b in zip(so, sb)] + [1])
            recv_end = max([int(o + b) for o, b in zip(ro, rb)] + [1])
            src = self._np.ctypeslib.as_array(ctypes.cast(send, ctypes.POINTER(ctypes.c_uint8)), shape=(send_end,))
            dst = self._np.ctypeslib.as_array(ctypes.cast(recv, ctypes.POINTER(ctypes.c_uint8)), shape=(recv_end,))
            # all_to_all_single takes the parts in rank order, contiguous
            ti = self._torch.from_numpy(self._np.concatenate([src[int(so[q]):int(so[q] + sb[q])] for q in range(W)]))
            to = self._torch.empty(int(sum(rb)), dtype=self._torch.uint8)
            self._dist.all_to_all_single(to, ti, [int(x) for x in rb], [int(x) for x in sb], group=self._group)
            got, at = to.numpy(), 0
            for q in range(W):
                dst[int(ro[q]):int(ro[q] + rb[q])] = got[at:at + int(rb[q])]
                at += int(rb[q])
            return 0
        except Exception:  # noqa: BLE001
            return self._failed()

    def install(self):
        """Route the collectives of every ModelChecker created from now on in this process through this group."""
        rc = load_library().rmc_set_transport(ctypes.byref(self._c))
        if rc != RMC_OK:
            raise RmcError(f"rmc_set_transport failed: {ERRORS.get(rc, rc)}")
        return self

    @staticmethod
    def uninstall():
        load_library().rmc_set_transport(None)


# ------------------------------------------------------------------------------ unpacked states
MSG_TYPES = ("VoteReq", "VoteResp", "AppendReq", "AppendResp")


def unpacked_len(n: int, V: int, nmsgs: int) -> int:
    return 5 * n + n * (V + 1) * 2 + 3 * n * n + 3 + V + 8 * nmsgs


def state_to_unpacked(d: dict, n: int, V: int) -> List[int]:
    """JSON state (oracle fixture format) -> rmc unpacked int32 layout (include/rmc.h)."""
    u: List[int] = []
    u += d["votedFor"] + d["currentTerm"] + d["role"] + d["commitIndex"] + [len(l) for l in d["logs"]]
    for log in d["logs"]:
        for x in range(V + 1):
            if x < len(log):
                u += [log[x][0], log[x][1]]
            else:
                u += [0, 0]
    for r in d["matchIndex"]:
        u += r
    for r in d["nextIndex"]:
        u += r
    for r in d["pendingResponse"]:
        u += [1 if b else 0 for b in r]
    u += [d["electionCount"], d["restartCount"]] + list(d["valSent"]) + [len(d["msgs"])]
    for m in d["msgs"]:
        t = MSG_TYPES.index(m["type"])
        rec = [t, m["src"], m["dst"], m["term"], 0, 0, 0, 0]
        if m["type"] == "VoteReq":
            rec[4:6] = [m["lastLogIndex"], m["lastLogTerm"]]
        elif m["type"] == "AppendResp":
            rec[4:6] = [m["prevLogIndex"], 1 if m["succ"] else 0]
        elif m["type"] == "AppendReq":
            e = m["entries"]
            rec[4:8] = [m["prevLogIndex"], m["prevLogTerm"], m["leaderCommit"], e[0][0] * 8 + e[0][1] if e else -1]
        u += rec
    return u


def unpacked_to_state(u: Sequence[int], n: int, V: int) -> dict:
    k = 0

    def take(c):
        nonlocal k
        r = list(u[k:k + c])
        k += c
        return r

    d: Dict[str, object] = {}
    d["votedFor"] = take(n)
    d["currentTerm"] = take(n)
    d["role"] = take(n)
    d["commitIndex"] = take(n)
    ll = take(n)
    logs = []
    for i in range(n):
        ent = take(2 * (V + 1))
        logs.append([[ent[2 * x], ent[2 * x + 1]] for x in range(ll[i])])
    d["logs"] = logs
    d["matchIndex"] = [take(n) for _ in range(n)]
    d["nextIndex"] = [take(n) for _ in range(n)]
    d["pendingResponse"] = [[bool(x) for x in take(n)] for _ in range(n)]
    d["electionCount"], d["restartCount"] = take(2)
    d["valSent"] = take(V)
    nm = take(1)[0]
    msgs = []
    for _ in range(nm):
        t, src, dst, term, x1, x2, x3, x4 = take(8)
        m = {"type": MSG_TYPES[t], "src": src, "dst": dst, "term": term}
        if t == 0:
            m.update(lastLogIndex=x1, lastLogTerm=x2)
        elif t == 3:
            m.update(prevLogIndex=x1, succ=bool(x2))
        elif t == 2:
            m.update(prevLogIndex=x1, prevLogTerm=x2, leaderCommit=x3,
                     entries=[] if x4 < 0 else [[x4 // 8, x4 % 8]])
        msgs.append(m)
    d["msgs"] = msgs
    return d


# ------------------------------------------------------------------------------ checker
@dataclass
class LevelStats:
    level: int
    status: str
    expanded: int
    generated: int
    new_states: int
    total_generated: int
    total_distinct: int
    queue: int
    seconds: float
    kernel_ms: List[float] = field(default_factory=list)
    kernel_launches: List[int] = field(default_factory=list)
    new_bytes: int = 0
    self_loops: int = 0  # ABI 5: successors equal to their parent, set apart (single-GPU split chunks)


class _LazyLevels(_SeqABC):
    """Per-level statistics of one run, converted to LevelStats on first access (a run's levels come
    back from the library as one array; building dozens of Python objects per exhaustion would cost
    more host time than a small configuration's whole GPU run)."""

    def __init__(self, raw, n: int):
        self._raw = (_LevelStats * n)()
        ctypes.memmove(self._raw, raw, ctypes.sizeof(_LevelStats) * n)
        self._cache: List[Optional[LevelStats]] = [None] * n

    def __len__(self):
        return len(self._cache)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError(i)
        if self._cache[i] is None:
            self._cache[i] = ModelChecker._stats(self._raw[i])
        return self._cache[i]

    def __eq__(self, other):
        return list(self) == list(other)

    def __repr__(self):
        return repr(list(self))


@dataclass
class Result:
    status: str
    depth: int
    generated: int
    distinct: int
    queue: int
    violated: Optional[str]
    trace_len: int
    seconds: float
    levels: List[LevelStats] = field(default_factory=list)
    seen_slots: int = 0
    seen_slot_bytes: int = 0
    frontier_ring_bytes: int = 0
    frontier_peak_bytes: int = 0


class ModelChecker:
    """One GPU model-checking run (TLC's ModelChecker for myrun.sh:3)."""

    def __init__(self, cfg: ModelConfig):
        self.lib = load_library()
        self.cfg = cfg
        self._c = cfg.to_c()
        h = ctypes.c_void_p()
        rc = self.lib.rmc_create(ctypes.byref(self._c), ctypes.byref(h))
        if rc != RMC_OK:
            raise RmcError(f"rmc_create failed: {ERRORS.get(rc, rc)} (see stderr)")
        self.h = h
        self.levels: List[LevelStats] = []
        self._inited = False

    def close(self):
        if getattr(self, "h", None):
            self.lib.rmc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _levels_list(self) -> list:
        if not isinstance(self.levels, list):
            self.levels = list(self.levels)
        return self.levels

    def _check(self, rc: int) -> int:
        if rc < 0:
            raise RmcError(f"{ERRORS.get(rc, rc)}: {self.lib.rmc_last_error(self.h).decode()}")
        return rc

    @staticmethod
    def _stats(s: _LevelStats) -> LevelStats:
        return LevelStats(s.level, STATUS_NAMES.get(s.status, str(s.status)), s.expanded, s.generated,
                          s.new_states, s.total_generated, s.total_distinct, s.queue, s.seconds,
                          list(s.kernel_ms), list(s.kernel_launches), s.new_bytes, s.self_loops)

    def init(self) -> LevelStats:
        st = _LevelStats()
        self._check(self.lib.rmc_init(self.h, ctypes.byref(st)))
        self._inited = True
        ls = self._stats(st)
        self._levels_list().append(ls)
        return ls

    def reset(self) -> None:
        """Start over from Init on the next run(), keeping the device buffers."""
        self._check(self.lib.rmc_reset(self.h))
        self.levels = []
        self._inited = False

    def checkpoint(self, path: str) -> None:
        """Write the run so far (seen set, current level, parent references, counters) to path (an RCCL
        rank of a world_size > 1 run: path + ".rank<r>"; virtual shards: all in path)."""
        self._check(self.lib.rmc_checkpoint(self.h, os.fsencode(path)))

    def resume(self, path: str) -> None:
        """Continue a checkpointed run of the same configuration (on a fresh or reset checker)."""
        self._check(self.lib.rmc_resume(self.h, os.fsencode(path)))
        self._inited = True

    def step(self) -> LevelStats:
        st = _LevelStats()
        self._check(self.lib.rmc_step(self.h, ctypes.byref(st)))
        ls = self._stats(st)
        self._levels_list().append(ls)
        return ls

    def set_timing(self, phases: int) -> None:
        """HIP-event phase timing from now on: 0 = off, 0xFFFFFFFF = all phases, else a phase mask."""
        self._check(self.lib.rmc_set_timing(self.h, phases))

    def steps(self, cap: int = 65) -> List[LevelStats]:
        """The levels one host round trip covers (rmc_steps): a device-driven batch on one GPU."""
        buf = (_LevelStats * cap)()
        n = ctypes.c_uint32()
        self._check(self.lib.rmc_steps(self.h, buf, cap, ctypes.byref(n)))
        out = [self._stats(buf[i]) for i in range(n.value)]
        self._levels_list().extend(out)
        return out

    def run(self) -> Result:
        """Exhaust the state space (or stop at the first error) inside the library."""
        cap = 4096
        if getattr(self, "_runbuf", None) is None:
            self._runbuf = (_LevelStats * cap)()  # reused by every run of this checker
        n = ctypes.c_uint32()
        self._check(self.lib.rmc_run_levels(self.h, self._runbuf, cap, ctypes.byref(n), None))
        self._inited = True
        lazy = _LazyLevels(self._runbuf, n.value)
        self.levels = lazy if not self.levels else list(self.levels) + list(lazy)
        return self.result()

    def result(self) -> Result:
        r = _Result()
        self._check(self.lib.rmc_get_result(self.h, ctypes.byref(r)))
        return Result(STATUS_NAMES.get(r.status, str(r.status)), r.depth, r.generated, r.distinct, r.queue,
                      INVARIANT_BY_BIT[r.violated] if r.violated >= 0 else None, r.trace_len, r.seconds,
                      self.levels if isinstance(self.levels, _LazyLevels) else list(self.levels), r.seen_slots,
                      r.seen_slot_bytes, r.frontier_ring_bytes,
                      r.frontier_peak_bytes)

    def trace(self) -> List[Tuple[Optional[Tuple[int, int, int]], dict]]:
        n = ctypes.c_uint32()
        self._check(self.lib.rmc_trace_len(self.h, ctypes.byref(n)))
        cap = unpacked_len(self.cfg.n_servers, self.cfg.n_vals, 256)
        buf = (ctypes.c_int32 * cap)()
        out = []
        for i in range(n.value):
            a, s, w = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
            k = self._check(self.lib.rmc_trace_state(self.h, i, buf, cap, ctypes.byref(a), ctypes.byref(s),
                                                     ctypes.byref(w)))
            st = unpacked_to_state(list(buf[:k]), self.cfg.n_servers, self.cfg.n_vals)
            out.append((None if a.value < 0 else (s.value, a.value, w.value), st))
        return out

    # ---- single-state hooks ------------------------------------------------------------
    def _unpacked(self, state: dict):
        u = state_to_unpacked(state, self.cfg.n_servers, self.cfg.n_vals)
        return (ctypes.c_int32 * len(u))(*u)

    def successors(self, state: dict, cap: int = 512):
        """[(key(server, action, witness), successor_state, fp128)] in TLC order; raises on Assert."""
        n, V = self.cfg.n_servers, self.cfg.n_vals
        stride = unpacked_len(n, V, 256)
        out = (ctypes.c_int32 * (stride * cap))()
        keys = (ctypes.c_uint32 * cap)()
        fps = (ctypes.c_uint64 * (2 * cap))()
        cnt = ctypes.c_uint32()
        rc = self._check(self.lib.rmc_successors(self.h, self._unpacked(state), out, stride, cap, keys, fps,
                                                 ctypes.byref(cnt)))
        if rc == RMC_ASSERT:
            raise AssertionError("split brain")
        res = []
        for i in range(cnt.value):
            k = keys[i]
            st = unpacked_to_state(list(out[i * stride:(i + 1) * stride]), n, V)
            res.append(((k >> 24, (k >> 16) & 0xFF, k & 0xFFFF), st, (fps[2 * i], fps[2 * i + 1])))
        return res

    def fingerprint(self, state: dict) -> Tuple[int, int]:
        fp = (ctypes.c_uint64 * 2)()
        self._check(self.lib.rmc_fingerprint(self.h, self._unpacked(state), fp))
        return fp[0], fp[1]

    # ---- checks of a finished run's deep levels (tests/test_gpu_deep.py) -----------------
    def state_path(self, gid: int):
        """(keys, gids): how each state on the path from Init to the explored state `gid` was reached
        ((server, action, witness) per step) and the global ids of the path's states (Init's 0 first)."""
        cap = 4096
        keys, gids, n = (ctypes.c_uint32 * cap)(), (ctypes.c_uint64 * cap)(), ctypes.c_uint32()
        self._check(self.lib.rmc_state_path(self.h, gid, keys, gids, cap, ctypes.byref(n)))
        return ([(k >> 24, (k >> 16) & 0xFF, k & 0xFFFF) for k in keys[1:n.value]], list(gids[:n.value]))

    def fingerprints_unpacked(self, unpacked, stride: int, n: int):
        """Fingerprints of n unpacked states (a contiguous int32 buffer, `stride` ints apart), one launch."""
        fps = (ctypes.c_uint64 * (2 * max(n, 1)))()
        buf = ctypes.cast(unpacked.ctypes.data if hasattr(unpacked, "ctypes") else unpacked,
                          ctypes.POINTER(ctypes.c_int32))
        self._check(self.lib.rmc_fingerprints(self.h, buf, stride, n, fps))
        return [(fps[2 * i], fps[2 * i + 1]) for i in range(n)]

    def seen_contains(self, fps: Sequence[Tuple[int, int]]) -> List[bool]:
        """Membership of each fingerprint in the seen set (TLC's FPSet)."""
        n = len(fps)
        arr = (ctypes.c_uint64 * (2 * max(n, 1)))(*[w for f in fps for w in f])
        out = (ctypes.c_uint8 * max(n, 1))()
        self._check(self.lib.rmc_seen_contains(self.h, arr, n, out))
        return [bool(out[i]) for i in range(n)]

    def eval_invariant(self, state: dict, name: str) -> Optional[bool]:
        """True / False, or None for a TLC evaluation error."""
        bit = INVARIANT_BY_BIT.index("Inv" if name == "LeaderHasAllCommittedEntries" else name)
        v = ctypes.c_int32()
        rc = self.lib.rmc_eval_invariant(self.h, self._unpacked(state), bit, ctypes.byref(v))
        if rc == RMC_EVAL_ERROR:
            return None
        self._check(rc)
        return bool(v.value)
