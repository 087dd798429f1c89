"""TEST INFRASTRUCTURE: the multi-GPU sharding protocol of the product (DESIGN.md section 7,
rmc_engine.hip step_sharded) restated over the Python oracle, one process per shard,
exchanging through torch.distributed (gloo on CPU).

Per BFS level and chunk c: every rank expands parents [c*C, (c+1)*C) of its frontier in TLC
order, partitions the successors by owner(fingerprint) keeping their order, all-to-all of
fingerprints, owners elect the first (source rank, index) per fingerprint not yet seen,
all-to-all of winner flags back, winners' states all-to-all to their owners, owners append
them source-major to the next level and mark them seen."""
import hashlib
import json

import torch
import torch.distributed as dist

import raft_ref as R


def fp64(canon) -> int:
    return int.from_bytes(hashlib.blake2b(repr(canon).encode(), digest_size=8).digest(), "little") >> 1


def a2a_counts(counts):
    W = len(counts)
    out = torch.empty(W, dtype=torch.int64)
    dist.all_to_all_single(out, torch.tensor(counts, dtype=torch.int64))
    return out.tolist()


def a2a_ints(per_peer):
    """all-to-all of variable-length int64 lists"""
    send_counts = [len(x) for x in per_peer]
    recv_counts = a2a_counts(send_counts)
    flat = torch.tensor([v for x in per_peer for v in x] or [0], dtype=torch.int64)[:sum(send_counts)]
    out = torch.empty(sum(recv_counts), dtype=torch.int64)
    dist.all_to_all_single(out, flat, output_split_sizes=recv_counts, input_split_sizes=send_counts)
    res, k = [], 0
    for c in recv_counts:
        res.append(out[k:k + c].tolist())
        k += c
    return res


def a2a_objs(per_peer):
    """all-to-all of lists of JSON-able objects, as bytes"""
    blobs = [json.dumps(x).encode() for x in per_peer]
    ints = [list(b) for b in blobs]
    got = a2a_ints(ints)
    return [json.loads(bytes(x).decode()) if x else [] for x in got]


def sharded_bfs(cfg: R.Config, chunk: int):
    W, rank = dist.get_world_size(), dist.get_rank()
    owner = lambda f: (f >> 40) % W  # noqa: E731
    s0 = R.init_state(cfg)
    f0 = fp64(R.canonical(cfg, s0))
    seen = set()
    frontier = []
    if owner(f0) == rank:
        seen.add(f0)
        frontier.append(s0)
    levels, generated = [1], 1
    while True:
        n_chunks = torch.tensor([(len(frontier) + chunk - 1) // chunk])
        dist.all_reduce(n_chunks, op=dist.ReduceOp.MAX)
        nxt = []
        gen = 0
        for c in range(int(n_chunks.item())):
            succ = []
            for st in frontier[c * chunk:(c + 1) * chunk]:
                for _, t in R.successors(cfg, st):
                    succ.append((fp64(R.canonical(cfg, t)), t))
            gen += len(succ)
            by_owner = [[i for i, (f, _) in enumerate(succ) if owner(f) == d] for d in range(W)]
            recv = a2a_ints([[succ[i][0] for i in idx] for idx in by_owner])
            flags, elected = [], set()
            for src in range(W):  # source-major = election order
                fl = []
                for f in recv[src]:
                    win = f not in seen and f not in elected
                    if win:
                        elected.add(f)
                    fl.append(1 if win else 0)
                flags.append(fl)
            back = a2a_ints(flags)
            out_states = [[R.state_to_json(succ[i][1]) for i, w in zip(by_owner[d], back[d]) if w] for d in range(W)]
            got = a2a_objs(out_states)
            for src in range(W):
                for js in got[src]:
                    st = R.state_from_json(js)
                    seen.add(fp64(R.canonical(cfg, st)))
                    nxt.append(st)
        tot = torch.tensor([gen, len(nxt)])
        dist.all_reduce(tot)
        generated += int(tot[0])
        if int(tot[1]) == 0:
            return levels, generated
        levels.append(int(tot[1]))
        frontier = nxt
