"""TEST INFRASTRUCTURE: the multi-GPU sharding protocol of the product (DESIGN.md section 7,
rmc_engine.hip step_sharded) restated over the Python oracle, one process per shard,
exchanging through torch.distributed (gloo on CPU).

Levels are block-cyclic: global index g of a level lives on rank (g // B) % W.  Round c of a
level expands global block c*W + rank on every rank, so rounds follow the level's order.  Each
successor goes to its fingerprint's owner with its global key (parent's global index, rank
among the parent's successors in TLC order); the owner drops fingerprints already seen and
elects the smallest key per new one (TLC -workers 1 meets that successor first); verdicts come
back, each rank keeps its winners in TLC order, and the winners go to the ranks owning their
global next-level indices, appended source-major -- the level's order."""
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
    """Per-level new-state counts and total generated; identical to TLC's single-worker BFS."""
    W, rank = dist.get_world_size(), dist.get_rank()
    B = chunk
    owner = lambda f: (f >> 40) % W  # noqa: E731
    s0 = R.init_state(cfg)
    f0 = fp64(R.canonical(cfg, s0))
    seen = set([f0]) if owner(f0) == rank else set()
    frontier = [s0] if rank == 0 else []  # Init: global index 0 -> block 0 -> rank 0
    levels, generated = [1], 1
    while True:
        Fg = torch.tensor([len(frontier)])
        dist.all_reduce(Fg)
        rounds = (int(Fg) + B * W - 1) // (B * W)
        nxt, gen, new = [], 0, 0
        for c in range(rounds):
            gblk = (c * W + rank) * B
            succ = []  # (fp, key, state), TLC order
            for i, st in enumerate(frontier[c * B:(c + 1) * B]):
                for r, (_, t) in enumerate(R.successors(cfg, st)):
                    succ.append((fp64(R.canonical(cfg, t)), ((gblk + i) << 8) | r, t))
            by_owner = [[i for i, (f, _, _) in enumerate(succ) if owner(f) == d] for d in range(W)]
            recv = a2a_ints([[v for i in idx for v in (succ[i][0], succ[i][1])] for idx in by_owner])
            best = {}
            for src in range(W):
                for f, k in zip(recv[src][0::2], recv[src][1::2]):
                    if f not in seen and (f not in best or k < best[f]):
                        best[f] = k
            flags = [[1 if best.get(f) == k else 0 for f, k in zip(recv[src][0::2], recv[src][1::2])]
                     for src in range(W)]
            seen.update(best)
            back = a2a_ints(flags)
            win = [False] * len(succ)
            for d in range(W):
                for i, w in zip(by_owner[d], back[d]):
                    win[i] = bool(w)
            mine = [succ[i][2] for i in range(len(succ)) if win[i]]  # TLC order
            counts = torch.zeros(W + 1, dtype=torch.int64)
            counts[rank] = len(mine)
            counts[W] = len(succ)
            dist.all_reduce(counts)
            x0 = new + int(counts[:rank].sum())
            out = [[] for _ in range(W)]
            for j, st in enumerate(mine):
                out[((x0 + j) // B) % W].append(R.state_to_json(st))
            got = a2a_objs(out)
            for src in range(W):  # source-major: the level's order
                nxt.extend(R.state_from_json(js) for js in got[src])
            new += int(counts[:W].sum())
            gen += int(counts[W])
        generated += gen
        if new == 0:
            return levels, generated
        levels.append(new)
        frontier = nxt
