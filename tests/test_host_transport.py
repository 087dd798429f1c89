"""raftmc.HostTransport on the CPU: the three collectives of include/rmc.h's rmc_transport, called
through their C function pointers as librmc.so calls them, between two gloo processes (world 2)."""
import ctypes
import os
import socket
import sys

import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(r, W, port, q):
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tla-raft_amd"))
    import torch.distributed as dist
    import raftmc
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=r, world_size=W)
    c = raftmc.HostTransport()._c
    u64 = ctypes.c_uint64
    v = (u64 * 3)(1 + r, 2, 5 * r)
    rs = c.allreduce_u64(None, v, 3, 0)
    m = (u64 * 2)(7 * r, 1)
    rm = c.allreduce_u64(None, m, 2, 1)
    row, out = (u64 * 2)(r, 100 + r), (u64 * (2 * W))()
    rg = c.allgather_u64(None, row, 2, out)
    # rank r sends r + 1 + p bytes of value 16 r + p to every peer p (none to itself), at offsets laid
    # out in reverse rank order, and receives p + 1 + r bytes from each peer at gapped offsets
    sb = [0 if p == r else r + 1 + p for p in range(W)]
    rb = [0 if p == r else p + 1 + r for p in range(W)]
    so, at = [0] * W, 0
    for p in reversed(range(W)):
        so[p], at = at, at + sb[p]
    ro, at = [0] * W, 0
    for p in range(W):
        ro[p], at = at + 3, at + 3 + rb[p]
    send = (ctypes.c_uint8 * max(1, sum(sb)))()
    for p in range(W):
        for i in range(sb[p]):
            send[so[p] + i] = 16 * r + p
    recv = (ctypes.c_uint8 * (at + 1))()
    ra = c.alltoallv(None, ctypes.cast(send, ctypes.c_void_p), (u64 * W)(*so), (u64 * W)(*sb),
                     ctypes.cast(recv, ctypes.c_void_p), (u64 * W)(*ro), (u64 * W)(*rb))
    got = {p: list(recv[ro[p]:ro[p] + rb[p]]) for p in range(W) if p != r}
    q.put((r, rs, list(v), rm, list(m), rg, list(out), ra, got))
    dist.destroy_process_group()


def test_host_transport_collectives():
    W = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, W, port, q)) for r in range(W)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(W))
    for p in ps:
        p.join(60)
    for r, rs, v, rm, m, rg, out, ra, got in res:
        assert (rs, rm, rg, ra) == (0, 0, 0, 0)
        assert v == [sum(1 + k for k in range(W)), 2 * W, 5 * sum(range(W))]
        assert m == [7 * (W - 1), 1]
        assert out == [x for k in range(W) for x in (k, 100 + k)]
        assert got == {p: [16 * p + r] * (p + 1 + r) for p in range(W) if p != r}

