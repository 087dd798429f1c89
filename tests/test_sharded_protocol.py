"""Multi-process (gloo, world_size 2 and 3) test of the sharding protocol the multi-GPU engine uses,
restated over the oracle (tests/sharded_model.py): the block-cyclic, owner-elected BFS must reach
exactly the golden per-level counts of TLC's single-worker order."""
import json
import os
import socket

import pytest
import torch.multiprocessing as mp

from conftest import GOLDEN


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cfg_kw, chunk, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "oracle"))
    import torch.distributed as dist
    import raft_ref as R
    import sharded_model
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    levels, gen = sharded_model.sharded_bfs(R.Config(**cfg_kw), chunk)
    if rank == 0:
        q.put((levels, gen))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name,chunk", [("n3_v1_e1_r3", 7), ("n2_v1_e2_r3", 5), ("n3_v2_e1_r3", 40)])
def test_sharded_protocol_matches_golden(name, chunk, world):
    g = json.load(open(os.path.join(GOLDEN, "levels.json")))[name]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    kw = dict(n=g["n"], V=g["V"], max_election=g["E"], max_restart=g["R"])
    procs = [ctx.Process(target=_worker, args=(r, world, port, kw, chunk, q)) for r in range(world)]
    for p in procs:
        p.start()
    levels, gen = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
    assert levels == g["levels"] and gen == g["generated"]
