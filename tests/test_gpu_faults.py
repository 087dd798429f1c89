"""Failure agreement of the sharded BFS (rmc_engine.hip step_sharded).

A shard that cannot allocate a buffer of the round must not leave its peers waiting in a
collective: it records the failure, keeps taking part in every exchange, and the next gathered
count matrix or all-reduce stops every shard with RMC_E_MEMORY in the same round (in an RCCL run,
every rank raises).  RMC_FAULT_INJECT="site,shard,round,level" (read at rmc_create) makes the
allocation at one site fail on one shard, as a full device would:
  1 send buffer  2 receive buffer (forced to grow)  3 owner seen set / election table  4 outbox
  5 regrouped winners  6 winner inbox (forced to grow)  7 next-level append  8 entering the layout
The run must then raise RMC_E_MEMORY (not hang, not crash), and a run without the hook on the same
checker configuration must still give the golden counts.  Virtual shards run the identical
protocol in one process; the one-rank RCCL communicator runs its collectives through RCCL."""
import json
import os

import pytest

import raftmc
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN, "levels.json")) as _f:
    LEVELS = json.load(_f)
G = LEVELS["n3_v1_e2_r3"]  # BASELINE configs[1]: 223,437 states, 37 levels


def run(inject=None, **kw):
    if inject is not None:
        os.environ["RMC_FAULT_INJECT"] = inject
    try:
        mc = raftmc.ModelChecker(raftmc.ModelConfig(n_servers=G["n"], n_vals=G["V"], max_election=G["E"],
                                                    max_restart=G["R"], **kw))
    finally:
        os.environ.pop("RMC_FAULT_INJECT", None)
    try:
        return mc.run(), None
    except raftmc.RmcError as e:
        return None, str(e)
    finally:
        mc.close()


def golden(res):
    return (res.status, res.distinct, res.generated, res.depth) == ("done", G["distinct"], G["generated"], G["depth"])


VIRT = dict(virtual_shards=3, chunk_successors=3000, shard_min_states=1)


@pytest.mark.parametrize("site", [1, 2, 3, 4, 6, 7])
def test_virtual_shards_agree_on_allocation_failure(site):
    """The failing shard is shard 1 of 3, in round 1 of level 14 (2,802 parents: 15 rounds of 3 blocks of
    64 parents)."""
    res, err = run(f"{site},1,1,14", **VIRT)
    assert res is None and err is not None, f"site {site}: the injected failure did not stop the run"
    assert "RMC_E_MEMORY" in err and "injected" in err, err
    res, err = run(None, **VIRT)
    assert err is None and golden(res)


def test_virtual_shards_agree_on_regroup_failure():
    """Site 5 only runs when a source's winners span more blocks than there are shards (the regrouped
    copy): some level of the run must reach it, and there the failure stops every shard."""
    hit = 0
    for level in range(10, 31):
        res, err = run(f"5,1,1,{level}", virtual_shards=2, chunk_successors=600, shard_min_states=1)
        if err is not None:
            assert "RMC_E_MEMORY" in err and "injected" in err, err
            hit += 1
        else:
            assert golden(res), level
    assert hit > 0


def test_failure_entering_the_sharded_layout():
    """Site 8: the transition from replicated to sharded levels fails on shard 0; the sharded
    level's first collective carries it."""
    res, err = run("8,0,0", virtual_shards=2, chunk_successors=3000, shard_min_states=40)
    assert res is None and "RMC_E_MEMORY" in err and "injected" in err, err


@pytest.mark.parametrize("site", [1, 2, 3, 4, 6, 7])
def test_rccl_one_rank_agrees_on_allocation_failure(site):
    """The same agreement through the RCCL collectives (gathered matrix, all-reduce)."""
    kw = dict(world_size=1, rank=0, comm_unique_id=raftmc.comm_unique_id(), chunk_successors=3000,
              shard_min_states=1)
    res, err = run(f"{site},0,1,14", **kw)
    assert res is None and err is not None and "RMC_E_MEMORY" in err and "injected" in err, (site, err)
    kw["comm_unique_id"] = raftmc.comm_unique_id()
    res, err = run(None, **kw)
    assert err is None and golden(res)


def test_resume_rejects_a_corrupt_checkpoint(tmp_path):
    """rmc_resume checks every data section (seen set, ring words, offsets, trace) against the
    checksum rmc_checkpoint wrote, and the frontier offsets against the record bounds, before the
    kernels can index the ring with them."""
    path = str(tmp_path / "c2.ckpt")
    cfg = raftmc.ModelConfig(n_servers=G["n"], n_vals=G["V"], max_election=G["E"], max_restart=G["R"])
    with raftmc.ModelChecker(cfg) as mc:
        mc.init()
        for _ in range(12):
            mc.step()
        mc.checkpoint(path)
    data = bytearray(open(path, "rb").read())
    with raftmc.ModelChecker(cfg) as mc:  # the intact file resumes and finishes with the golden counts
        mc.resume(path)
        res = mc.run()
        assert golden(res)
    for at in (len(data) // 2, len(data) - 200):  # the seen set; the trace near the end
        bad = bytearray(data)
        bad[at] ^= 0x5A
        bp = str(tmp_path / f"bad{at}.ckpt")
        open(bp, "wb").write(bytes(bad))
        with raftmc.ModelChecker(cfg) as mc:
            with pytest.raises(raftmc.RmcError, match="corrupt|inconsistent"):
                mc.resume(bp)
