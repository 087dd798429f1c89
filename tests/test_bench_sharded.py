"""bench.py's configs[3] leg at N > 1 (c4_child) on CPU with gloo, world_size 2: every decision the
ranks must take together -- the budget (minimum over ranks), the stop after a level (any rank's
prediction), a capacity failure raised on every rank in the same level -- and rank 0's report.
The model checker is a stand-in that grows levels x2 and advances a simulated clock, so the
orchestration runs in a second without a GPU; the engine itself is covered by the -m gpu tests."""
import json
import os
import socket
import sys
import types

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_raftmc(clock, fail_at, step_s):
    m = types.ModuleType("raftmc")

    class RmcError(RuntimeError):
        pass

    class Level:
        def __init__(self, n):
            self.new_states, self.status = n, "ok"

    class ModelChecker:
        def __init__(self, cfg):
            self.n, self.level = 1, 1

        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

        def init(self):
            return Level(1)

        def step(self):
            self.level += 1
            if fail_at and self.level == fail_at:
                raise RmcError("RMC_E_MEMORY: frontier ring full (stand-in)")
            clock[0] += step_s * self.n  # a level's time grows with its size
            self.n *= 2
            return Level(self.n)

    m.RmcError, m.ModelChecker = RmcError, ModelChecker
    return m


def _worker(rank, world, port, budgets, fail_at, out):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    import bench
    clock = [0.0]
    sys.modules["raftmc"] = _fake_raftmc(clock, fail_at, 0.5)
    bench.time = types.SimpleNamespace(perf_counter=lambda: clock[0])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    args = types.SimpleNamespace(child_budget=budgets[rank], sharded_out=out)
    bench.c4_child(args, None, bench.WORKLOADS["c4"], rank, world)
    dist.destroy_process_group()


def _run(tmp_path, budgets, fail_at=0):
    out = str(tmp_path / "c4.json")
    mp.spawn(_worker, args=(2, _free_port(), budgets, fail_at, out), nprocs=2, join=True)
    with open(out) as f:
        return json.load(f)


def test_c4_leg_stops_together_on_the_budget(tmp_path):
    # level k+1 takes 0.5 * 2^(k-1) s: levels 2..7 end at 31.5 s; the 8th is predicted past 40 s
    r = _run(tmp_path, [60.0, 40.0])
    assert r["levels_completed"] == 7 and r["distinct_states"] == 127 and r["last_level_states"] == 64
    assert r["stopped"].startswith("time budget (40 s)")
    assert r["seconds"] == pytest.approx(31.5) and r["n_gpus"] == 2


def test_c4_leg_stops_together_on_capacity(tmp_path):
    r = _run(tmp_path, [120.0, 120.0], fail_at=5)
    assert r["levels_completed"] == 4 and r["stopped"].startswith("RMC_E_MEMORY")


def test_c4_leg_skipped_when_any_rank_lacks_time(tmp_path):
    r = _run(tmp_path, [120.0, 10.0])
    assert "skipped" in r and "levels_completed" not in r


def _measure_worker(rank, world, port, out):
    """bench.measure at N = 2 with a stand-in checker whose exhaustion takes 1 s on rank 0 and 3 s on
    rank 1 (a simulated clock): W warmup steps untimed, exactly K timed, the max over ranks."""
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    import bench
    clock = [0.0]
    calls = {"run": 0, "timing": []}

    class Res:
        distinct, status, levels = 7, "done", ["levels"]

    class MC:
        def reset(self):
            pass

        def set_timing(self, m):
            calls["timing"].append(m)

        def run(self):
            calls["run"] += 1
            clock[0] += 1.0 + 2.0 * rank
            return Res()

    bench.time = types.SimpleNamespace(perf_counter=lambda: clock[0])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res, elapsed, timed, first_s = bench.measure(MC(), 5, 2, world, lambda: None, "t", timing_every=2,
                                                 report_steps=False)
    dist.destroy_process_group()
    if rank == 0:
        with open(out, "w") as f:
            json.dump({"elapsed": elapsed, "timed": len(timed), "first": first_s, "runs": calls["run"],
                       "timing": calls["timing"]}, f)


def test_bench_measure_takes_the_slowest_rank(tmp_path):
    out = str(tmp_path / "m.json")
    mp.spawn(_measure_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r = json.load(open(out))
    assert r["runs"] == 7 and r["first"] == 1.0
    assert r["elapsed"] == pytest.approx(15.0)  # rank 1: 5 timed steps of 3 s
    assert r["timed"] == 3 and r["timing"] == [2, 0, 2, 0, 2]
