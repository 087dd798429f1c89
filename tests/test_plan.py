"""Sharded round bookkeeping (tla-raft_amd/csrc/rmc_plan.h), compiled for the host with g++.

The engine's RCCL branch and its virtual-shard branch derive every offset of the round's three
all-to-all-v payloads from rmc_plan.h; tests/plan_test.cpp simulates those payloads at W = 1..8 on
host arrays and checks that the RCCL ranks' posted sends/receives equal the virtual copies, that
verdicts come back to their slots, that winners land on their block-cyclic owners in global order,
and that receive growth is decided identically on every rank (no W > 1 path can run here)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_sharded_round_plan_w1_to_w8(tmp_path):
    exe = tmp_path / "plan_test"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-Wall", "-I", os.path.join(ROOT, "tla-raft_amd", "csrc"),
                           os.path.join(ROOT, "tests", "plan_test.cpp"), "-o", str(exe)])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "plan ok" in r.stdout
