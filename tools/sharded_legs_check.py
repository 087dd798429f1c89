#!/usr/bin/env python3
"""Run bench.py's two sharded legs (the children it starts at N > 1) on this one GPU as a one-rank
RCCL communicator: the orchestration (ports, budgets, time limits, result files) end to end.
usage: RANK=0 WORLD_SIZE=1 MASTER_PORT=29650 python tools/sharded_legs_check.py OUT.json"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

raft, c4 = bench.run_sharded_children(argparse.Namespace())
json.dump({"at_scale_sharded": raft, "at_scale_sharded_configs3": c4}, open(sys.argv[1], "w"), indent=1)
print(json.dumps({"at_scale_sharded": raft, "at_scale_sharded_configs3": c4}))
