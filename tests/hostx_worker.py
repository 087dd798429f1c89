"""One rank of a multi-process sharded run over the host-staged transport (test helper).

usage: python hostx_worker.py SPEC_JSON -- SPEC = {"rank", "world", "port", "cfg": ModelConfig
keywords, "inject": RMC_FAULT_INJECT value or null, "out": result path}.  The ranks meet in a
torch.distributed gloo group on 127.0.0.1, install raftmc.HostTransport (include/rmc.h
rmc_transport) and run the configuration with world_size = W on device 0 -- separate processes,
separate contexts, the collectives of step_sharded between them through host memory."""
import datetime
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tla-raft_amd"))

import torch.distributed as dist  # noqa: E402

import raftmc  # noqa: E402


def main():
    spec = json.loads(sys.argv[1])
    r, W = spec["rank"], spec["world"]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{spec['port']}", rank=r, world_size=W,
                            timeout=datetime.timedelta(seconds=spec.get("timeout", 120)))
    raftmc.HostTransport().install()
    if spec.get("inject"):
        os.environ["RMC_FAULT_INJECT"] = spec["inject"]
    out = {"rank": r}
    try:
        cfg = dict(spec["cfg"])
        if os.environ.get("RMC_TEST_DEVICE_LEVELS"):  # (debugging: levels per host round trip)
            cfg["device_levels"] = int(os.environ["RMC_TEST_DEVICE_LEVELS"])
        mc = raftmc.ModelChecker(raftmc.ModelConfig(rank=r, world_size=W, device=0, **cfg))
        os.environ.pop("RMC_FAULT_INJECT", None)
        try:
            res = mc.run()
            out.update(status=res.status, generated=res.generated, distinct=res.distinct, depth=res.depth,
                       queue=res.queue, violated=res.violated, trace_len=res.trace_len,
                       levels=[[ls.level, ls.expanded, ls.generated, ls.new_states, ls.queue, ls.total_generated,
                                ls.total_distinct, ls.status] for ls in res.levels])
            if spec.get("trace"):
                out["trace"] = [[list(k) if k else None, st] for k, st in mc.trace()]
        finally:
            mc.close()
    except raftmc.RmcError as e:
        out["error"] = str(e)
    with open(spec["out"], "w") as f:
        json.dump(out, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
