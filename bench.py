#!/usr/bin/env python3
"""bench.py -- distinct states/sec of the MI355X model checker on BASELINE.json's workload.

One "step" = one complete breadth-first exhaustion of the workload's state space from
Init (TLC's whole myrun.sh run, minus JVM start-up): successor generation, symmetry +
VIEW fingerprinting, seen-set dedup in TLC -workers 1 order, invariant checks.  The
state space starts empty and every step re-explores it (rmc_reset keeps only device
buffers; inputs = the compiled spec tables, resident in HBM).

Workload at N=1: BASELINE.json configs[1] ("3 servers, 1 value, MaxTerm=2, MaxLogLen=2 on
one MI355X") = Raft.tla with Servers={s1,s2,s3}, Vals={v1}, MaxElection=2, MaxRestart=3,
SYMMETRY symmServers, VIEW view, INVARIANT Inv, -deadlock (MaxTerm is
MaxElection, MaxLogLen is |Vals|+1).  The `at_scale` key exhausts configs[0]/[2] -- Raft.cfg as
shipped (3 servers, 2 values, MaxElection 3: 10,946,499,503 distinct states, depth 72) -- on the
same GPU and reports its wall time and distinct states/s (N = 1 only).

N>1 (torchrun, one process per GPU): the same workload is exhausted ONCE by all ranks
together through the engine's multi-GPU mode: levels below
rmc_config.shard_min_states (default 2^20 states) are expanded whole on every rank --
replicated, no exchange, TLC order -- and from the first level that reaches it the seen
set and frontier are sharded by fingerprint owner with one RCCL exchange of fingerprints /
winner flags / winner records per chunk.  configs[1]'s levels never exceed ~2*10^4 states,
so at this workload every level is replicated and the whole-node rate is the one-GPU rate
(a per-level exchange would cost more than the level: tools/shard_timing.py).  value =
distinct states of the run / max-over-ranks time, scaling "strong" (total work fixed).  If
the RCCL communicator fails to initialise, each rank exhausts its own copy instead and the
line says "replicas" with the error.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tla-raft_amd"))

WORKLOADS = {
    "raftcfg": dict(n=3, V=2, E=3, R=3, desc="BASELINE configs[0]/[2]: Raft.cfg as shipped -- Raft.tla, 3 servers, "
                                             "2 values, MaxElection 3, MaxRestart 3, SYMMETRY+VIEW, INVARIANT Inv, "
                                             "-deadlock"),
    "c2": dict(n=3, V=1, E=2, R=3, desc="BASELINE configs[1]: Raft.tla, 3 servers, 1 value, MaxElection(=MaxTerm)=2, "
                                         "MaxRestart=3, MaxLogLen=2, SYMMETRY+VIEW, INVARIANT Inv, -deadlock"),
    "c4": dict(n=5, V=1, E=3, R=3, desc="BASELINE configs[3]: Raft.tla, 5 servers, 1 value, MaxElection(=MaxTerm)=3, "
                                         "MaxRestart=3, SYMMETRY+VIEW, INVARIANT Inv, -deadlock"),
    "n3v2e2": dict(n=3, V=2, E=2, R=3, desc="Raft.tla, 3 servers, 2 values, MaxElection=2, MaxRestart=3 "
                                             "(18.5M states; between configs[1] and configs[2])"),
}

# HBM peak from /opt/skills/guides/MI355X_MICROARCH.md (spec 8.0 TB/s)
HBM_PEAK_GBS = 8000.0
PHASES = ["expand_count", "expand_hash", "dedup", "materialize", "exchange", "other"]
TIMED_PHASES = 1 << PHASES.index("expand_hash")  # HIP-event timing of the dominant kernel only
TIMING_EVERY = 8


def alg_bytes(phase, F, G, N, S, CCWB, slot_bytes=16, SWB=32, split=False, CTXB=112, Gself=0):
    """Algorithmic HBM bytes of one phase of the fused single-GPU level (DESIGN.md "Kernels"):
    F parents of S-byte records (S = the run's average packed record: CCWB core bytes + message
    ids), G generated successors, N new states; SWB = staging bytes per successor (the acting row),
    slot_bytes = seen-set slot (16 full, 8 compact), CTXB = a split chunk's hash context per parent
    (ctx_bytes).  split: the host-driven chunk's expansion only stages (k_expand_items); the
    fingerprints, probe and election run in k_hash_probe ("probe").  Gself: of the G successors, the
    self-loops a split chunk sets apart (rmc_level_stats.self_loops): never staged, fingerprinted or probed."""
    if phase == "expand_hash" and split:  # k_expand_items: parents in, count + |msgs| + hash context out,
        # the staged rows of the successors other than self-loops out
        return F * S + F * 8 + F * CTXB + (G - Gself) * SWB
    if phase == "expand_hash":   # k_expand_items<FUSE>: parents in, count + |msgs| out; per successor other than
        # a self-loop: staged row + fp + election slot, one seen-set probe (a self-loop: its slot word only); per
        # new fingerprint at least one election (16-B slot, 8-B word, count)
        return F * S + F * 8 + (G - Gself) * (SWB + 16 + 4 + slot_bytes) + Gself * 4 + N * (16 + 8 + 4)
    if phase == "probe":         # k_hash_probe: per parent its count and hash context; per successor its staged
        # row in, fingerprint + verdict out, one seen-set probe; per new fingerprint at least one election
        # (16-B slot, 8-B word, count)
        return F * (4 + CTXB) + (G - Gself) * (SWB + 16 + 4 + slot_bytes) + N * (16 + 8 + 4)
    if phase == "insert":        # k_insert_winners: per parent its count; per successor its slot word; per new
        # state its election word, fingerprint, seen-set insert and verdict
        return F * 4 + G * 4 + N * (8 + 16 + slot_bytes + 4)
    if phase == "dedup":         # k_wincount: per parent successor count, packed winner count (read + re-arm),
        # |msgs|; out winner count and the two scans
        return F * (4 + 4 + 4 + 4 + 4 + 4 + 4)
    if phase == "materialize":   # k_commit: per parent counts/offsets + its record; per slot of a parent with
        # winners its election slot + word; per new state: staged row + fp in, seen insert, trace, offset, record out
        return F * (4 * 6) + F * S + G * (4 + 8) + N * (SWB + 16 + slot_bytes + 8 + 2 + 8 + S)
    return 0


def survey_roofline(levels, S, wall_s, probes_per_s):
    """SURVEY.md 8(d)'s whole-run model: B_L = F_L*S + G_L*64 + N_{L+1}*(S + 16) algorithmic bytes per
    level (one 64-B bucket probe per generated successor), roofline time = sum_L G_L*64 / BW_rand +
    (F_L*S + N_{L+1}*(S + 16)) / BW_stream with BW_stream = 8 TB/s and BW_rand = the measured random
    64-B probe rate of this GPU (rmc_probe_peak, HBM-resident table).  frac = roofline time / wall."""
    F = sum(ls.expanded for ls in levels)
    G = sum(ls.generated for ls in levels[1:])
    N = sum(ls.new_states for ls in levels[1:])
    rand_b = G * 64
    stream_b = F * S + N * (S + 16)
    out = {"bytes": int(rand_b + stream_b), "achieved_GBps": round((rand_b + stream_b) / wall_s / 1e9, 2),
           "record_bytes_avg": round(S, 2)}
    if probes_per_s:
        bw_rand = probes_per_s * 64
        t = rand_b / bw_rand + stream_b / (HBM_PEAK_GBS * 1e9)
        out.update({"bw_rand_GBps": round(bw_rand / 1e9, 1), "roofline_s": round(t, 6), "wall_s": round(wall_s, 6),
                    "frac": round(t / wall_s, 4)})
    return out


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(w, budget_s=12.0):
    """oracle/raft_mt.c -- the C restatement of Raft.tla + TLC -workers 1 BFS semantics, level-
    synchronous on every host core this process may use -- exhausting the same workload."""
    so = os.path.join(ROOT, "oracle", "build", "libraft_mt.so")
    if not os.path.exists(so):
        return None
    lib = ctypes.CDLL(so)
    lib.orc_mt_run.argtypes = [ctypes.c_int] * 5 + [ctypes.POINTER(ctypes.c_uint64)] * 2 + [ctypes.POINTER(ctypes.c_int)]
    # the host cores this job may use: the box's share (OMP_NUM_THREADS is set to it on the GPU
    # boxes; the affinity mask there shows the whole machine)
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))
    runs, states = 0, 0
    d, g, dep = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        rc = lib.orc_mt_run(w["n"], w["V"], w["E"], w["R"], threads, ctypes.byref(d), ctypes.byref(g), ctypes.byref(dep))
        assert rc == 0
        states += d.value
        runs += 1
    dt = time.perf_counter() - t0
    return {"value": states / dt, "unit": "distinct states/s", "cores": threads, "cpu_model": cpu_model(),
            "kind": "port",
            "sample": f"{runs} full exhaustions ({d.value} distinct, {g.value} generated, depth {dep.value}) of the "
                      f"same workload by oracle/raft_mt.c on {threads} threads (C restatement of Raft.tla, exact "
                      f"canonical forms, level-synchronous first-wins BFS; not TLC: no JVM/tla2tools.jar on the "
                      f"box), {dt:.1f} s"}


SHARDED_TIMEOUT_S = 420  # the multi-GPU Raft.cfg exhaustion (child processes) must finish within this
SHARDED_TOTAL_S = 480    # ... and both sharded legs (Raft.cfg, then configs[3] as deep as it goes) within this
C4_BUDGET_S = 120        # levels of configs[3] are started until this much time has passed
C4_ONE_GPU_LEVELS = 30   # configs[3] on one MI355X, single-GPU path, 48 GB seen set / 200 GB ring: levels 1-30


def xgmi_model(levels, world, shard_min=1 << 20):
    """SURVEY.md 8(d)'s multi-GPU addition, for the engine's exchange: from
    the first level of >= shard_min parents on, every successor crosses to its fingerprint's owner
    as a 24-B item {fp, key} and comes back as a 4-B verdict, and every winner's record (new_bytes)
    plus a 16-B sidecar goes to the owner of its next-level index; (W-1)/W of it leaves the GPU."""
    if world < 2:
        return 0
    total, on = 0, False
    for ls in levels:
        on = on or ls.expanded >= shard_min
        if on:
            total += ls.generated * (24 + 4) + ls.new_bytes + 16 * ls.new_states
    return int(total * (world - 1) / world)


def sharded_child(args):
    """One rank of the multi-GPU Raft.cfg exhaustion (configs[2] at N GPUs), run in a child process of
    each bench rank before the bench touches the GPU: the levels are sharded over the N GPUs (RCCL,
    block-cyclic frontier, fingerprint-owner seen set) from the first level of
    >= 2^20 states.  Rank 0 writes the result to args.sharded_out."""
    import torch
    import torch.distributed as dist
    import raftmc
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # a port of its own per child (the Raft.cfg child's store may still hold its port when the next starts)
    port = int(os.environ.get("MASTER_PORT", "29500")) + (17 if args.child_workload == "raftcfg" else 19)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    idt = torch.zeros(128, dtype=torch.uint8)
    if rank == 0:
        idt = torch.tensor(list(raftmc.comm_unique_id()), dtype=torch.uint8)
    dist.broadcast(idt, 0)
    w = WORKLOADS[args.child_workload]
    cfg = raftmc.ModelConfig(n_servers=w["n"], n_vals=w["V"], max_election=w["E"], max_restart=w["R"],
                             invariants=("Inv",), check_deadlock=False, device=local, rank=rank, world_size=world,
                             comm_unique_id=bytes(idt.tolist()))
    if args.child_workload == "c4":
        # per GPU: a 48 GB seen-set shard (6.4 G compact slots) and a 160 GB frontier ring, ~80 GB
        # left for the rounds' buffers; the default gives the seen set half of HBM, far more than
        # this configuration's levels fill before the ring does
        cfg.seen_mem_bytes, cfg.frontier_mem_bytes = 48 << 30, 160 << 30
        cfg.chunk_successors = 1 << 27  # rounds of 2^27 slots: the rounds' buffers stay within the ~80 GB left
        c4_child(args, cfg, w, rank, world)
        dist.destroy_process_group()
        return
    with raftmc.ModelChecker(cfg) as mc:
        dist.barrier()
        t0 = time.perf_counter()
        res = mc.run()
        dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    if rank == 0:
        gold = {}
        gpath = os.path.join(ROOT, "tests", "golden", "levels_prefix.json")
        if os.path.exists(gpath):
            gold = json.load(open(gpath)).get("n3_v2_e3_r3", {})
        got = [ls.new_states for ls in res.levels]
        out = {"workload": w["desc"], "n_gpus": world, "parallelism": f"rccl-{world}: block-cyclic levels, "
               "fingerprint-owner seen set, TLC-order global-key election, from the first level of >= 2^20 states",
               "distinct_states": res.distinct, "states_generated": res.generated, "depth": res.depth,
               "verdict": "Inv holds" if res.status == "done" else res.status,
               "seconds_to_exhaust": round(dt, 3), "distinct_per_s": round(res.distinct / dt, 1),
               "matches_c_oracle_prefix_levels": (got[:len(gold["levels"])] == gold["levels"]) if gold else None}
        xb = xgmi_model(res.levels, world)
        out["xgmi_bytes_model"] = xb
        out["xgmi_GBps_avg"] = round(xb / dt / 1e9, 2)
        with open(args.sharded_out, "w") as f:
            json.dump(out, f)
    dist.destroy_process_group()


def c4_child(args, cfg, w, rank, world):
    """configs[3] sharded over the N GPUs, level by level, as deep as the node's HBM and the time
    budget allow (its exhaustion is beyond any node: DESIGN.md section 9).  All ranks agree on
    every decision: the budget (minimum over ranks), stopping after a level (any rank past the
    budget), and a capacity failure (the engine raises it on every rank in the same round)."""
    import torch
    import torch.distributed as dist
    import raftmc
    b = torch.tensor([args.child_budget], dtype=torch.float64)
    dist.all_reduce(b, op=dist.ReduceOp.MIN)
    budget = float(b.item())
    out = {"workload": w["desc"], "n_gpus": world, "one_gpu_levels": C4_ONE_GPU_LEVELS}
    if budget < 30:
        out["skipped"] = f"{budget:.0f} s left of the sharded legs' {SHARDED_TOTAL_S} s"
        if rank == 0:
            with open(args.sharded_out, "w") as f:
                json.dump(out, f)
        return
    gold = {}
    gpath = os.path.join(ROOT, "tests", "golden", "levels_prefix.json")
    if os.path.exists(gpath):
        gold = json.load(open(gpath)).get("n5_v1_e3_r3", {})

    def report(levels, stop, dt):  # rank 0, after every level: a child killed at its limit still reports
        k = min(len(levels), len(gold.get("levels", [])))
        out.update({"parallelism": f"rccl-{world}", "levels_completed": len(levels), "distinct_states": sum(levels),
                    "last_level_states": levels[-1], "stopped": stop, "seconds": round(dt, 3),
                    "distinct_per_s": round(sum(levels) / dt, 1) if dt > 0 else None,
                    "matches_c_oracle_prefix_levels": (levels[:k] == gold["levels"][:k]) if k else None,
                    "c_oracle_prefix_levels_compared": k})
        if rank == 0:
            with open(args.sharded_out + ".tmp", "w") as f:
                json.dump(out, f)
            os.replace(args.sharded_out + ".tmp", args.sharded_out)

    levels, stop = [], "exhausted"
    with raftmc.ModelChecker(cfg) as mc:
        dist.barrier()
        t0 = time.perf_counter()
        levels.append(mc.init().new_states)
        tl = time.perf_counter()
        while True:
            try:
                ls = mc.step()
            except raftmc.RmcError as e:  # capacity: every rank raises in the same round
                stop = str(e)[:200]
                break
            if ls.new_states == 0 or ls.status != "ok":
                stop = "exhausted" if ls.status in ("ok", "done") else ls.status
                break
            levels.append(ls.new_states)
            now = time.perf_counter()
            # the next level is predicted from this one's time and growth; stop if it would end
            # past the budget (any rank's view stops all)
            nxt = (now - tl) * (levels[-1] / max(1, levels[-2]))
            tl = now
            report(levels, "in progress (the child's time limit ended the run)", now - t0)
            past = torch.tensor([1 if now - t0 + nxt > budget else 0], dtype=torch.int32)
            dist.all_reduce(past, op=dist.ReduceOp.MAX)
            if int(past.item()):
                stop = f"time budget ({budget:.0f} s): the next level was predicted past it"
                break
        dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    report(levels, stop, float(t.item()))


def run_child(args, workload, timeout_s, budget_s=0.0):
    """Start this rank's sharded child for `workload` (before this process initialises the GPU), wait
    for it with a time limit, and return rank 0's result (or what went wrong)."""
    import subprocess
    import tempfile
    rank = int(os.environ.get("RANK", "0"))
    out = os.path.join(tempfile.gettempdir(), f"rmc_sharded_{workload}_{os.environ.get('MASTER_PORT', '0')}.json")
    if rank == 0 and os.path.exists(out):
        os.remove(out)
    cmd = [sys.executable, os.path.abspath(__file__), "--sharded-child", "--sharded-out", out,
           "--child-workload", workload, "--child-budget", str(budget_s)]
    t0 = time.perf_counter()
    p = subprocess.Popen(cmd, stdout=sys.stderr, stderr=sys.stderr)
    try:
        rc = p.wait(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        p.kill()
        p.wait()
        err = {"error": f"timed out after {timeout_s:.0f} s", "wall_s": round(time.perf_counter() - t0, 1)}
        if rank == 0 and os.path.exists(out):  # what the child reported before its limit (configs[3])
            with open(out) as f:
                err.update(json.load(f))
        return err if rank == 0 else None
    if rank != 0:
        return None
    if rc != 0 or not os.path.exists(out):
        return {"error": f"child exited with {rc}", "wall_s": round(time.perf_counter() - t0, 1)}
    with open(out) as f:
        return json.load(f)


def run_sharded_children(args):
    """The two sharded legs at N > 1: Raft.cfg exhausted over the N GPUs (configs[2]), then configs[3]
    as deep as the remaining time allows.  Every rank always starts both children; the configs[3]
    child agrees on its budget across ranks (the minimum), so no rank is left in a collective."""
    t0 = time.perf_counter()
    raft = run_child(args, "raftcfg", SHARDED_TIMEOUT_S)
    left = SHARDED_TOTAL_S - (time.perf_counter() - t0)
    c4 = run_child(args, "c4", max(30.0, left), budget_s=min(C4_BUDGET_S, left - 60.0))
    return raft, c4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe-peak", action="store_true")
    ap.add_argument("--no-scale", action="store_true", help="skip the at-scale reference exhaustion (N=1) / the "
                    "multi-GPU Raft.cfg exhaustion (N>1)")
    ap.add_argument("--sharded-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--sharded-out", default="", help=argparse.SUPPRESS)
    ap.add_argument("--child-workload", default="raftcfg", choices=("raftcfg", "c4"), help=argparse.SUPPRESS)
    ap.add_argument("--child-budget", type=float, default=C4_BUDGET_S, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.sharded_child:
        sharded_child(args)
        return
    sharded = sharded_c4 = None
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and not args.no_scale:
        sharded, sharded_c4 = run_sharded_children(args)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")  # control plane only: barriers and the max-over-ranks time
    torch.cuda.set_device(local)

    import raftmc
    w = WORKLOADS[args.workload]
    cfg = raftmc.ModelConfig(n_servers=w["n"], n_vals=w["V"], max_election=w["E"], max_restart=w["R"],
                             invariants=("Inv",), check_deadlock=False, device=local,
                             timing_phases=TIMED_PHASES)
    parallelism = "single-gpu"
    if world > 1:
        # rank 0 creates the RCCL id; the control-plane group (gloo) broadcasts it
        idt = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            idt = torch.tensor(list(raftmc.comm_unique_id()), dtype=torch.uint8)
        dist.broadcast(idt, 0)
        cfg.rank, cfg.world_size, cfg.comm_unique_id = rank, world, bytes(idt.tolist())
        parallelism = (f"rccl-{world}: fingerprint-owner sharding from the first level of >= 2^20 states, "
                       f"smaller levels replicated on every GPU (all of this workload's)")
    mc, err = None, ""
    try:
        mc = raftmc.ModelChecker(cfg)
    except raftmc.RmcError as e:
        if world == 1:
            raise
        err = str(e)
    if world > 1:
        ok = torch.tensor([0 if mc is None else 1], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)  # every rank takes the same mode
        if int(ok.item()) == 0:
            print(f"rank {rank}: sharded RCCL path unavailable ({err or 'another rank failed'}); running replicas",
                  file=sys.stderr, flush=True)
            if mc is not None:
                mc.close()
            cfg.rank, cfg.world_size, cfg.comm_unique_id = 0, 1, None
            mc = raftmc.ModelChecker(cfg)
            parallelism = f"replicas (sharded RCCL init failed: {err or 'on another rank'})"
    res = None
    for _ in range(args.warmup):
        mc.reset()
        res = mc.run()

    def barrier():
        if world > 1:
            dist.barrier()

    phase_ms = [0.0] * 6
    launches = [0] * 6
    Fs = Gs = Ns = Gself = 0
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # HIP events between kernels cost a few microseconds of queue time each on this
    # latency-bound workload, so only every TIMING_EVERY-th timed step carries them; the
    # dominant kernel's average launch duration comes from those steps' events.
    for k in range(args.steps):
        mc.set_timing(TIMED_PHASES if k % TIMING_EVERY == 0 else 0)
        mc.reset()
        res = mc.run()
        if k % TIMING_EVERY:
            continue
        for ls in res.levels:  # the event-timed steps: their launches and the bytes they moved
            for i in range(6):
                phase_ms[i] += ls.kernel_ms[i]
                launches[i] += ls.kernel_launches[i]
            Fs += ls.expanded
            Gs += ls.generated
            Ns += ls.new_states
            Gself += ls.self_loops
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert res is not None and res.status == "done", res
    ms_per_step = elapsed / args.steps * 1e3
    # replicas (RCCL unavailable) each exhaust the whole space: the job is still ONE exhaustion, so
    # value stays its distinct states / time (never multiplied by the replica count)
    units = res.distinct
    value = units * args.steps / elapsed

    # dominant kernel phase: the one with the most device time (HIP events on the engine's stream)
    S, CCWB = record_bytes(res, mc.cfg)
    slot_b = res.seen_slot_bytes or 16
    dom = max(range(4), key=lambda i: phase_ms[i])
    per_launch_ms = phase_ms[dom] / max(1, launches[dom])
    bytes_total = alg_bytes(PHASES[dom], Fs, Gs, Ns, S, CCWB, slot_b, staging_bytes(mc.cfg), Gself=Gself)
    achieved = bytes_total / max(1, launches[dom]) / (per_launch_ms / 1e3) / 1e9 if per_launch_ms > 0 else 0.0
    pmc = pmc_kernel(mc, PHASES[dom], args.workload, res.depth)
    roof = {"bound": "hbm", "kernel": PHASES[dom], "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": pmc.get("traffic"),
            "traffic_source": pmc.get("source"),
            "algorithmic_bytes_per_launch": round(bytes_total / max(1, launches[dom])),
            "avg_launch_ms": round(per_launch_ms, 5), "launches": launches[dom],
            "timed_steps": len(range(0, args.steps, TIMING_EVERY)),
            "record_bytes_avg": round(S, 2), "seen_slot_bytes": slot_b,
            "phase_ms_per_step": {PHASES[i]: round(phase_ms[i] / len(range(0, args.steps, TIMING_EVERY)), 4)
                                  for i in range(4)}}
    if pmc.get("valu_insts") and per_launch_ms > 0:
        # the binding limit of the expansion kernel: VALU issue.  A wave64 VALU instruction occupies a
        # SIMD-32 for 2 cycles (MI355X_MICROARCH.md constants table): peak = CUs x 4 SIMDs x clock / 2
        rate = pmc["valu_insts"] / (per_launch_ms / 1e3)
        roof["valu"] = {"insts_per_launch": round(pmc["valu_insts"]), "achieved_insts_per_s": round(rate),
                        "peak_insts_per_s": VALU_PEAK, "frac": round(rate / VALU_PEAK, 4),
                        "source": pmc.get("source")}
    # seen-set probe throughput of the run (one probe per generated successor in the expansion
    # pass, one insert per new state in commit) against the random-probe peak of the same slot
    # layout measured on this GPU: a table the size of the run's (2^22 slots, L2/MALL-resident)
    # and one far beyond the caches (2^28 slots = 4 GiB, HBM-resident)
    probes = (res.generated + res.distinct) * args.steps * (world if parallelism.startswith("replicas") else 1)
    seen = {"probes_per_step": res.generated + res.distinct,
            "achieved_probes_per_s": round(probes / elapsed, 1)}
    pk_hbm = None
    if rank == 0 and not args.no_probe_peak:
        pk_small = raftmc.probe_peak(local, 22, 1 << 26)
        pk_hbm = raftmc.probe_peak(local, 28, 1 << 28)
        seen.update({"peak_probes_per_s_2^22_slots": round(pk_small, 1),
                     "peak_probes_per_s_2^28_slots": round(pk_hbm, 1),
                     "frac_of_hbm_probe_peak": round(probes / elapsed / pk_hbm, 5),
                     "slot_bytes": 16})
    line = {
        "metric": "distinct states/sec (whole node) + wall-time to exhaust",
        "value": round(value, 1),
        "unit": "distinct states/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: the state space of Raft.tla itself, generated from Init on the GPU each step",
        "config": {"workload": w["desc"], "distinct_states": res.distinct, "states_generated": res.generated,
                   "depth": res.depth, "verdict": "Inv holds" if res.status == "done" else res.status,
                   "parallelism": parallelism},
        "roofline": roof,
        "seen_set": seen,
        "survey_roofline": survey_roofline(res.levels, S, elapsed / args.steps, pk_hbm),
    }
    if rank == 0 and world == 1 and not args.no_scale:
        mc.close()  # the at-scale run gets the whole device (this checker's chunk buffers are ~12 GB)
        line["at_scale"] = dict(path="single-gpu", n_gpus=1, **at_scale(local, probes_per_s=pk_hbm))
        if not args.no_cpu_baseline:
            line["cpu_baseline_at_scale"] = cpu_baseline_at_scale(local)
    if rank == 0 and sharded is not None:
        # N > 1: the same workload (Raft.cfg exhausted) under the same key, over all N GPUs
        line["at_scale"] = dict(path=f"sharded over {world} GPUs (RCCL)", **sharded)
    if rank == 0 and sharded_c4 is not None:
        line["at_scale_sharded_configs3"] = sharded_c4
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(w)
    if rank == 0:
        print(json.dumps(line), flush=True)
    mc.close()
    if world > 1:
        dist.destroy_process_group()


def counters_at_scale(workload="raftcfg"):
    """The at-scale kernel counters committed under profiles/ (tools/pmc_scale.sh on Raft.cfg's first
    levels + tools/pmc_scale_report.py): per kernel, the HBM traffic (PMC FETCH_SIZE x2 + WRITE_SIZE)
    and the algorithmic bytes of its launches at >= 0.5 M parents against their HIP-event time, and
    the VALU-issue fraction (SQ_INSTS_VALU).  Recomputable from the per-level rows in the file."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_scale_{workload}_levels.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    out = {"source": os.path.relpath(files[-1], ROOT), "workload": d.get("workload")}
    for k, v in d.get("kernels", {}).items():
        a = v["aggregate"]
        out[k] = {x: a[x] for x in ("levels", "alg_frac", "hbm_frac", "ratio", "ratio_fetch_x1", "valu_frac",
                                    "valu_per_successor", "alg_GBps", "hbm_GBps")}
    return out


def cpu_baseline_at_scale(device, workload="raftcfg", max_states=20_000_000):
    """The CPU restatement (oracle/raft_mt.c, every host thread this job may use) on the at-scale workload's
    first levels -- up to the first level boundary past max_states (Raft.cfg: 24 levels, 21.6 M states, a
    bounded 10-30 s sample) -- and the GPU over the same levels (a fresh checker, Init + one rmc_step per
    level): same workload, same host, same levels."""
    import raftmc
    so = os.path.join(ROOT, "oracle", "build", "libraft_mt.so")
    if not os.path.exists(so):
        return None
    w = WORKLOADS[workload]
    lib = ctypes.CDLL(so)
    P64 = ctypes.POINTER(ctypes.c_uint64)
    lib.orc_mt_levels.argtypes = [ctypes.c_int] * 5 + [ctypes.c_uint64, P64, P64, ctypes.c_int, P64, P64,
                                                       ctypes.POINTER(ctypes.c_int)]
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))
    cap = 256
    d, g = (ctypes.c_uint64 * cap)(), (ctypes.c_uint64 * cap)()
    dist, gen, depth = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
    t0 = time.perf_counter()
    v = lib.orc_mt_levels(w["n"], w["V"], w["E"], w["R"], threads, max_states, d, g, cap, ctypes.byref(dist),
                          ctypes.byref(gen), ctypes.byref(depth))
    dt = time.perf_counter() - t0
    D = depth.value
    cpu_levels = list(d[:D])
    # the GPU's levels 1..D: Init plus the expansions of levels 1..D-1
    cfg = raftmc.ModelConfig(n_servers=w["n"], n_vals=w["V"], max_election=w["E"], max_restart=w["R"],
                             invariants=("Inv",), check_deadlock=False, device=device)
    with raftmc.ModelChecker(cfg) as mc:
        mc.init()  # (buffers grow on the way: one untimed pass first)
        for _ in range(D - 1):
            mc.step()
        mc.reset()
        t0 = time.perf_counter()
        gpu_levels = [mc.init().new_states]
        for _ in range(D - 1):
            gpu_levels.append(mc.step().new_states)
        gpu_s = time.perf_counter() - t0
    return {"value": round(dist.value / dt, 1), "unit": "distinct states/s", "cores": threads, "cpu_model": cpu_model(),
            "kind": "port", "levels": D, "distinct_states": dist.value, "seconds": round(dt, 3),
            "gpu_seconds_same_levels": round(gpu_s, 4),
            "gpu_distinct_per_s_same_levels": round(dist.value / gpu_s, 1) if gpu_s > 0 else None,
            "gpu_over_cpu_same_levels": round(dt / gpu_s, 1) if gpu_s > 0 else None,
            "levels_match_gpu": cpu_levels == gpu_levels, "verdict_code": v,
            "sample": f"Raft.cfg levels 1-{D} ({dist.value} distinct states) by oracle/raft_mt.c on {threads} threads "
                      f"(C restatement of Raft.tla, exact canonical forms, level-synchronous first-wins BFS; not TLC: no "
                      f"JVM/tla2tools.jar on the box), {dt:.1f} s; the GPU's seconds are those of the same levels of the "
                      f"at-scale run (the small early levels are latency-bound on the GPU, so the ratio over the whole "
                      f"exhaustion is larger)"}


def at_scale(device, workload="raftcfg", probes_per_s=None):
    """configs[0]/[2] -- Raft.cfg as shipped -- exhausted on this GPU (not the headline: one run is
    ~46 s).  The first run includes growing every buffer (the seen set's move to 8-B slots, the
    frontier ring, the host trace); the second, after rmc_reset, is the steady state.  Its
    first 34 levels are compared with the C oracle's (tests/golden/levels_prefix.json)."""
    import raftmc
    w = WORKLOADS[workload]
    cfg = raftmc.ModelConfig(n_servers=w["n"], n_vals=w["V"], max_election=w["E"], max_restart=w["R"],
                             invariants=("Inv",), check_deadlock=False, device=device, timing_phases=TIMED_PHASES)
    with raftmc.ModelChecker(cfg) as mc:
        mc.set_timing(TIMED_PHASES)
        t0 = time.perf_counter()
        cold = mc.run()
        dt_cold = time.perf_counter() - t0
        mc.reset()
        mc.set_timing(0)
        t0 = time.perf_counter()
        res = mc.run()
        dt = time.perf_counter() - t0
    ms = sum(ls.kernel_ms[PHASES.index("expand_hash")] for ls in cold.levels)
    S, CCWB = record_bytes(cold, cfg)
    # each expansion's bytes, chunk by chunk as the engine cuts the level (chunk_parents): a chunk of >= 2^16
    # parents is split (k_expand<SPLIT>: no fingerprints, probe or election -- those are k_hash_probe's);
    # a level's successors and new states are spread over its chunks in proportion to their parents
    cp = chunk_parents(w["n"], w["V"])
    alg = 0
    for ls in cold.levels[1:]:  # (levels[0] is Init's)
        F = ls.expanded
        for c0 in range(0, F, cp):
            f = min(cp, F - c0)
            alg += alg_bytes("expand_hash", f, ls.generated * f / F, ls.new_states * f / F, S, CCWB,
                             cold.seen_slot_bytes, staging_bytes(cfg), split=f >= (1 << 16),
                             CTXB=ctx_bytes(w["n"], w["V"]), Gself=ls.self_loops * f / F)
    gbs = alg / (ms / 1e3) / 1e9 if ms > 0 else 0.0
    gold = {}
    gpath = os.path.join(ROOT, "tests", "golden", "levels_prefix.json")
    if os.path.exists(gpath):
        with open(gpath) as f:
            gold = json.load(f).get(f"n{w['n']}_v{w['V']}_e{w['E']}_r{w['R']}", {})
    match = None
    if gold:
        got = [ls.new_states for ls in res.levels]
        match = got[:len(gold["levels"])] == gold["levels"]
    return {"workload": w["desc"], "distinct_states": res.distinct, "states_generated": res.generated,
            "depth": res.depth, "verdict": "Inv holds" if res.status == "done" else res.status,
            "seconds_to_exhaust": round(dt, 3), "distinct_per_s": round(res.distinct / dt, 1),
            "generated_per_s": round(res.generated / dt, 1),
            "self_loops": sum(ls.self_loops for ls in res.levels),
            "self_loop_frac": round(sum(ls.self_loops for ls in res.levels) / max(1, res.generated), 4),
            "first_run_seconds_incl_allocation": round(dt_cold, 3),
            "matches_c_oracle_prefix_levels": match, "c_oracle_prefix_levels": len(gold.get("levels", [])),
            "seen_set": f"{res.seen_slots} x {res.seen_slot_bytes} B slots",
            "frontier_ring_bytes": res.frontier_ring_bytes, "frontier_peak_bytes": res.frontier_peak_bytes,
            "record_bytes_avg": round(S, 2),
            "expand_kernel_ms": round(ms, 3), "expand_alg_GBps": round(gbs, 1),
            "expand_frac_of_hbm_peak": round(gbs / HBM_PEAK_GBS, 4),
            "counters": counters_at_scale(workload),
            "survey_roofline": survey_roofline(res.levels, S, dt, probes_per_s)}


# kernel-name prefixes per phase: the item-parallel fused kernels (round 5) first, then round 4's
KERNEL_NAME = {"expand_hash": ["void rmc::k_expand_items<{n}, {V}, {mr}, false, true,",
                               "void rmc::k_expand<{n}, {V}, {mr}, 4, false>(rmc::KParams)",
                               "void rmc::k_expand<{n}, {V}, {mr}, 4>(rmc::KParams)"],
               "dedup": ["void rmc::k_wincount<{n}, {V}, {mr}>(rmc::KParams)"],
               "materialize": ["void rmc::k_commit_items<{n}, {V}, {mr}, ",
                               "void rmc::k_commit<{n}, {V}, {mr}, false>(rmc::KParams)",
                               "void rmc::k_commit<{n}, {V}, {mr}>(rmc::KParams)"]}


PMC_RUNS = 6  # tools/pmc.sh: bench.py --steps 5 --warmup 1 per counter pass
VALU_PEAK = 256 * 4 * 2.4e9 / 2  # wave64 VALU instructions per second on MI355X


def pmc_kernel(mc, phase, workload, depth):
    """Per launch of the dominant kernel, from the committed rocprofv3 PMC summary
    (tools/pmc.sh + tools/pmc_summary.py): HBM bytes (FETCH_SIZE x2 correction per
    MI355X_MICROARCH.md + WRITE_SIZE) and VALU wave-instructions (SQ_INSTS_VALU)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{workload}.json")))
    if not files or phase not in KERNEL_NAME:
        return {}
    n, V = mc.cfg.n_servers, mc.cfg.n_vals
    mr = 1 if (mc.cfg.msg_cap or (64 if n <= 3 else 128)) <= 64 else 2
    d = json.load(open(files[-1]))
    e = None
    for name in KERNEL_NAME[phase]:  # kernel-name prefixes, newest first
        pre = name.format(n=n, V=V, mr=mr)
        e = e or next((d[k] for k in sorted(d) if k.startswith(pre) and isinstance(d[k], dict)), None)
    if not e:
        return {}
    # the device-driven level loop enqueues a few levels past the last one, whose launches
    # return at once: spread each pass's totals over the launches that expanded a level
    real = PMC_RUNS * depth
    scale = e["dispatches"] / real if e["dispatches"] >= real else 1.0
    out = {"source": os.path.relpath(files[-1], ROOT)}
    if "hbm_bytes_per_dispatch" in e:
        out["traffic"] = round(e["hbm_bytes_per_dispatch"] * scale)
    if "SQ_INSTS_VALU" in e:
        out["valu_insts"] = e["SQ_INSTS_VALU"] * scale
    return out


def codec_words(n, V):
    """Packed core words (rmc_spec.h Codec<N, V>::CCW)."""
    bits_for = lambda m: 0 if m <= 0 else m.bit_length()
    b_ix, b_ni, b_ent = bits_for(V + 1), bits_for(V + 2), 3 + bits_for(V - 1)
    bits = n * (bits_for(n) + 3 + 2 + 2 * b_ix) + n * V * b_ent + n * n * (b_ix + b_ni) + n * n + 3 + 4 + V + 8
    return (bits + 31) // 32


def chunk_parents(n, V, chunk_successors=1 << 28):
    """Parents per host-driven chunk on one GPU (rmc_engine.hip: Gcap / maxsucc, at most the winner count's
    1024 x 4096 tiles); maxsucc = Spec::MAXS of one message round (n <= 3) or two."""
    mcap = 64 if n <= 3 else 128
    maxsucc = mcap + n * (4 + V + n - 1)
    return min(chunk_successors // maxsucc, 1024 * 4096)


def ctx_bytes(n, V):
    """A split chunk's hash context per parent (rmc_kernels.hip ctx_words): the packed core padded to
    16 B, then 16 B of message-hash sums per ordered server pair."""
    return 4 * ((codec_words(n, V) + 3) // 4 * 4 + 4 * n * (n - 1))


def staging_bytes(cfg):
    return 48 if cfg.n_servers >= 4 else 32  # Spec::SW4 uint4s per successor slot


def record_bytes(res, cfg):
    """(average bytes of the run's packed frontier records, bytes of the packed core)."""
    nb = sum(ls.new_bytes for ls in res.levels)
    ns = sum(ls.new_states for ls in res.levels)
    ccwb = 4 * codec_words(cfg.n_servers, cfg.n_vals)
    return (nb / ns if ns else float(ccwb)), ccwb


if __name__ == "__main__":
    main()
