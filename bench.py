#!/usr/bin/env python3
"""bench.py -- distinct states/sec of the MI355X model checker on BASELINE.json's workload.

One "step" = one complete breadth-first exhaustion of the workload's state space from Init (TLC's
whole myrun.sh run, minus JVM start-up): successor generation, symmetry + VIEW fingerprinting,
seen-set dedup in TLC -workers 1 order, invariant checks.  The state space starts empty and every
step re-explores it (rmc_reset keeps only device buffers; inputs = the compiled spec tables,
resident in HBM).

Headline workload: BASELINE.json configs[0]/[2] -- Raft.cfg as shipped (myrun.sh:3), the
configuration the metric ("distinct states/sec (whole node) + wall-time to exhaust, 1/2/4/8
MI355X") is quoted on: Raft.tla with Servers = {s1, s2, s3}, Vals = {v1, v2}, MaxElection 3,
MaxRestart 3, SYMMETRY symmServers, VIEW view, INVARIANT Inv, -deadlock -- 10,946,499,503 distinct
states, depth 72, on one GPU in ~13 s.  `value` = its distinct states / the time of one
exhaustion, `ms_per_step` = that time.  The `roofline` block is its dominant kernel, the split
chunks' item-parallel expansion (k_expand_items<..., false, 64>), timed with HIP events on the
engine's stream.  BASELINE configs[1] (3 servers, 1 value, MaxElection 2: 223,437 states in ~1.8 ms)
is reported under the `configs1` key (N = 1).

N > 1 (torchrun, one process per GPU): the same Raft.cfg exhaustion by all ranks together through
the engine's multi-GPU mode: levels below rmc_config.shard_min_states (2^20)
are expanded whole on every rank, and from the first level that reaches it the frontier is
block-cyclic over the ranks and the seen set sharded by fingerprint owner, the successors, verdicts
and winner records exchanged over RCCL each round.  value = distinct states of the exhaustion /
max-over-ranks time, scaling "strong" (total work fixed).  If the RCCL communicator fails to
initialise, each rank exhausts its own copy instead and the line says "replicas" with the error.
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
PH_EXPAND = PHASES.index("expand_hash")
TIMED_PHASES = 1 << PH_EXPAND  # HIP-event timing of the expansion kernels only
SPLIT_MIN = 1 << 16            # rmc_engine.hip split_min: chunks of this many parents run the split pipeline


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


def host_threads():
    # the host cores this job may use: the box's share (OMP_NUM_THREADS is set to it on the GPU boxes;
    # the affinity mask there shows the whole machine)
    return int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))


def cpu_baseline(w, budget_s=12.0):
    """oracle/raft_mt.c -- the C restatement of Raft.tla + TLC -workers 1 BFS semantics, level-
    synchronous on every host core this process may use -- exhausting the same workload (configs[1]:
    a full exhaustion takes ~0.15 s on 16 threads, so the sample is as many as fit in budget_s)."""
    so = os.path.join(ROOT, "oracle", "build", "libraft_mt.so")
    if not os.path.exists(so):
        return None
    lib = ctypes.CDLL(so)
    lib.orc_mt_run.argtypes = [ctypes.c_int] * 5 + [ctypes.POINTER(ctypes.c_uint64)] * 2 + [ctypes.POINTER(ctypes.c_int)]
    threads = host_threads()
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


def cpu_baseline_raftcfg(device, max_states=20_000_000):
    """The CPU restatement (oracle/raft_mt.c, every host thread this job may use) on Raft.cfg's first
    levels -- up to the first level boundary past max_states (24 levels, 21.6 M states: a bounded 10-30 s
    sample of the headline workload; the whole exhaustion would take over an hour) -- and the GPU over the
    same levels (a fresh checker, Init + one rmc_step per level): same workload, same host, same levels."""
    import raftmc
    so = os.path.join(ROOT, "oracle", "build", "libraft_mt.so")
    if not os.path.exists(so):
        return None
    w = WORKLOADS["raftcfg"]
    lib = ctypes.CDLL(so)
    P64 = ctypes.POINTER(ctypes.c_uint64)
    lib.orc_mt_levels.argtypes = [ctypes.c_int] * 5 + [ctypes.c_uint64, P64, P64, ctypes.c_int, P64, P64,
                                                       ctypes.POINTER(ctypes.c_int)]
    threads = host_threads()
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
                      f"JVM/tla2tools.jar on the box), {dt:.1f} s; the GPU's seconds are those of the same levels run "
                      f"level by level (the small early levels are latency-bound on the GPU, so the ratio over the whole "
                      f"exhaustion is larger)"}


C4_TIMEOUT_S = 240  # --configs3 at N > 1: the configs[3] child must finish within this
C4_BUDGET_S = 120   # levels of configs[3] are started until this much time has passed
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
            total += (ls.generated - ls.self_loops) * (24 + 4) + ls.new_bytes + 16 * ls.new_states
    return int(total * (world - 1) / world)


def sharded_child(args):
    """One rank of configs[3] sharded over the N GPUs (--configs3 at N > 1), run in a child process of
    each bench rank before the bench touches the GPU.  Rank 0 writes the result to args.sharded_out."""
    import torch
    import torch.distributed as dist
    import raftmc
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    port = int(os.environ.get("MASTER_PORT", "29500")) + 19  # a port of the child's own
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    idt = torch.zeros(128, dtype=torch.uint8)
    if rank == 0:
        idt = torch.tensor(list(raftmc.comm_unique_id()), dtype=torch.uint8)
    dist.broadcast(idt, 0)
    w = WORKLOADS["c4"]
    cfg = raftmc.ModelConfig(n_servers=w["n"], n_vals=w["V"], max_election=w["E"], max_restart=w["R"],
                             invariants=("Inv",), check_deadlock=False, device=local, rank=rank, world_size=world,
                             comm_unique_id=bytes(idt.tolist()))
    # per GPU: a 48 GB seen-set shard (6.4 G compact slots) and a 160 GB frontier ring, ~80 GB left for the
    # rounds' buffers; the default gives the seen set half of HBM, far more than this configuration's levels
    # fill before the ring does
    cfg.seen_mem_bytes, cfg.frontier_mem_bytes = 48 << 30, 160 << 30
    cfg.chunk_successors = 1 << 27  # rounds of 2^27 slots: the rounds' buffers stay within the ~80 GB left
    c4_child(args, cfg, w, rank, world)
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
        out["skipped"] = f"{budget:.0f} s of budget"
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
           "--child-budget", str(budget_s)]
    t0 = time.perf_counter()
    p = subprocess.Popen(cmd, stdout=sys.stderr, stderr=sys.stderr)
    try:
        rc = p.wait(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        p.kill()
        p.wait()
        err = {"error": f"timed out after {timeout_s:.0f} s", "wall_s": round(time.perf_counter() - t0, 1)}
        if rank == 0 and os.path.exists(out):  # what the child reported before its limit
            with open(out) as f:
                err.update(json.load(f))
        return err if rank == 0 else None
    if rank != 0:
        return None
    if rc != 0 or not os.path.exists(out):
        return {"error": f"child exited with {rc}", "wall_s": round(time.perf_counter() - t0, 1)}
    with open(out) as f:
        return json.load(f)


def progress(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def measure(mc, steps, warmup, world, sync, label, timing_every=1, report_steps=True):
    """W untimed warmup steps, then exactly K timed steps bracketed by a barrier + device sync on both sides;
    the max over ranks of the timed region.  Every timing_every-th timed step carries HIP events on the
    expansion kernels (rmc_set_timing); their per-level statistics are kept for the roofline."""
    import torch.distributed as dist
    res, first_s = None, None
    for i in range(warmup):
        mc.reset()
        t0 = time.perf_counter()
        res = mc.run()
        dt = time.perf_counter() - t0
        first_s = dt if first_s is None else first_s
        if report_steps:
            progress(f"{label} warmup {i + 1}/{warmup}: {dt:.3f} s ({res.distinct} distinct, {res.status})")

    def barrier():
        if world > 1:
            dist.barrier()

    timed = []  # per event-timed step: its level statistics
    barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(steps):
        on = k % timing_every == 0
        mc.set_timing(TIMED_PHASES if on else 0)
        mc.reset()
        ts = time.perf_counter()
        res = mc.run()
        if on:
            timed.append(res.levels)
        if report_steps:
            progress(f"{label} step {k + 1}/{steps}: {time.perf_counter() - ts:.3f} s ({res.distinct} distinct, "
                     f"{res.status})")
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if first_s is None and timed:  # no warmup: the first timed step was the cold one
        first_s = sum(ls.seconds for ls in timed[0])
    return res, elapsed, timed, first_s


def split_roofline(timed, S, cfg, world=1):
    """The headline's roofline: k_expand_items<..., false, 64>, the split chunks' expansion (DESIGN.md
    section 4), over the event-timed steps' levels whose every chunk is split (>= SPLIT_MIN parents; a
    level with a tail chunk below it, which the fused kernel expands, is left out).  Algorithmic bytes per
    chunk: alg_bytes("expand_hash", split=True) with the level's successors, self-loops and new states
    spread over its chunks by their parents; time and launches: the HIP events of those levels' expansion
    phase on the engine's stream.  At N > 1 a rank expands 1/N of each level (block-cyclic rounds)."""
    n, V = cfg.n_servers, cfg.n_vals
    cp = chunk_parents(n, V, cfg.chunk_successors or (1 << 28))
    ms, launches, alg, levels_used = 0.0, 0, 0.0, 0
    for levels in timed:
        for ls in levels[1:]:
            F = ls.expanded
            if F < SPLIT_MIN or 0 < F % cp < SPLIT_MIN or not ls.kernel_launches[PH_EXPAND]:
                continue
            levels_used += 1
            ms += ls.kernel_ms[PH_EXPAND]
            launches += ls.kernel_launches[PH_EXPAND]
            for c0 in range(0, F, cp):
                f = min(cp, F - c0)
                alg += alg_bytes("expand_hash", f, ls.generated * f / F, ls.new_states * f / F, S, 4 * codec_words(n, V),
                                 SWB=staging_bytes(cfg), split=True, CTXB=ctx_bytes(n, V),
                                 Gself=ls.self_loops * f / F) / world
    if not launches or ms <= 0:
        return {"bound": "hbm", "kernel": "k_expand_items (split chunks)", "achieved": None, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": None, "traffic": None}
    per_launch_ms = ms / launches
    per_launch_b = alg / launches
    achieved = per_launch_b / (per_launch_ms / 1e3) / 1e9
    mr = 1 if n <= 3 else 2
    roof = {"bound": "hbm", "kernel": f"k_expand_items<{n}, {V}, {mr}, false, false, 64> (split chunks)",
            "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": None, "algorithmic_bytes_per_launch": round(per_launch_b), "avg_launch_ms": round(per_launch_ms, 5),
            "launches": launches, "levels": levels_used, "timed_steps": len(timed), "record_bytes_avg": round(S, 2)}
    pmc = pmc_kernel(n, V, "raftcfg", split_kernel_name(n, V), dispatches_real=None)
    if pmc.get("traffic"):
        # the PMC run's own split launches: traffic per launch and its ratio to their algorithmic bytes
        roof["traffic"] = pmc["traffic"]
        roof["traffic_source"] = pmc["source"]
        if pmc.get("dispatches"):
            roof["traffic_dispatches"] = pmc["dispatches"]
    if pmc.get("valu_insts"):
        # the expansion's other limit: VALU issue.  A wave64 VALU instruction occupies a SIMD-32 for 2 cycles
        # (MI355X_MICROARCH.md constants table): peak = CUs x 4 SIMDs x clock / 2; the PMC run's instructions
        # per launch over this run's average launch (the same workload's launches)
        rate = pmc["valu_insts"] / (per_launch_ms / 1e3)
        roof["valu"] = {"insts_per_launch": round(pmc["valu_insts"]), "achieved_insts_per_s": round(rate),
                        "peak_insts_per_s": VALU_PEAK, "frac": round(rate / VALU_PEAK, 4), "source": pmc["source"]}
    return roof


def phase_roofline(timed, S, cfg, workload, depth):
    """configs[1]'s roofline (all its levels run in the device loop): the phase with the most HIP-event time
    -- the fused expansion k_expand_items<..., true, 16> -- its algorithmic bytes per launch over its average
    launch duration."""
    phase_ms, launches = [0.0] * 6, [0] * 6
    F = G = N = Gself = 0
    for levels in timed:
        for ls in levels:
            for i in range(6):
                phase_ms[i] += ls.kernel_ms[i]
                launches[i] += ls.kernel_launches[i]
            F += ls.expanded
            G += ls.generated
            N += ls.new_states
            Gself += ls.self_loops
    dom = max(range(4), key=lambda i: phase_ms[i])
    per_launch_ms = phase_ms[dom] / max(1, launches[dom])
    bytes_total = alg_bytes(PHASES[dom], F, G, N, S, 4 * codec_words(cfg.n_servers, cfg.n_vals), 16,
                            staging_bytes(cfg), Gself=Gself)
    achieved = bytes_total / max(1, launches[dom]) / (per_launch_ms / 1e3) / 1e9 if per_launch_ms > 0 else 0.0
    n, V = cfg.n_servers, cfg.n_vals
    mr = 1 if n <= 3 else 2
    name = KERNEL_NAME.get(PHASES[dom], "").format(n=n, V=V, mr=mr)
    # the device-driven level loop enqueues a few levels past the last one, whose launches return at once:
    # the PMC pass's totals are spread over the launches that expanded a level
    pmc = pmc_kernel(n, V, workload, name, dispatches_real=PMC_RUNS * depth) if name else {}
    roof = {"bound": "hbm", "kernel": PHASES[dom], "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": pmc.get("traffic"),
            "traffic_source": pmc.get("source"),
            "algorithmic_bytes_per_launch": round(bytes_total / max(1, launches[dom])),
            "avg_launch_ms": round(per_launch_ms, 5), "launches": launches[dom], "timed_steps": len(timed),
            "record_bytes_avg": round(S, 2),
            "phase_ms_per_step": {PHASES[i]: round(phase_ms[i] / max(1, len(timed)), 4) for i in range(4)}}
    if pmc.get("valu_insts") and per_launch_ms > 0:
        rate = pmc["valu_insts"] / (per_launch_ms / 1e3)
        roof["valu"] = {"insts_per_launch": round(pmc["valu_insts"]), "achieved_insts_per_s": round(rate),
                        "peak_insts_per_s": VALU_PEAK, "frac": round(rate / VALU_PEAK, 4), "source": pmc.get("source")}
    return roof


def oracle_prefix_match(res, w):
    gpath = os.path.join(ROOT, "tests", "golden", "levels_prefix.json")
    if not os.path.exists(gpath):
        return None, 0
    with open(gpath) as f:
        gold = json.load(f).get(f"n{w['n']}_v{w['V']}_e{w['E']}_r{w['R']}", {})
    if not gold:
        return None, 0
    got = [ls.new_states for ls in res.levels]
    return got[:len(gold["levels"])] == gold["levels"], len(gold["levels"])


def configs1_leg(device, args, probes_per_s):
    """BASELINE configs[1] on this GPU (N = 1): its own checker, 5 warmup + 20 timed exhaustions of ~1.8 ms
    (latency-bound: every level runs in the device-driven loop), the dominant kernel's roofline, and the
    C restatement's rate on the same workload."""
    import raftmc
    import torch
    w = WORKLOADS["c2"]
    cfg = raftmc.ModelConfig(n_servers=w["n"], n_vals=w["V"], max_election=w["E"], max_restart=w["R"],
                             invariants=("Inv",), check_deadlock=False, device=device, timing_phases=TIMED_PHASES)
    steps = 20
    with raftmc.ModelChecker(cfg) as mc:
        res, elapsed, timed, _ = measure(mc, steps, 5, 1, torch.cuda.synchronize, "configs[1]", timing_every=8,
                                         report_steps=False)
    S, _ = record_bytes(res, cfg)
    out = {"workload": w["desc"], "value": round(res.distinct * steps / elapsed, 1), "unit": "distinct states/s",
           "ms_per_step": round(elapsed / steps * 1e3, 4), "steps": steps, "warmup": 5,
           "distinct_states": res.distinct, "states_generated": res.generated, "depth": res.depth,
           "verdict": "Inv holds" if res.status == "done" else res.status,
           "roofline": phase_roofline(timed, S, cfg, "c2", res.depth),
           "survey_roofline": survey_roofline(res.levels, S, elapsed / steps, probes_per_s)}
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(w)
    return out


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


# kernel-name prefixes per phase of the fused (device-loop) levels
KERNEL_NAME = {"expand_hash": "void rmc::k_expand_items<{n}, {V}, {mr}, false, true,",
               "dedup": "void rmc::k_wincount<{n}, {V}, {mr}>(rmc::KParams)",
               "materialize": "void rmc::k_commit_items<{n}, {V}, {mr}, "}


def split_kernel_name(n, V):
    return f"void rmc::k_expand_items<{n}, {V}, {1 if n <= 3 else 2}, false, false, 64>"


PMC_RUNS = 6  # tools/pmc.sh: bench.py --workload c2 --steps 5 --warmup 1 per counter pass
VALU_PEAK = 256 * 4 * 2.4e9 / 2  # wave64 VALU instructions per second on MI355X


def pmc_kernel(n, V, workload, prefix, dispatches_real=None):
    """Per launch of a kernel, from the committed rocprofv3 PMC summary of bench.py's workload
    (profiles/r*_pmc_<workload>.json: tools/pmc.sh + tools/pmc_summary.py): HBM bytes (FETCH_SIZE x2
    correction per MI355X_MICROARCH.md + WRITE_SIZE) and VALU wave-instructions (SQ_INSTS_VALU).
    dispatches_real: the launches that did work (the device loop's trailing launches return at once)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{workload}.json")))
    if not files:
        return {}
    d = json.load(open(files[-1]))
    e = next((d[k] for k in sorted(d) if k.startswith(prefix) and isinstance(d[k], dict)), None)
    if not e:
        return {}
    scale = e["dispatches"] / dispatches_real if dispatches_real and e["dispatches"] >= dispatches_real else 1.0
    out = {"source": os.path.relpath(files[-1], ROOT), "dispatches": e["dispatches"]}
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="raftcfg", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe-peak", action="store_true")
    ap.add_argument("--no-configs1", action="store_true", help="skip the configs[1] leg (N = 1)")
    ap.add_argument("--chunk-successors", type=int, default=0,
                    help="successor slots per chunk (0: the engine's default; a tuning run)")
    ap.add_argument("--configs3", action="store_true", help="N > 1: first take configs[3] as deep as the node's "
                    "HBM and a time budget allow (child processes, before the bench touches the GPU)")
    ap.add_argument("--sharded-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--sharded-out", default="", help=argparse.SUPPRESS)
    ap.add_argument("--child-budget", type=float, default=C4_BUDGET_S, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.sharded_child:
        sharded_child(args)
        return
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    sharded_c4 = None
    if world > 1 and args.configs3:
        sharded_c4 = run_child(args, "c4", C4_TIMEOUT_S, budget_s=C4_BUDGET_S)

    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")  # control plane only: barriers and the max-over-ranks time
    torch.cuda.set_device(local)

    import raftmc
    w = WORKLOADS[args.workload]
    cfg = raftmc.ModelConfig(n_servers=w["n"], n_vals=w["V"], max_election=w["E"], max_restart=w["R"],
                             invariants=("Inv",), check_deadlock=False, device=local,
                             timing_phases=TIMED_PHASES, chunk_successors=args.chunk_successors)
    parallelism = "single-gpu"
    if world > 1:
        # rank 0 creates the RCCL id; the control-plane group (gloo) broadcasts it
        idt = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            idt = torch.tensor(list(raftmc.comm_unique_id()), dtype=torch.uint8)
        dist.broadcast(idt, 0)
        cfg.rank, cfg.world_size, cfg.comm_unique_id = rank, world, bytes(idt.tolist())
        parallelism = (f"rccl-{world}: levels of >= 2^20 states block-cyclic over the GPUs with a fingerprint-owner "
                       f"seen set and TLC-order global-key election (RCCL exchange per round); smaller levels "
                       f"replicated on every GPU")
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
    big = args.workload != "c2"
    res, elapsed, timed, first_s = measure(mc, args.steps, args.warmup, world, torch.cuda.synchronize,
                                           args.workload, timing_every=1 if big else 8, report_steps=big)
    assert res is not None and res.status == "done", res
    ms_per_step = elapsed / args.steps * 1e3
    # replicas (RCCL unavailable) each exhaust the whole space: the job is still ONE exhaustion, so
    # value stays its distinct states / time (never multiplied by the replica count)
    value = res.distinct * args.steps / elapsed
    S, _ = record_bytes(res, mc.cfg)
    rworld = world if parallelism.startswith("rccl") else 1
    if big:
        roof = split_roofline(timed, S, mc.cfg, rworld)
        roof["counters_at_scale"] = counters_at_scale(args.workload) if args.workload == "raftcfg" else None
    else:
        roof = phase_roofline(timed, S, mc.cfg, args.workload, res.depth)
    self_loops = sum(ls.self_loops for ls in res.levels)
    match, prefix_levels = oracle_prefix_match(res, w)
    config = {"workload": w["desc"], "distinct_states": res.distinct, "states_generated": res.generated,
              "depth": res.depth, "verdict": "Inv holds" if res.status == "done" else res.status,
              "parallelism": parallelism, "self_loops": self_loops,
              "self_loop_frac": round(self_loops / max(1, res.generated), 4),
              "seen_set": f"{res.seen_slots} x {res.seen_slot_bytes} B slots (rank 0)",
              "frontier_ring_bytes": res.frontier_ring_bytes, "frontier_peak_bytes": res.frontier_peak_bytes,
              "first_run_seconds_incl_allocation": round(first_s, 3) if first_s else None,
              "matches_c_oracle_prefix_levels": match, "c_oracle_prefix_levels": prefix_levels}
    # seen-set probe throughput of the run (one probe per fingerprinted successor, one insert per new state)
    # against the random-probe peak of the slot layout measured on this GPU: a table far beyond the caches
    # (2^28 16-B slots = 4 GiB, HBM-resident) and one of 2^22 slots (L2/MALL-resident)
    probes = res.generated - self_loops + res.distinct
    seen = {"probes_per_step": probes, "achieved_probes_per_s": round(probes * args.steps / elapsed, 1)}
    pk_hbm = None
    if rank == 0 and not args.no_probe_peak:
        pk_small = raftmc.probe_peak(local, 22, 1 << 26)
        pk_hbm = raftmc.probe_peak(local, 28, 1 << 28)
        seen.update({"peak_probes_per_s_2^22_slots": round(pk_small, 1),
                     "peak_probes_per_s_2^28_slots": round(pk_hbm, 1),
                     "frac_of_hbm_probe_peak": round(probes * args.steps / elapsed / pk_hbm, 5), "slot_bytes": 16})
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
        "config": config,
        "roofline": roof,
        "seen_set": seen,
        "survey_roofline": survey_roofline(res.levels, S, elapsed / args.steps, pk_hbm),
    }
    if world > 1:
        line["xgmi_bytes_model"] = xgmi_model(res.levels, rworld)
        line["xgmi_GBps_avg"] = round(line["xgmi_bytes_model"] / (elapsed / args.steps) / 1e9, 2)
    mc.close()
    if rank == 0 and world == 1 and args.workload != "c2" and not args.no_configs1:
        line["configs1"] = configs1_leg(local, args, pk_hbm)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = (cpu_baseline_raftcfg(local) if args.workload == "raftcfg" else
                                cpu_baseline(w) if args.workload == "c2" else None)
    if rank == 0 and sharded_c4 is not None:
        line["at_scale_sharded_configs3"] = sharded_c4
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
