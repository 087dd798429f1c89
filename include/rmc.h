/*
 * rmc.h -- C-ABI of the MI355X-native Raft model checker (librmc.so).
 *
 * The reference (kikimo/tla-raft) has no library API: its only interface is the
 * TLC command line in myrun.sh:3
 *
 *     java -Xms4g -Xmx12g -jar tla2tools.jar -deadlock -workers 4 -config Raft.cfg Raft.tla $@
 *
 * which reads Raft.tla + Raft.cfg, runs TLC's breadth-first model checker and
 * prints TLC text.  Every entry point below replaces one piece of that run and
 * cites what it replaces.  A TLC-compatible host driver (tla-raft_amd/launcher,
 * or a Java FFM / Python ctypes binding -- INTEGRATION.md) sits on top.
 *
 * Conventions: plain C types only; every function returns RMC_OK (0) or a
 * negative RMC_E_* code, with text from rmc_last_error().  A context is owned by
 * one host thread.  All device memory is owned by the context.  The library
 * never falls back to a CPU path: without a usable gfx950 device rmc_create
 * fails with RMC_E_DEVICE.
 */
#ifndef RMC_H
#define RMC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RMC_ABI_VERSION 5

/* ---- return codes ---------------------------------------------------------- */
#define RMC_OK 0
#define RMC_DONE 1          /* rmc_step: the state space is exhausted */
#define RMC_VIOLATION 2     /* an INVARIANT is FALSE in a new state (TLC exit 12) */
#define RMC_ASSERT 3        /* Assert(role[s] # Leader, "split brain") failed, Raft.tla:185 */
#define RMC_EVAL_ERROR 4    /* TLC evaluation error while checking an invariant (Raft.tla:499) */
#define RMC_DEADLOCK 5      /* a state without successors while deadlock checking is on */
#define RMC_E_ARG -1
#define RMC_E_DEVICE -2
#define RMC_E_MEMORY -3
#define RMC_E_CAPACITY -4   /* a state exceeded the packed layout (|msgs| > msg_cap) */
#define RMC_E_STATE -5      /* call out of sequence */
#define RMC_E_PARSE -6      /* cfg / spec validation failed */
#define RMC_E_COMM -7       /* multi-GPU communicator failure */

/* ---- invariants (Raft.cfg:33-34 selects Inv) --------------------------------- */
#define RMC_INV_LEADER_HAS_ALL_COMMITTED (1u << 0) /* Inv == LeaderHasAllCommittedEntries, Raft.tla:491-503 */
#define RMC_INV_NO_SPLIT_VOTE (1u << 1)            /* Raft.tla:444-448 */
#define RMC_INV_RAFT_CAN_COMMIT (1u << 2)          /* RaftCanCommt, Raft.tla:434 */
#define RMC_INV_FOLLOWER_CAN_COMMIT (1u << 3)      /* Raft.tla:436-439 */
#define RMC_INV_COMMIT_ALL (1u << 4)               /* Raft.tla:442 */
#define RMC_INV_NO_ALL_COMMIT (1u << 5)            /* Raft.tla:451-481 (reads msgs) */
#define RMC_INV_EXIST_LEADER_AND_CANDIDATE (1u << 6) /* Raft.tla:483-487 */

/* ---- spec variants ------------------------------------------------------------ */
#define RMC_SPEC_RAFT 0    /* Raft.tla as shipped */
#define RMC_SPEC_SEEDED 1  /* RaftSeeded: Median's threshold (Raft.tla:72) is Cardinality(Servers) */
#define RMC_SPEC_BECOME_FOLLOWER 2  /* Raft.tla with Next's `\/ BecomeFollower(s)` uncommented (Raft.tla:420):
                                       FollowerUpdateTerm / CandidateToFollower / LeaderToFollower
                                       (Raft.tla:190-229) right after UpdateTerm; trace action id 12 */
/* Test variants (tools/make_seeded_spec.py --split-brain / --commit-past-log) in which TLC's two error
 * kinds other than an invariant violation are reachable in a BFS, so their precedence and counters
 * are checked end to end (the shipped specs reach neither): */
#define RMC_SPEC_SPLIT_BRAIN 3      /* RaftSplitBrain: BecomeLeader's quorum (Raft.tla:164) is 1 -> two
                                       leaders of one term -> UpdateTerm's Assert (Raft.tla:185) fails */
#define RMC_SPEC_COMMIT_PAST_LOG 4  /* RaftCommitPastLog: FollowerAcceptEntry's newCommitIndex (Raft.tla:294)
                                       is Max(commitIndex, leaderCommit) -> Inv's logs[p][index]
                                       (Raft.tla:499) out of its domain */

/* Model configuration: what Raft.cfg's CONSTANTS (Raft.cfg:1-21), INVARIANT
 * (Raft.cfg:33-34) and TLC's -deadlock flag (myrun.sh:3) bind.  VIEW view
 * (Raft.cfg:26) is always on; SYMMETRY symmServers (Raft.cfg:24) unless
 * no_symmetry.  A zero-initialised struct plus the four constants and
 * invariants = RMC_INV_LEADER_HAS_ALL_COMMITTED is Raft.cfg under myrun.sh. */
typedef struct rmc_config {
    int32_t n_servers;      /* |Servers|   Raft.cfg:18, 1..5 */
    int32_t n_vals;         /* |Vals|      Raft.cfg:21, 0..3 */
    int32_t max_election;   /* MaxElection Raft.cfg:4,  0..7 */
    int32_t max_restart;    /* MaxRestart  Raft.cfg:3,  0..15 */
    uint32_t invariants;    /* RMC_INV_* bits (order: invariant_order) */
    int32_t check_deadlock; /* 0 = TLC -deadlock (myrun.sh:3) */
    int32_t spec_variant;   /* RMC_SPEC_* */
    int32_t device;         /* HIP device ordinal (-1 = current) */
    int32_t msg_cap;        /* max |msgs| per state: 0 = auto (64 for n<=3, 128 otherwise) */
    int32_t seen_log2;      /* initial seen-set slots = 2^seen_log2 (0 = auto); grows on demand */
    int32_t no_symmetry;    /* 0 = SYMMETRY symmServers (Raft.cfg:24); 1 = cfg without SYMMETRY */
    uint64_t chunk_successors; /* successors per device chunk (0 = auto) */
    /* multi-GPU (one process per GPU): world_size 0 or 1 = single GPU */
    int32_t rank, world_size;  /* world_size 0 or 1 = single GPU; world_size 1 WITH comm_unique_id = a one-rank
                                  RCCL communicator running the sharded protocol (self send/recv) */
    const void *comm_unique_id; /* 128-byte RCCL unique id (rmc_comm_unique_id on rank 0), same on every rank;
                                  NULL with world_size > 1: the host-staged transport (rmc_set_transport) */
    int32_t virtual_shards;    /* > 1: run that many fingerprint-owner shards in this process on one device
                                  (the multi-GPU partition/exchange logic with device copies for transport) */
    uint32_t timing_phases;    /* bit i: HIP-event time phase i into rmc_level_stats.kernel_ms (0 = all) */
    uint32_t device_levels;    /* single GPU: BFS levels enqueued per host round trip by rmc_run /
                                  rmc_run_levels (0 = auto, 1 = the host drives every level) */
    uint64_t shard_min_states; /* world_size or virtual_shards > 1: levels with fewer states than this are
                                  expanded whole on every shard (replicated, no exchange, TLC order); the run
                                  switches to the sharded level (block-cyclic frontier, fingerprint-owner seen
                                  set, TLC-order election by global key) at the first level that reaches it
                                  and stays sharded (0 = auto: 2^20; 1 = sharded from Init's level) */
    /* ---- ABI 3 ---- */
    uint32_t invariant_order;  /* the INVARIANTs in cfg order (Raft.cfg:33-34; TLC checks them in that order):
                                  invariant bit index + 1 per 4-bit nibble, first in the low nibble;
                                  0 = the bits of `invariants` in bit order */
    uint32_t compact_log2;     /* seen set: 16-B slots {fp} while the table has at most 2^compact_log2 slots,
                                  then one migration to 8-B slots sized from seen_mem_bytes and never grown
                                  (0 = auto: 27) */
    uint64_t seen_mem_bytes;   /* device bytes for the compact seen set (0 = auto: half of the free memory
                                  at migration, per shard) */
    uint64_t frontier_mem_bytes; /* device bytes for the frontier ring once the seen set is compact (0 = auto:
                                  70 % of the free memory left then, per shard) */
} rmc_config;

/* Statistics of one BFS level (what TLC's progress line reports). */
typedef struct rmc_level_stats {
    int32_t level;            /* BFS level whose states were just expanded (1 = Init's level) */
    int32_t status;           /* RMC_OK / RMC_DONE / RMC_VIOLATION / ... */
    uint64_t expanded;        /* states of that level expanded (all ranks) */
    uint64_t generated;       /* successors generated while expanding it (all ranks) */
    uint64_t new_states;      /* distinct states first found (all ranks) */
    uint64_t total_generated; /* TLC "states generated", Init included */
    uint64_t total_distinct;  /* TLC "distinct states found" */
    uint64_t queue;           /* TLC "states left on queue" */
    double seconds;           /* wall time of this level */
    double kernel_ms[6];      /* expand-count, expand-hash, dedup, materialize, exchange, other */
    uint64_t kernel_launches[6];
    uint64_t new_bytes;       /* ABI 3: bytes of the new states' frontier records (packed core + message ids) */
    uint64_t self_loops;      /* ABI 5: generated successors equal to their parent (FollowerAcceptEntry that
                                 changes nothing), among `generated`.  Single-GPU levels set them apart (never
                                 fingerprinted: the parent is in the seen set); sharded rounds set them apart in
                                 split rounds and route them in smaller rounds, counting them either way */
} rmc_level_stats;

/* Final result of a run: TLC's closing lines. */
typedef struct rmc_result {
    int32_t status;           /* RMC_DONE / RMC_VIOLATION / RMC_ASSERT / RMC_EVAL_ERROR / RMC_DEADLOCK */
    int32_t depth;            /* "The depth of the complete state graph search is D" */
    uint64_t generated, distinct, queue;
    int32_t violated;         /* index (bit) of the violated invariant, -1 if none */
    uint32_t trace_len;
    double seconds;
    /* ABI 3: memory of the run (this rank) */
    uint64_t seen_slots;          /* seen-set capacity in slots */
    int32_t seen_slot_bytes;      /* 16 (full fingerprints) or 8 (compact) */
    int32_t pad_;
    uint64_t frontier_ring_bytes; /* device bytes of the frontier ring */
    uint64_t frontier_peak_bytes; /* largest live frontier (current + next level records) */
} rmc_result;

int rmc_abi_version(void);

/* RCCL unique id for a multi-GPU run (call on rank 0, broadcast the 128 bytes to every
 * rank, pass as rmc_config.comm_unique_id).  Replaces nothing in the reference: TLC runs
 * in one JVM; this is the seen-set sharding of SURVEY.md 8(e). */
int rmc_comm_unique_id(void *out128);

/* ABI 4: a host-staged transport for the sharded protocol (world_size > 1 without comm_unique_id).
 * The ranks' collectives go through these callbacks instead of RCCL: every rank of the run installs
 * one (process-wide, before rmc_create; NULL removes it) whose calls meet their peers' -- e.g. a
 * torch.distributed gloo group (raftmc.HostTransport).  It carries the same protocol as RCCL through
 * host memory, so the multi-rank path runs as separate processes on one device (tests) or on hosts
 * without a GPU interconnect.  Each callback returns 0 on success; anything else fails the step with
 * RMC_E_COMM.
 *   allreduce_u64  v[0..n) <- the elementwise sum (is_max = 0) or maximum over the ranks, in place
 *   allgather_u64  out[0..W*k) <- every rank's row[0..k), in rank order
 *   alltoallv      bytes send + send_off[p] .. + send_bytes[p] go to rank p, bytes from rank p land at
 *                  recv + recv_off[p] (recv_bytes[p] of them); the caller's own entries are 0 */
typedef struct rmc_transport {
    void *user;
    int32_t (*allreduce_u64)(void *user, uint64_t *v, int32_t n, int32_t is_max);
    int32_t (*allgather_u64)(void *user, const uint64_t *row, int32_t k, uint64_t *out);
    int32_t (*alltoallv)(void *user, const void *send, const uint64_t *send_off, const uint64_t *send_bytes,
                         void *recv, const uint64_t *recv_off, const uint64_t *recv_bytes);
} rmc_transport;
int rmc_set_transport(const rmc_transport *t);

/* Parse Raft.cfg text (replaces TLC's ModelConfig for the subset Raft.cfg uses,
 * Raft.cfg:1-34) and validate Raft.tla text by content (replaces SANY; only
 * Raft.tla, the documented RaftSeeded variant and Raft.tla with FollowerAppendEntry
 * uncommented in Next -- never enabled, so RMC_SPEC_RAFT -- are recognised).  tla_text
 * may be NULL to skip the spec check (then spec_variant is left unchanged). */
int rmc_parse_config(const char *cfg_text, const char *tla_text, rmc_config *out, char *err, size_t err_cap);

/* Replaces TLC start-up (myrun.sh:3): allocates device state, builds the
 * message universe and symmetry tables for the configuration. */
int rmc_create(const rmc_config *cfg, void **ctx_out);

/* Init (Raft.tla:93-105): level 1, invariant check on the initial state. */
int rmc_init(void *ctx, rmc_level_stats *st);

/* One BFS level of TLC's worker loop: successors of every state of the current
 * level (Next, Raft.tla:416-430), SYMMETRY+VIEW fingerprint (Raft.tla:21,38),
 * seen-set insertion with TLC -workers 1 first-discovery order, INVARIANT check
 * on new states (Raft.cfg:33).  Returns RMC_OK, RMC_DONE or an error status. */
int rmc_step(void *ctx, rmc_level_stats *st);

/* As many BFS levels as one host round trip covers: on a single GPU up to
 * cfg.device_levels levels enqueued back to back, each level's kernels taking its
 * size from the previous level's commit on the device (stopping early at the end,
 * an error, or a level that needs larger buffers); otherwise one rmc_step.
 * Per-level statistics go to levels[0..*n); cap >= 1.  Same return as rmc_step for
 * the last level reported. */
int rmc_steps(void *ctx, rmc_level_stats *levels, uint32_t cap, uint32_t *n);

/* Phase timing from now on: 0 = off (no HIP events between kernels), 0xFFFFFFFF = every
 * phase, otherwise a mask as cfg.timing_phases. */
int rmc_set_timing(void *ctx, uint32_t phases);

/* Forget every explored state (seen set, levels, trace) but keep the device
 * buffers, so the next rmc_init starts a fresh run (TLC: a new invocation). */
int rmc_reset(void *ctx);

/* Checkpoint / resume between BFS levels (TLC's states/ metadir and -recover, .gitignore:2;
 * SURVEY 8(f) item 4).  rmc_checkpoint writes the seen set, the current level, every state's
 * parent reference and TLC's counters to `path`, after rmc_init and before the run finishes.
 * Sharded runs too: a context with virtual shards writes all of them to `path`; an RCCL rank of
 * a world_size > 1 run writes its own shards to `path` + ".rank<r>" (every rank calls it between
 * the same two levels).  rmc_resume loads such a file into a context created with the same
 * configuration and shard layout (world size, rank, virtual shards, chunk size, shard_min) and
 * not yet initialised; rmc_step / rmc_run then carry on as if the run had never stopped (same
 * counts, same TLC order, same counterexample). */
int rmc_checkpoint(void *ctx, const char *path);
int rmc_resume(void *ctx, const char *path);

/* Loop rmc_step until done or an error; fills the final result. */
int rmc_run(void *ctx, rmc_result *res);
int rmc_get_result(void *ctx, rmc_result *res);

/* rmc_init + rmc_step until done inside the library (no per-level host round trip of the
 * caller); per-level statistics go to levels[0..*n_levels) (as many as fit in cap). */
int rmc_run_levels(void *ctx, rmc_level_stats *levels, uint32_t cap, uint32_t *n_levels, rmc_result *res);

/* Counterexample (TLC's "The behavior up to this point is"): states 1..len from
 * Init to the error state.  Unpacked layout below.  action/server/witness
 * describe how state i was reached (action -1 for state 0 = Initial predicate). */
int rmc_trace_len(void *ctx, uint32_t *len);
int rmc_trace_state(void *ctx, uint32_t i, int32_t *unpacked, size_t cap_ints,
                    int32_t *action, int32_t *server, int32_t *witness);

/* Measurement support (bench.py): the random-probe peak of the seen-set layout -- `probes`
 * one-slot reads of 16-B slots at uniformly random indices of a 2^table_log2-slot table,
 * best of 3 timed launches; no model-checking state is touched. */
int rmc_probe_peak(int device, uint32_t table_log2, uint64_t probes, double *probes_per_s, double *seconds);

const char *rmc_last_error(void *ctx);
void rmc_destroy(void *ctx);
/* Frees every device allocation of the context (seen set, frontier ring, chunk buffers, streams, the
 * communicator) and its pinned buffers, but not the host copy of the trace (~110 GB at Raft.cfg): a
 * process about to exit returns the device at once and leaves the host memory to the kernel.  Only
 * rmc_destroy may follow (every other call returns RMC_E_STATE).  The launcher's detached worker calls it
 * before it reports TLC's exit code, so a GPU job started when myrun.sh returns finds the device free. */
int rmc_release_device(void *ctx);

/* ---- single-state hooks (parity tests; same kernels as rmc_step) -------------- */
/* Successors of one state, in TLC enumeration order.  keys[i] = server<<24 |
 * action<<16 | witness (witness: index into the sorted msgs for message actions,
 * value for ClientReq, destination for LeaderAppendEntry, else 0).  fps gets the
 * 128-bit symmetry+view fingerprint of each successor (2 words).  Returns the
 * count, or RMC_ASSERT if UpdateTerm's Assert fails. */
int rmc_successors(void *ctx, const int32_t *unpacked, int32_t *out, size_t stride_ints, uint32_t cap,
                   uint32_t *keys, uint64_t *fps, uint32_t *count);
int rmc_fingerprint(void *ctx, const int32_t *unpacked, uint64_t fp[2]);
/* ABI 4 -- checks of a finished run's deep levels (tests/test_gpu_deep.py).  The path of the explored
 * state with global id `gid` (BFS order, Init = 0): len = its depth, keys[i] = how state i of the path
 * was reached from state i - 1 (rmc_successors' key format; keys[0] = 0), gids[i] = its global id
 * (gids[0] = 0, gids[len - 1] = gid); from TLC's parent pointers (the trace), any shard layout. */
int rmc_state_path(void *ctx, uint64_t gid, uint32_t *keys, uint64_t *gids, uint32_t cap, uint32_t *len);
/* Fingerprints of n unpacked states, stride_ints apart (2 words each), in one launch. */
int rmc_fingerprints(void *ctx, const int32_t *unpacked, size_t stride_ints, uint64_t n, uint64_t *fps);
/* Seen-set membership (TLC's FPSet) of n fingerprints: out[i] = 1 if present.  Not for RCCL ranks. */
int rmc_seen_contains(void *ctx, const uint64_t *fps, uint64_t n, uint8_t *out);
/* 1 = TRUE, 0 = FALSE, RMC_EVAL_ERROR; one invariant bit */
int rmc_eval_invariant(void *ctx, const int32_t *unpacked, uint32_t invariant_bit, int32_t *value);

/* Unpacked state (int32), the interchange format of every hook:
 *   votedFor[n] (-1 = None)  currentTerm[n]  role[n] (0 F, 1 C, 2 L)  commitIndex[n]  logLen[n]
 *   logs[n][V+1][2]          (term, val) per index 1..V+1; index 1 = (0,-1); unused = (0,0)
 *   matchIndex[n][n]  nextIndex[n][n]  pendingResponse[n][n]
 *   electionCount  restartCount  valSent[V] (-1 = None, 0 = FALSE)
 *   nmsgs  msgs[nmsgs][8], sorted in TLC order:
 *     type (0 VoteReq, 1 VoteResp, 2 AppendReq, 3 AppendResp) src dst term x1 x2 x3 x4
 *     VoteReq x1 = lastLogIndex x2 = lastLogTerm; AppendResp x1 = prevLogIndex x2 = succ;
 *     AppendReq x1 = prevLogIndex x2 = prevLogTerm x3 = leaderCommit x4 = entry (-1 none, else term*8+val)
 */
#define RMC_UNPACKED_INTS(n, V, nmsgs) (5 * (n) + (n) * ((V) + 1) * 2 + 3 * (n) * (n) + 3 + (V) + 8 * (nmsgs))

#ifdef __cplusplus
}
#endif
#endif /* RMC_H */
