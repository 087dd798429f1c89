// rmc_kernels.h -- host-side declarations of the device kernel set.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rmc_spec.h"

namespace rmc {

// Device-resident lookup tables built by the host (Universe) for one configuration.
struct Tables {
    const uint32_t *info;     // [U]        message info word by id (TLC order)
    const uint16_t *nat2id;   // [nat_total] natural index -> id
    const ulonglong2 *gmsg;   // [U]        per-message hash, families 0/1 (no src/dst)
    const uint64_t *seeds;    // [2][MAXN*MAXN] odd position constants K_f[a][b] of the fingerprint (rmc_spec.h)
    int np;                   // |Permutations(Servers)| (1: no SYMMETRY)
    uint32_t bmw;             // 32-bit words of a bitmap over the universe's ids: ceil(U / 32)
};

// An election slot (the fused / split chunk's election table, a sharded round's owner table): the
// fingerprint a slot holds, both words tagged in their low 16 bits, and the slot's election word -- in
// one 32-B sector, so a candidate's claim and its bid touch one line (round 4 kept x / y and the word in
// two arrays: two random lines per new fingerprint).
struct ESlot {
    unsigned long long x, y;  // the fingerprint, tagged (elect_tag / the owner table's round tag)
    unsigned long long k;     // the election word (elect_key / owner_key): the smallest bid wins
    unsigned long long pad;
};

// Seen set (TLC's FPSet): open addressing over 128-bit fingerprints {x | 1, y}.
//   full:    16-B slots {x, y} (T != nullptr), grown x4 by rehash while small;
//   compact:  8-B slots holding x only (Tc != nullptr), eight to a 64-B bucket: the bucket probe run,
//             which starts at the home bucket derived from y, carries the rest of the identity.  Used
//             once the run is large (rmc_config.compact_log2); sized once from the memory budget (any
//             multiple of 64 slots: the home bucket is the high half of hash * buckets), never grown.
struct Seen {
    ulonglong2 *T;
    unsigned long long *Tc;
    uint64_t mask;  // full table: slots - 1 (a power of two)
    uint64_t cap;   // slots; the compact table may have any number (home slot by multiply-shift)
};

enum ErrSlot { ERR_ASSERT = 0, ERR_DEADLOCK = 1, ERR_INV = 2, ERR_EVAL = 3, ERR_NSLOTS = 4 };

// Device-driven level loop (single GPU): the host enqueues several BFS levels without
// reading anything back.  Each level's kernels take their parent count, id bases, election
// epoch, table size and frontier ring positions from this block, which the previous level's
// commit wrote; once `stop` is set every later kernel returns at once.
enum CtlStop : uint32_t { CTL_RUN = 0, CTL_DONE = 1, CTL_ERROR = 2, CTL_HOST = 3 };
struct LevelCtl {
    unsigned long long cur_n;    // parents of the level being expanded
    unsigned long long gid_cur;  // global id of its first state
    unsigned long long T_count;  // fingerprints in the seen set
    unsigned long long Lmask;    // election table mask for this level
    unsigned long long cur_wbase, cur_words;  // ring position and words of the level being expanded
    // capacities (host-written before the batch)
    unsigned long long off_cap, rcap, trace_base, trace_cap, T_cap, chunk_parents, Lcap_max;
    uint32_t level;              // level being expanded (1 = Init's level)
    uint32_t epoch;              // election table epoch of this level
    uint32_t stop;               // CtlStop: RUN, DONE (empty level), ERROR, HOST (next level needs the host)
    uint32_t done_levels;        // levels committed in this batch (index into LevelRec)
    uint32_t batch;              // levels the host enqueued: the loop hands back after that many
    uint32_t pad_;
};
struct LevelRec { unsigned long long expanded, generated, new_states, words, self_loops; };
constexpr int LREC_CAP = 1024;   // levels per batch at most
// Device-loop mirror in pinned, mapped host memory: finish_level writes each level's record and
// the control block here, then the level count and (once the loop stops) the stop code with
// system-scope stores.  The host polls done / stop while the loop runs -- no event or copy in the
// stream between levels -- and reads the rest once the stream has drained.
struct HostLoop {
    uint32_t done;               // levels committed in this batch
    uint32_t stop;               // CtlStop; CTL_RUN while the loop runs
    uint32_t pad_[2];
    LevelCtl ctl;                // the control block as the last finished level left it
    LevelRec rec[LREC_CAP];
};
constexpr uint32_t WTILE = 1024; // parents per tile of the winner-count scan
constexpr uint32_t WTILES_MAX = 4096; // tiles per chunk (the last block scans four per thread)
constexpr int SUM_WORDS = 7;     // chunk summary slot of the new states' record words
constexpr int SUM_INS = 9;       // ... a sharded round's fingerprints inserted into the owner's seen set by k_owner_flags /
                                 // k_local_flags, and (SUM_INS_COMMIT) by a split round's commit (its own winners)
constexpr int SUM_INS_COMMIT = 10;
constexpr int SUM_NZ = 16;       // ... and of the parents with winners (KParams::plist)
constexpr int SUM_SELF = 17;     // ... and the self-loops set apart (KParams::hcnt, or a host-driven fused chunk's;
                                 // zeroed by the host per chunk)
constexpr int SUM_HFP = 18;      // ... and a split chunk's successors to fingerprint (its expansion counts them; the
                                 // election of k_hash_probe takes a table of twice as many slots; zeroed with SUM_SELF)
constexpr int SUM_OCNT = 20;     // ... a sharded round's successors per owner shard (u32[64] over sum[20 .. 52): zeroed
                                 // with SUM_INS .. SUM_HFP by one memset per round)
// the fused expansion's self-loop counters: SELF_STRIPES words a 128-B line apart (block b adds to stripe
// b % SELF_STRIPES), folded by finish_level (k_set_ctl zeroes them for the device loop; 0 between levels)
constexpr int SUM_SELF_STRIPE = 64, SELF_STRIDE = 16, SELF_STRIPES = 8;  // sum[64 .. 176]
constexpr int SUM_WORDS_TOTAL = 192;  // the chunk summary's words

// In device-loop mode the host sizes every grid on a bound of the level's parents (p_end -
// p_begin of the KParams it passes); the kernels read the real range from the LevelCtl.

// Kernel parameters (passed by value).
struct KParams {
    Dims d;
    int E, R, seeded, check_deadlock;
    uint32_t inv_mask;
    uint32_t inv_order;        // invariants in cfg order, 4 bits each (id + 1), 0 = end of list
    Tables t;
    // current level: records in the frontier ring, word k of parent p at
    // front[ring_wrap(fbase + foff[p] + k, rcap)]; foff == nullptr: fixed stride RECW_MAX, no ring
    const uint32_t *front;
    const uint64_t *foff;
    uint64_t fbase, rcap;
    uint64_t p_begin, p_end;   // parents of this chunk (level-local indices)
    // per parent (chunk-local: index p - p_begin)
    uint32_t *cnt;             // successor counts
    // split chunk (single GPU): successors per parent that need a fingerprint -- the expansion stages a
    // parent's self-loops (a successor equal to it: FollowerAcceptEntry of an entry it holds, already in
    // the seen set with the parent) after them, and every later pass of the chunk visits hcnt[pl] slots
    // only; nullptr: cnt (every successor)
    uint32_t *hcnt;
    // split chunk (single GPU): the first of each parent's successor slots, dense over the chunk -- the
    // expansion allocates a round's slots at a time (SUM_HFP), so fp / lslot / score are written and read
    // without the MAXS-per-parent stride of the sparse layout (q = parent * MAXS + rank, which the
    // election keys keep as TLC's order either way); nullptr: the sparse layout
    uint32_t *hoff;
    const uint32_t *off;       // exclusive scan of cnt (chunk-local successor index)
    // per successor (chunk-local index j)
    ulonglong2 *fp;
    const uint32_t *wflag;     // 1 = winner (new, first in TLC order)
    uint32_t *wpos;            // exclusive scan of wflag (fused level: of wcnt inside a tile)
    Seen seen;
    // next level: records in the same ring at nbase + noff[i]; noff holds level-relative offsets
    uint32_t *next;            // ring (== front) or a fixed-stride buffer (noff == nullptr)
    uint64_t *noff;
    uint64_t nbase;            // ring position of the next level's first word
    uint64_t next_wbase;       // level-relative word offset of this chunk's first winner
    uint64_t next_base;        // next-level index of this chunk's first winner
    // trace: parent global id + slot key, indexed by global id - trace_base
    uint64_t *par;
    uint16_t *pslot;
    uint64_t trace_base;
    uint64_t gid_next_base;    // global id of next-level index 0
    uint64_t gid_parent_base;  // global id of level-local parent 0
    // errors: atomicMin keys (p << 16 | slot), level-local p
    unsigned long long *err;
    uint32_t *flags;           // [0] msg-cap overflow, [1] violated invariant bit, [2] eval-error invariant bit
    // sharded round (W > 1): expand writes fingerprints only (the owners probe and elect), commit
    // takes lslot == LS_WIN as the verdict and writes each winner's trace entry to its sidecar
    // xside[i] = {parent global id lo, hi, slot key, record words} instead of par / pslot
    int route;
    uint4 *xside;
    uint32_t *ocnt;            // sharded split round: k_hash_probe counts the successors per owner here
    uint32_t nown;             // ... of that many owners (W)
    // ... and, with OT set, the shard's own successors bid in its owner table (k_local_elect's work):
    // lslot = LS_ELECT (another shard's), LS_SEEN, or the table slot; key (gblk + pl) << 10 | rank
    ESlot *OT;
    uint64_t ot_mask, gblk;
    uint32_t ot_round, self;
    // split chunk (host-driven chunks of many parents): the expansion (M_SPLIT) stages the successors
    // and writes each parent's hash context (hctx, ctx_words per parent), and k_hash_probe gives every
    // successor a lane of its own for its fingerprint, the seen-set probe and the election (bit 0);
    // bit 1: k_insert_winners puts the winners into the seen set, not the commit; bit 2: ... and leaves
    // its verdicts in lslot (LS_WIN / LS_SEEN) for the commit
    int split;
    uint32_t *hctx;
    // test variants: bit 0 RaftSplitBrain (BecomeLeader's quorum 1), bit 1 RaftCommitPastLog
    // (FollowerAcceptEntry's newCommitIndex without Min(., Len(newLog)))
    uint32_t quirks;
    // fused single-shard level: expand (+hash, +seen-set probe, +election, +staging) -> wincount
    // -> commit.  Successor slot q = (p - p_begin) * maxsucc + rank is sparse and increases in
    // TLC order; it indexes fp, lslot and score (the staged successor: its acting server's row,
    // slot key and added message ids, Spec::SW4 uint4 each; stage_succ).  wpos / wposw are then
    // the exclusive scans of winners / their record words per parent inside each WTILE-parent
    // tile, and a parent's first winner lands at boff[tile] + wpos (words boffw[tile] + wposw).
    uint4 *score;
    uint32_t *lslot;           // LS_SEEN, LS_ELECT, or the election slot in ET
    ESlot *ET;                 // chunk election table: per slot the fingerprint, both words tagged with the
                               // chunk's 16-bit tag (elect_tag) in their low bits, and the election word
                               // ((0xFFFFFFFF - epoch) << 32) | q << 2 | e (elect_key)
    uint64_t Lmask;
    uint32_t epoch;
    uint32_t *wcnt;            // winners per parent (chunk-local)
    uint32_t *wacc;            // per parent, as the election counts them: winners | extra words << 12
    uint32_t *pnm;             // |msgs| per parent (chunk-local)
    uint32_t *wposw;           // record words of the parent's winners, exclusive scan inside the tile
    uint32_t *bw, *bg, *boff;  // per tile: winners, successors generated, first winner's offset
    uint32_t *bww, *boffw;     // per tile: winners' record words, first winner's word offset
    uint32_t *bn, *boffn;      // per tile: parents with winners, their exclusive scan (plist)
    uint32_t *plist;           // split chunk: the chunk-local indices of the parents with winners, in
                               // order (k_nzlist), sum[SUM_NZ] of them -- the commit's waves visit only
                               // these; nullptr: every parent of the chunk
    uint32_t *tickets;         // [0] winner-count pass: last-block counter (0 between launches)
    uint32_t *ctick;           // commit pass: arrival counters (last_commit_block; 0 between launches)
    unsigned long long *sum;   // chunk summary {generated, winners, error keys[ERR_NSLOTS], flags, words}
    LevelCtl *ctl;             // device-driven level loop (nullptr: the host drives the chunk)
    LevelCtl *ctl_next;        // device loop: the block the next level reads (finish_level writes it)
    LevelRec *lrec;            // statistics of each level the device loop commits
    HostLoop *hloop;           // device loop: host-mapped mirror of the loop's progress (k_expand, finish_level)
    uint32_t done_levels;      // device loop: levels of the batch committed before this one (level_args)
    // single-state hook outputs
    uint32_t *out_keys;
    uint32_t *out_count;
};

struct KernelSet {
    int N, V, MR, MCAP, CCW, RECW_MAX, maxsucc;
    int ctxw;                                                 // hash-context words per parent (split chunks)
    void (*single)(const KParams &, hipStream_t);           // all successors of front[0] -> next, fp, out_keys
    void (*fused)(const KParams &, hipStream_t);            // expand + hash + probe + election + staging
    void (*split)(const KParams &, hipStream_t);            // split chunk: expand + staging + hash context
    void (*hash_probe)(const KParams &, uint64_t np, hipStream_t);  // split chunk: fingerprint + seen set + election
                                                                   // per successor (P.route: fingerprint only)
    void (*insert)(const KParams &, uint64_t np, hipStream_t);    // split chunk: winners into the seen set
    void (*wincount)(const KParams &, uint64_t np, hipStream_t);  // winners per parent + their scan, successors generated
    void (*commit)(const KParams &, hipStream_t);           // winners -> next level, seen set, trace, invariants;
                                                            // chunk summary (and the device loop's next level)
    void (*commit_split)(const KParams &, uint64_t np, hipStream_t);  // ... a lane per successor slot of the parents
                                                            // with winners (plist; LS_WIN verdicts) + summary
    // sharded round, the successors the shard owns itself: bids in the round's owner table, then
    // (every bid in) verdicts in lslot, winners into the seen set and onto wacc
    void (*local_elect)(const KParams &, uint64_t np, Seen, ESlot *OT, uint64_t mask,
                        uint32_t round, uint32_t W, uint32_t self, uint64_t g0, hipStream_t);
    void (*local_flags)(const KParams &, uint64_t np, Seen, const ESlot *OT, uint32_t round, uint32_t W,
                        uint32_t self, uint64_t g0, unsigned long long *inserted, hipStream_t);
    void (*fp_states)(const KParams &, uint64_t n, hipStream_t);  // fp of front[0..n) -> fp
    void (*inv_states)(const KParams &, uint64_t n, int32_t *out, hipStream_t); // per state: 1/0/-1 for inv_mask bits
    // host codec of the packed core (rmc_spec.h Codec)
    void (*encode)(const uint32_t *nibble_core, uint32_t *packed);
    void (*decode)(const uint32_t *packed, uint32_t *nibble_core);
};

// returns false if (N, V) has no compiled instantiation; become_follower: the tla:420 variant's kernels
// (BecomeFollower candidates, maxsucc larger by msg_cap)
bool get_kernels(int N, int V, int msg_cap, bool become_follower, KernelSet *ks);

// generic (template-free) kernels
constexpr uint32_t LS_SEEN = 0xFFFFFFFFu, LS_ELECT = 0xFFFFFFFEu, LS_WIN = 0xFFFFFFFDu;
// full-slot table -> (full or compact) table
void launch_rehash(const ulonglong2 *Told, uint64_t old_cap, Seen dst, hipStream_t s);
// every slot free: fingerprint words 0, election word all ones (older than every epoch / round)
void launch_eslot_clear(ESlot *t, uint64_t n, hipStream_t s);
void launch_insert_fps(const ulonglong2 *fp, uint64_t n, Seen seen, hipStream_t s);
// the control block of a device-driven batch, passed by value (no copy-engine hand-off)
void launch_set_ctl(LevelCtl *dst, int n, const LevelCtl &v, unsigned long long *gen, hipStream_t s);
// Init's level from the cached Init record and fingerprint: record into the ring at word 0, its
// offset 0, its fingerprint into the seen set
void launch_init_level(uint32_t *ring, const uint32_t *rec, uint32_t words, uint64_t *off,
                       const ulonglong2 *fp, Seen seen, hipStream_t s);
// out[i] = in[i] - sub (offset arrays rebased to a new level start)
void launch_rebase(const uint64_t *in, uint64_t n, uint64_t sub, uint64_t *out, hipStream_t s);
// after the winner count of a chunk with P.plist: the list of its parents with winners
void launch_nzlist(const KParams &P, uint64_t np, hipStream_t s);

// sharded round (W > 1), rmc_engine.hip step_sharded: a successor on its way to its fingerprint's
// owner shard -- the fingerprint and its global key (owner_order: parent's index in the level, rank)
struct XItem { unsigned long long x, y, key; };
void launch_route_count(const ulonglong2 *fp, const uint32_t *cnt, uint64_t np, uint32_t maxsucc, uint32_t W,
                        uint32_t *ocnt, hipStream_t s);
void launch_route_place(const ulonglong2 *fp, const uint32_t *cnt, uint64_t np, uint32_t maxsucc, uint32_t W,
                        uint32_t *cursor, uint64_t g0, XItem *items, uint32_t *perm, uint32_t self, hipStream_t s);
// (wacc, g0, np: the owner's own parents of the round, whose winners the bids count -- owner_bid)
void launch_owner_elect(const XItem *it, uint64_t R, Seen seen, ESlot *OT, uint64_t mask,
                        uint32_t round, uint32_t *rslot, uint32_t *wacc, uint64_t g0, uint64_t np, hipStream_t s);
void launch_owner_flags(const XItem *it, uint64_t R, const uint32_t *rslot, const ESlot *OT, uint32_t round,
                        Seen seen, uint32_t *flag, unsigned long long *inserted, hipStream_t s);
void launch_scatter_win(const uint32_t *perm, const uint32_t *flag, uint64_t G, const uint4 *score, uint32_t sw4,
                        const uint32_t *pnm, uint32_t maxsucc, uint32_t *lslot, uint32_t *wacc, hipStream_t s);
void launch_side_sizes(const uint4 *side, uint64_t n, uint32_t *sz, hipStream_t s);
void launch_accept_side(const uint4 *side, const uint32_t *off, uint64_t n, uint64_t rel0, uint64_t *noff,
                        uint64_t *par, uint16_t *pslot, hipStream_t s);
void launch_owner_of(const ulonglong2 *fp, uint32_t W, uint32_t *out, hipStream_t s);
// out[i] = 1 if fp[i] is in `seen` -- for the fingerprints the shard `self` of W owns (W = 1: all)
void launch_seen_query(const ulonglong2 *fp, uint64_t n, Seen seen, uint32_t W, uint32_t self, uint8_t *out,
                       hipStream_t s);

}  // namespace rmc
