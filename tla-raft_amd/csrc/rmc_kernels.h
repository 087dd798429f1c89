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
    const uint8_t *perms;     // [np][MAXN] server permutations (pi[i] = image of i)
    const uint64_t *seeds;    // [2][MAXN + MAXN*MAXN] position seeds of the structured hash
    int np;
};

enum ErrSlot { ERR_ASSERT = 0, ERR_DEADLOCK = 1, ERR_INV = 2, ERR_EVAL = 3, ERR_NSLOTS = 4 };

// Device-driven level loop (single GPU): the host enqueues several BFS levels without
// reading anything back.  Each level's kernels take their parent count, id bases,
// election epoch and table size from this block, which the previous level's commit
// wrote; once `stop` is set every later kernel returns at once.
enum CtlStop : uint32_t { CTL_RUN = 0, CTL_DONE = 1, CTL_ERROR = 2, CTL_HOST = 3 };
struct LevelCtl {
    unsigned long long cur_n;    // parents of the level being expanded
    unsigned long long gid_cur;  // global id of its first state
    unsigned long long T_count;  // fingerprints in the seen set
    unsigned long long Lmask;    // election table mask for this level
    // capacities (host-written before the batch)
    unsigned long long nxt_cap, trace_cap, T_cap, chunk_parents, Lcap_max;
    uint32_t level;              // level being expanded (1 = Init's level)
    uint32_t epoch;              // election table epoch of this level
    uint32_t stop;               // CtlStop: RUN, DONE (empty level), ERROR, HOST (next level needs the host)
    uint32_t done_levels;        // levels committed in this batch (index into LevelRec)
    uint32_t batch;              // levels the host enqueued: the loop hands back after that many
    uint32_t pad_;
};
struct LevelRec { unsigned long long expanded, generated, new_states; };
constexpr int LREC_CAP = 1024;   // levels per batch at most
constexpr uint32_t WTILE = 1024; // parents per tile of the winner-count scan (1024 tiles at most)

// In device-loop mode the host sizes every grid on a bound of the level's parents (p_end -
// p_begin of the KParams it passes); the kernels read the real range from the LevelCtl.

// Kernel parameters (passed by value).
struct KParams {
    Dims d;
    int E, R, seeded, check_deadlock;
    uint32_t inv_mask;
    Tables t;
    // current level
    const uint32_t *front;     // records, RECW words each
    uint64_t p_begin, p_end;   // parents of this chunk (level-local indices)
    // per parent (chunk-local: index p - p_begin)
    uint32_t *cnt;             // successor counts
    const uint32_t *off;       // exclusive scan of cnt (chunk-local successor index)
    // per successor (chunk-local index j)
    ulonglong2 *fp;
    const uint32_t *wflag;     // 1 = winner (new, first in TLC order)
    uint32_t *wpos;            // exclusive scan of wflag (fused level: of wcnt inside a tile)
    // seen set (open addressing, 16-B slots, lo word |= 1, 0 = empty)
    ulonglong2 *T;
    uint64_t Tmask;
    // next level
    uint32_t *next;            // records
    uint64_t next_base;        // next-level index of this chunk's first winner
    uint64_t *par;             // parent global id, indexed by global id
    uint16_t *pslot;           // slot key, indexed by global id
    uint64_t gid_next_base;    // global id of next-level index 0
    uint64_t gid_parent_base;  // global id of level-local parent 0
    // errors: atomicMin keys (p << 16 | slot), level-local p
    unsigned long long *err;
    uint32_t *flags;           // [0] msg-cap overflow, [1] violated invariant bit, [2] eval-error invariant bit
    // sharded mode: winners go to owner-grouped exchange records (RECW + 4 words each)
    uint32_t *xrec;
    // fused single-shard level: expand (+hash, +seen-set probe, +election, +staging) -> wincount
    // -> scan -> commit.  Successor slot q = (p - p_begin) * maxsucc + rank is sparse and
    // increases in TLC order; it indexes fp, lslot, score (core words, CW/4 uint4 each) and
    // saux {key | nadd << 16, add0 | add1 << 16, add2 | add3 << 16, 0}.  wpos is then the
    // exclusive scan of wcnt (winners per parent) inside each WTILE-parent tile, and a
    // parent's first winner lands at boff[tile] + wpos.
    uint4 *score;
    uint4 *saux;
    uint32_t *lslot;           // LS_SEEN, LS_ELECT, or the election slot in L
    unsigned long long *L;     // chunk election table: sharded path (epoch << 32) | q; fused path
                               // the election word ((0xFFFFFFFF - epoch) << 32) | q (elect_key)
    ulonglong2 *LXY;           // fused path: the fingerprint each election slot holds, both words
                               // tagged with the chunk's 16-bit tag (elect_tag) in their low bits
    uint64_t Lmask;
    uint32_t epoch;
    uint32_t *wcnt;            // winners per parent (chunk-local)
    uint32_t *wacc;            // winners per parent as the election counts them (0 between chunks)
    uint32_t *bw, *bg, *boff;  // per tile: winners, successors generated, first winner's offset
    uint32_t *tickets;         // [0] winner-count pass: last-block counter (0 between launches)
    uint32_t *ctick;           // commit pass: arrival counters (last_commit_block; 0 between launches)
    unsigned long long *sum;   // chunk summary {generated, winners, error keys[ERR_NSLOTS], flags}
    LevelCtl *ctl;             // device-driven level loop (nullptr: the host drives the chunk)
    LevelRec *lrec;            // statistics of each level the device loop commits
    // single-state hook outputs
    uint32_t *out_keys;
    uint32_t *out_count;
};

struct KernelSet {
    int N, V, MR, MCAP, CW, RECW, maxsucc;
    void (*count)(const KParams &, hipStream_t);
    void (*hash)(const KParams &, hipStream_t);
    void (*materialize)(const KParams &, hipStream_t);
    void (*single)(const KParams &, hipStream_t);           // all successors of front[0] -> next, fp, out_keys
    void (*fused)(const KParams &, hipStream_t);            // expand + hash + probe + election + staging
    void (*wincount)(const KParams &, uint64_t np, hipStream_t);  // winners per parent + their scan, successors generated
    void (*commit)(const KParams &, hipStream_t);           // winners -> next level, seen set, trace, invariants;
                                                            // chunk summary (and the device loop's next level)
    void (*fp_states)(const KParams &, uint64_t n, hipStream_t);  // fp of front[0..n) -> fp
    void (*inv_states)(const KParams &, uint64_t n, int32_t *out, hipStream_t); // per state: 1/0/-1 for inv_mask bits
};

// returns false if (N, V) has no compiled instantiation
bool get_kernels(int N, int V, int msg_cap, KernelSet *ks);

// generic (template-free) kernels
void launch_dedup(const ulonglong2 *fp, const uint32_t *Gp, uint64_t Gub, const ulonglong2 *T, uint64_t Tmask,
                  unsigned long long *L, uint64_t Lmask, uint32_t epoch, uint32_t *lslot, hipStream_t s);
void launch_winflag(const uint32_t *lslot, const unsigned long long *L, const uint32_t *Gp, uint64_t Gub,
                    uint32_t *wflag, hipStream_t s);
void launch_summary(const uint32_t *Gp, const uint32_t *wpos, const unsigned long long *err, const uint32_t *flags,
                    unsigned long long *out, hipStream_t s);
constexpr uint32_t LS_SEEN = 0xFFFFFFFFu, LS_ELECT = 0xFFFFFFFEu;
void launch_scan_small(const uint32_t *in, uint64_t n, uint32_t *out, hipStream_t s);
void launch_winscan_small(const uint32_t *lslot, const unsigned long long *L, const uint32_t *Gp, uint64_t Gub,
                          uint32_t *wflag, uint32_t *wpos, hipStream_t s);
void launch_owner_keys(const ulonglong2 *fp, uint64_t G, uint32_t W, uint32_t *key, uint32_t *iota,
                       unsigned long long *cnt, hipStream_t s);
void launch_gather_fp(const ulonglong2 *fp, const uint32_t *perm, uint64_t G, ulonglong2 *out, hipStream_t s);
void launch_recv_flags(const uint32_t *lslot, const unsigned long long *L, uint64_t R, uint32_t *flag, hipStream_t s);
void launch_scatter_flags(const uint32_t *perm, const uint32_t *sflag, const uint32_t *spos, uint64_t G,
                          uint32_t *wflag, uint32_t *wpos, hipStream_t s);
void launch_accept(const uint32_t *xrec, uint64_t n, uint32_t recw, uint32_t *next, uint64_t *par, uint16_t *pslot,
                   uint64_t src_tag, hipStream_t s);
void launch_insert_flagged(const ulonglong2 *fp, const uint32_t *flag, uint64_t n, ulonglong2 *T, uint64_t mask,
                           hipStream_t s);
void launch_pick(const uint32_t *a, const uint64_t *idx, int n, unsigned long long *out, hipStream_t s);
void launch_owner_of(const ulonglong2 *fp, uint32_t W, uint32_t *out, hipStream_t s);
void launch_rehash(const ulonglong2 *Told, uint64_t old_cap, ulonglong2 *Tnew, uint64_t new_mask, hipStream_t s);
void launch_insert_fps(const ulonglong2 *fp, uint64_t n, ulonglong2 *T, uint64_t Tmask, hipStream_t s);

}  // namespace rmc
