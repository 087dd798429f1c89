// rmc_kernels.hip -- CDNA4 (gfx950) kernels of the BFS hot path.
//
// One wavefront expands one frontier state ("parent").  Lane k of message round r
// owns message r*64+k of the parent's msgs set and evaluates every message-witness
// disjunct for it (UpdateTerm tla:175, ResponseVote tla:132, FollowerAcceptEntry
// tla:275, FollowerRejectEntry tla:302, HandleAppendResp tla:374 -- for a given
// message at most one is enabled, because they split on (role, type, term)).  The
// last round's lanes own the non-message slots (BecomeCandidate tla:107,
// BecomeLeader tla:157, ClientReq tla:233 per value, LeaderAppendEntry tla:242 per
// destination, LeaderCanCommit tla:398, Restart tla:409).  Enabling conditions are
// evaluated per lane; a ballot + in-wave rank by slot key puts the successors in
// TLC's enumeration order (Next, tla:416-430) without any sort.
//
// Frontier records live in a ring of 32-bit words: packed core (rmc_spec.h Codec) + the
// sorted u16 message ids, CCW + ceil(|msgs|/2) words each, located by a level-relative
// word offset per state.
//
// Modes of the same expansion:
//   COUNT        successors per parent (+ Assert tla:185 / deadlock detection)
//   HASH         symmetry+view fingerprint of every successor -> fp[off[p] + rank]
//   MATERIALIZE  winners (new states, first in TLC order) -> owner exchange records,
//                INVARIANT check (Raft.cfg:33)
//   SINGLE       every successor of one state -> records (parity-test hook)
//   FUSED        single-GPU level: expand + fingerprint + seen-set probe + election + staging
#include <hip/hip_runtime.h>


#include "rmc_kernels.h"

// waves per SIMD the n >= 4 / two-round expansion kernel is compiled for (register budget)
// phase profile (tools/phase_prof.py): a build with -DRMC_PHASE_PROF adds up, per phase of
// k_expand, the shader clock its waves spend there (lane 0 of each wave, flushed once per wave)
#ifdef RMC_PHASE_PROF
// (slots 0-7 k_expand, 8-15 k_commit: PHASE_BASE)
__device__ unsigned long long g_phase[16];
#define PHASE_DECL unsigned long long _acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; long long _tp = clock64();
#define PHASE(k) do { const long long _t = clock64(); _acc[k] += (unsigned long long)(_t - _tp); _tp = _t; } while (0)
#define PHASE_FLUSH_AT(b) do { if (threadIdx.x == 0) for (int _k = 0; _k < 8; _k++) atomicAdd(&g_phase[(b) + _k], _acc[_k]); } while (0)
#define PHASE_FLUSH PHASE_FLUSH_AT(0)
extern "C" int rmc_debug_phases(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 16;
}
#else
#define PHASE_DECL
#define PHASE(k) do {} while (0)
#define PHASE_FLUSH do {} while (0)
#define PHASE_FLUSH_AT(b) do {} while (0)
#endif

#ifndef RMC_N3_WAVES  // n = 3 expansion (and commit): waves per SIMD the register budget is cut for
#define RMC_N3_WAVES 4
#endif
#ifndef RMC_N3_COMMIT_WAVES
#define RMC_N3_COMMIT_WAVES 1
#endif
#ifndef RMC_GRID_PER_CU  // one-wave blocks per CU in the expansion / commit grids
#define RMC_GRID_PER_CU 32
#endif
#ifndef RMC_WIDE_WAVES
#define RMC_WIDE_WAVES 2
#endif

namespace rmc {

// SINGLE: every successor of one state (parity hook); FUSED: expand + fingerprint + staging, the
// fingerprints routed to their owners (sharded rounds below the split size).  Single-GPU levels and
// split chunks use the item-parallel k_expand_items.
enum Mode { M_SINGLE = 3, M_FUSED = 4 };

template <int N>
__device__ __forceinline__ uint32_t sel(const uint32_t *a, int i) {
    uint32_t r = a[0];
#pragma unroll
    for (int k = 1; k < N; k++) r = (i == k) ? a[k] : r;
    return r;
}

__device__ __forceinline__ uint32_t rdlane(uint32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, int l) {
    uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
    uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// exclusive prefix sum over the wave's lanes
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, int lane, uint32_t *total) {
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    *total = __shfl(x, 63, 64);
    return x - v;
}

// ---- race probe (a test build: -DRMC_RACE_PROBE, tools/build_variant.sh race) -----------------------
// Every place where blocks of one launch hand state to each other gets a forced worst-case schedule:
//   * the device loop's commit: the first block without a parent of its level waits until the
//     launch's last arriver has written the next level's control block, then reads its own -- the
//     late-block race of round 4, made to happen on every level;
//   * the last-arriver counters (k_wincount's tickets, k_commit's ticks): block 0 arrives last;
//   * the elections (elect_slot, owner_bid): a claimer holds its y word back, so candidates of the
//     same fingerprint find x claimed and y not yet visible.
// rmc_debug_race(1) switches the device loop back to one control block per level (read and written
// in place, the logic before the pair): with the late block forced, that must give wrong results.
#ifdef RMC_RACE_PROBE
__device__ int g_race_single = 0;
extern "C" int rmc_debug_race(int single) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_race_single), &single, sizeof single) == hipSuccess ? 0 : -1;
}
// the block a level reads and the one its commit writes (single: the pair's first block for both)
__device__ __forceinline__ LevelCtl *ctl_cur(const KParams &P) {
    return g_race_single ? (P.ctl < P.ctl_next ? P.ctl : P.ctl_next) : P.ctl;
}
__device__ __forceinline__ LevelCtl *ctl_nxt(const KParams &P) { return g_race_single ? ctl_cur(P) : P.ctl_next; }
// bounded wait: s_sleep 127 (~8 K clocks) up to `n` times while pred()
template <class F>
__device__ __forceinline__ void race_wait(int n, F &&pred) {
    for (int i = 0; i < n && pred(); i++) __builtin_amdgcn_s_sleep(127);
}
__device__ __forceinline__ void race_delay(int n) { race_wait(n, [] { return true; }); }
#else
__device__ __forceinline__ LevelCtl *ctl_cur(const KParams &P) { return P.ctl; }
__device__ __forceinline__ LevelCtl *ctl_nxt(const KParams &P) { return P.ctl_next; }
#endif

// ---- device-driven level loop -------------------------------------------------------------
// With P.ctl set, a level's kernels take the parent range, id bases, ring positions, election
// epoch and table size from the control block the previous level's commit wrote (a kernel
// boundary makes it visible); once the loop has stopped every block returns at once.
__device__ __forceinline__ bool level_args(KParams &P) {
    if (!P.ctl) return true;
    const LevelCtl *c = ctl_cur(P);
    if (c->stop != CTL_RUN) return false;
    P.done_levels = c->done_levels;
    P.p_begin = 0;
    P.p_end = c->cur_n;
    P.gid_parent_base = c->gid_cur;
    P.gid_next_base = c->gid_cur + c->cur_n;
    P.next_base = 0;
    P.next_wbase = 0;
    P.fbase = c->cur_wbase;
    P.nbase = ring_wrap(c->cur_wbase + c->cur_words, P.rcap);
    P.epoch = c->epoch;
    P.Lmask = c->Lmask;
    return true;
}

template <int N, int V, int MR>
struct Spec {
    using L = Layout<N, V>;
    static constexpr int NW = L::NW, CW = L::CW;
    static constexpr int CCW = Codec<N, V>::CCW;               // packed core words
    static constexpr int MCAP = 64 * MR;
    static constexpr int RECW_MAX = CCW + MCAP / 2;            // longest record
    static constexpr int NADD = (N > 1) ? N - 1 : 1;
    static constexpr int SLOTS_PER_SERVER = 4 + V + (N - 1);  // BC BL CR*V LAE*(N-1) LCC RS
    static_assert(N * SLOTS_PER_SERVER <= 64, "non-message slots must fit one wave");
    static constexpr int MAXS = MCAP + N * SLOTS_PER_SERVER;  // successor slots per parent (sparse stride)
    // staging of one successor (uint4s): its acting server's row -- the only part of the state an
    // action changes (see stage_succ) -- plus slot key, |added| and the added message ids
    static constexpr int SW4 = NADD > 2 ? 3 : 2;
};

// per-lane successor candidate
template <int N, int V, int MR>
struct Succ {
    uint32_t c[Spec<N, V, MR>::NW];
    uint32_t add[Spec<N, V, MR>::NADD];
    uint32_t nadd;
    uint32_t key;  // KEY_NONE = disabled
    uint32_t s;    // acting server (row of the structured hash that changed)
    uint32_t lw, mirow, nirow;  // logs[s], matchIndex[s][*], nextIndex[s][*] of the successor
    bool self;  // the parent itself (FollowerAcceptEntry changing nothing): in the seen set already
};

template <int N, int V, int MR>
__device__ __forceinline__ void succ_adds(const Succ<N, V, MR> &o, uint32_t *a01, uint32_t *a23) {
    uint32_t a[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < Spec<N, V, MR>::NADD; k++) a[k] = o.add[k];
    *a01 = a[0] | (a[1] << 16);
    *a23 = a[2] | (a[3] << 16);
}

// ---- log helpers (logs[i][x], tla:97, 1-based) ---------------------------------------
template <int N, int V>
__device__ __forceinline__ uint32_t log_word(const uint32_t *c, int i) {
    return sel<N>(c + Layout<N, V>::W_LOG, i);
}
__device__ __forceinline__ uint32_t lw_term(uint32_t lw, uint32_t x) {  // x >= 1
    return x <= 1 ? 0u : (lw >> (8 * (x - 2))) & 15u;
}
__device__ __forceinline__ uint32_t lw_byte(uint32_t lw, uint32_t x) {  // x >= 2: term | val<<4
    return (lw >> (8 * (x - 2))) & 0xFFu;
}

// m \in msgs for the parent of the wave: one LDS read of the wave's bitmap over the universe's ids
// (k_expand builds it with the parent: msg_bitmap); replaced a binary search over the sorted ids --
// a chain of up to 7 dependent LDS reads per test, several tests per successor kind
__device__ __forceinline__ bool in_msgs(const uint32_t *bm, uint32_t id) { return (bm[id >> 5] >> (id & 31u)) & 1u; }

// Median(F) (tla:70-75): smallest F[s] with |{p : F[p] <= F[s]}| >= k.
template <int N>
__device__ __forceinline__ uint32_t median_row(uint32_t row, uint32_t k) {
    uint32_t best = 15;
#pragma unroll
    for (int s = 0; s < N; s++) {
        uint32_t fs = nib(row, s), cnt = 0;
#pragma unroll
        for (int p = 0; p < N; p++) cnt += nib(row, p) <= fs;
        if (cnt >= k && fs < best) best = fs;
    }
    return best;
}

// ---- frontier ring access ---------------------------------------------------------------------
// First word of parent p's record: a level-relative offset into the ring, or a fixed stride.
template <int RECW_MAX>
__device__ __forceinline__ uint64_t rec_start(const KParams &P, uint64_t p) {
    return P.foff ? ring_wrap(P.fbase + P.foff[p], P.rcap) : p * (uint64_t)RECW_MAX;
}
__device__ __forceinline__ uint32_t ring_word(const uint32_t *ring, uint64_t start, uint32_t k, uint64_t rcap) {
    return ring[ring_wrap(start + k, rcap)];
}
// message id k of a record whose ids begin at word `start`
__device__ __forceinline__ uint32_t ring_id(const uint32_t *ring, uint64_t start, uint32_t k, uint64_t rcap) {
    return (ring_word(ring, start, k >> 1, rcap) >> ((k & 1u) * 16u)) & 0xFFFFu;
}
__device__ __forceinline__ void ring_put_id(uint32_t *ring, uint64_t start, uint32_t k, uint64_t rcap, uint32_t id) {
    const uint64_t w = ring_wrap(start + (k >> 1), rcap);
    reinterpret_cast<uint16_t *>(ring)[2 * w + (k & 1u)] = (uint16_t)id;
}

// ---- invariants (on a concrete state; TLC's left-to-right short-circuit) ---------------
// returns 1 TRUE, 0 FALSE, -1 evaluation error
template <int N, int V>
__device__ __forceinline__ int inv_lhace(const uint32_t *c) {  // LeaderHasAllCommittedEntries tla:491-499
    using Lo = Layout<N, V>;
    bool any = false;
#pragma unroll
    for (int p = 0; p < N; p++) any |= nib(c[Lo::W_ROLE], p) == LEA;
    if (!any) return 1;
#pragma unroll
    for (int l = 0; l < N; l++) {
        if (nib(c[Lo::W_ROLE], l) != LEA) continue;
        bool bad = false;
        const uint32_t ll_l = nib(c[Lo::W_LL], l), lw_l = c[Lo::W_LOG + l], ct_l = nib(c[Lo::W_CT], l);
#pragma unroll
        for (int p = 0; p < N; p++) {
            if (p == l || bad) continue;
            if (!(nib(c[Lo::W_CT], p) <= ct_l)) continue;
            const uint32_t ci_p = nib(c[Lo::W_CI], p);
            if (ci_p > ll_l) { bad = true; continue; }
            const uint32_t ll_p = nib(c[Lo::W_LL], p), lw_p = c[Lo::W_LOG + p];
            for (uint32_t i = 2; i <= ci_p; i++) {  // index 1 is [0,None] on both sides
                if (i > ll_p) return -1;                 // logs[p][index] out of domain (tla:499)
                if (lw_byte(lw_p, i) != lw_byte(lw_l, i)) { bad = true; break; }
            }
        }
        if (!bad) return 1;
    }
    return 0;
}

// The message set of the state an invariant is checked on: msgs only grow (SendMsg, tla:43-45),
// so a successor's set is its parent's sorted id list plus the ids its action added.
struct MsgView {
    const uint32_t *ring;  // parent's ids: ring words from `start` on
    uint64_t start, rcap;
    uint32_t nm;
    uint32_t add0, add1;   // added ids, two u16 each (staging layout)
    uint32_t nadd;
    const uint32_t *info;  // message info word by id
};

__device__ __forceinline__ uint32_t mv_id(const MsgView &mv, uint32_t k) {
    if (k < mv.nm) return ring_id(mv.ring, mv.start, k, mv.rcap);
    k -= mv.nm;
    const uint32_t w = k < 2 ? mv.add0 : mv.add1;
    return (k & 1u) ? (w >> 16) : (w & 0xFFFFu);
}

// NoAllCommit tla:451-481.  The state conjuncts come first in the formula, so the message scans
// (three \E m \in msgs, each short-circuiting on type before prevLogIndex/succ: no evaluation
// error is possible) run only for a (s1, s2, s3) that passes them.
// The words NoAllCommit reads, as scalars: the check is out of line (its message scans would
// swell the commit kernel), and an out-of-line call given a pointer to the core -- or an aggregate,
// passed in memory -- would put the core of every checked state on the stack.
template <int N, int V>
__device__ __noinline__ int inv_nac(uint32_t role, uint32_t ci, uint32_t ct, uint32_t m0, uint32_t m1, uint32_t m2,
                                    uint32_t m3, uint32_t m4, const uint32_t *ring, uint64_t start, uint64_t rcap,
                                    uint32_t nm, uint32_t add0, uint32_t add1, uint32_t nadd, const uint32_t *info) {
    struct { uint32_t role, ci, ct; } c{role, ci, ct};
    const MsgView mv{ring, start, rcap, nm, add0, add1, nadd, info};
    uint32_t mi_s1 = 0;
    for (int s1 = 0; s1 < N; s1++) {
        if (nib(c.role, s1) != LEA || nib(c.ci, s1) != 2) continue;
        mi_s1 = s1 == 0 ? m0 : s1 == 1 ? m1 : s1 == 2 ? m2 : s1 == 3 ? m3 : m4;
        for (int s2 = 0; s2 < N; s2++) {
            if (s2 == s1 || nib(c.role, s2) != FOL || nib(c.ci, s2) != 2 || nib(mi_s1, s2) != 2)
                continue;
            for (int s3 = 0; s3 < N; s3++) {
                if (s3 == s2 || nib(c.role, s3) != FOL) continue;
                const uint32_t t3 = nib(c.ct, s3);
                if (nib(c.ct, s1) != t3 || nib(c.ci, s3) != 1 || nib(mi_s1, s3) != 2)
                    continue;
                bool c1 = false, c2 = false, c3 = false;
                for (uint32_t k = 0; k < mv.nm + mv.nadd; k++) {
                    const uint32_t m = mv.info[mv_id(mv, k)];
                    const uint32_t ty = mi_type(m), sr = mi_src(m), ds = mi_dst(m);
                    if (ds == (uint32_t)s3 && sr == (uint32_t)s1 && mi_term(m) == t3 && ty == AREQ && mi_x1(m) == 1) c1 = true;
                    if (ds == (uint32_t)s1 && sr == (uint32_t)s3 && mi_term(m) == t3 && ty == ARESP && mi_x1(m) == 1 &&
                        mi_x2(m) == 1)
                        c2 = true;
                    if (ds == (uint32_t)s3 && sr == (uint32_t)s1 && ty == AREQ && mi_x1(m) == 2) c3 = true;
                }
                if (c1 && c2 && c3) return 1;
            }
        }
    }
    return 0;
}

template <int N, int V>
__device__ __forceinline__ int inv_eval(const uint32_t *c, int id, const MsgView &mv) {
    using Lo = Layout<N, V>;
    switch (id) {
    case 0: return inv_lhace<N, V>(c);
    case 5: {
        uint32_t mi[5] = {0, 0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < N; q++) mi[q] = c[Lo::W_MI + q];
        return inv_nac<N, V>(c[Lo::W_ROLE], c[Lo::W_CI], c[Lo::W_CT], mi[0], mi[1], mi[2], mi[3], mi[4], mv.ring,
                             mv.start, mv.rcap, mv.nm, mv.add0, mv.add1, mv.nadd, mv.info);
    }
    case 1: {  // NoSplitVote tla:444-448
#pragma unroll
        for (int a = 0; a < N; a++)
#pragma unroll
            for (int b = 0; b < N; b++)
                if (a != b && nib(c[Lo::W_CT], a) == nib(c[Lo::W_CT], b) && nib(c[Lo::W_ROLE], a) == LEA &&
                    nib(c[Lo::W_ROLE], b) == LEA)
                    return 0;
        return 1;
    }
    case 2: {  // RaftCanCommt tla:434
#pragma unroll
        for (int s = 0; s < N; s++) if (nib(c[Lo::W_CI], s) > 1) return 1;
        return 0;
    }
    case 3: {  // FollowerCanCommit tla:436-439
#pragma unroll
        for (int s = 0; s < N; s++) if (nib(c[Lo::W_ROLE], s) == FOL && nib(c[Lo::W_CI], s) > 1) return 1;
        return 0;
    }
    case 4: {  // CommitAll tla:442
#pragma unroll
        for (int s = 0; s < N; s++) if (nib(c[Lo::W_CI], s) != 3) return 0;
        return 1;
    }
    case 6: {  // ExistLeaderAndCandidate tla:483-487
#pragma unroll
        for (int a = 0; a < N; a++)
#pragma unroll
            for (int b = 0; b < N; b++)
                if (a != b && nib(c[Lo::W_ROLE], a) == LEA && nib(c[Lo::W_ROLE], b) == CAN) return 1;
        return 0;
    }
    default: return 1;
    }
}

// The selected invariants in the order the cfg lists them (TLC checks them in that order,
// Raft.cfg:33-34): P.inv_order holds id + 1 per nibble, first invariant in the low nibble.
// Returns 1 ok, 0 violated, -1 eval error; *which = the invariant's id (bit).
template <int N, int V>
__device__ __forceinline__ int check_invs(const uint32_t *c, uint32_t order, int *which, const MsgView &mv) {
    for (; order; order >>= 4) {
        const int i = (int)(order & 15u) - 1;
        const int r = inv_eval<N, V>(c, i, mv);
        if (r != 1) { *which = i; return r; }
    }
    return 1;
}

// ---- symmetry fingerprint (rmc_spec.h: content matrix, position constants, signature coset) -----
// The fingerprint is the minimum over permutations pi of H(pi) = sum_{t,j} C[t][j] K[pi(t)][pi(j)].
// Any permutation-equivariant signature of a server (a function of its data that does not name
// other servers) orders the servers; taking the minimum only over the permutations that send the
// servers to their signature-sorted positions (the coset fixed by the signature ties) is still
// constant on every symmetry class (Raft.tla:21 SYMMETRY): for y = sigma(x) the allowed set of y is
// that of x composed with sigma^-1.  The signature is the server's row sum of C_1 -- its own word and
// its outgoing pair contents (message hashes to each peer, matchIndex / nextIndex / vote for it).
// Without SYMMETRY the identity is the only permutation (coset_ident).

// per server t, 6 bits: lo_t (servers with a smaller signature) | (ties_t - 1) << 3
template <int N>
__device__ __forceinline__ uint32_t coset_ranks(const uint64_t *sig) {
    uint32_t rk = 0;
#pragma unroll
    for (int t = 0; t < N; t++) {
        uint32_t lo = 0, eq = 0;
#pragma unroll
        for (int u = 0; u < N; u++) {
            lo += sig[u] < sig[t] ? 1u : 0u;
            eq += (u != t && sig[u] == sig[t]) ? 1u : 0u;
        }
        rk |= (lo | (eq << 3)) << (6 * t);
    }
    return rk;
}
// no symmetry: server t at position t, no ties
template <int N>
__device__ __forceinline__ uint32_t coset_ident() {
    uint32_t rk = 0;
#pragma unroll
    for (int t = 0; t < N; t++) rk |= (uint32_t)t << (6 * t);
    return rk;
}
__device__ __forceinline__ uint32_t small_fact(uint32_t g) {
    return g <= 1 ? 1u : g == 2 ? 2u : g == 3 ? 6u : g == 4 ? 24u : 120u;
}
// number of allowed permutations: product over tie groups of |group|!
template <int N>
__device__ __forceinline__ uint32_t coset_size(uint32_t rk) {
    uint32_t K = 1;
#pragma unroll
    for (int t = 0; t < N; t++) {
        const uint32_t lo = (rk >> (6 * t)) & 7u, g = ((rk >> (6 * t + 3)) & 7u) + 1u;
        bool head = true;
#pragma unroll
        for (int u = 0; u < t; u++) head &= ((rk >> (6 * u)) & 7u) != lo;
        if (head) K *= small_fact(g);
    }
    return K;
}
// the k-th allowed permutation (k < coset_size), packed: server t goes to position (img >> 3t) & 7.
// Tie groups in server order, each group's members (in server order) take the positions
// [lo, lo + g) in the k-th arrangement (factorial number system, group by group).  (Packed, not an
// array: the group members' positions are computed at run time, and an array written that way
// lives in scratch.)
template <int N>
__device__ __forceinline__ uint32_t coset_img(uint32_t rk, uint32_t k) {
    uint32_t img = 0;
#pragma unroll
    for (int t = 0; t < N; t++) {
        const uint32_t lo = (rk >> (6 * t)) & 7u, g = ((rk >> (6 * t + 3)) & 7u) + 1u;
        if (g == 1u) {  // untied: its position is its rank
            img |= lo << (3 * t);
            continue;
        }
        bool head = true;
#pragma unroll
        for (int u = 0; u < t; u++) head &= ((rk >> (6 * u)) & 7u) != lo;
        if (!head) continue;
        const uint32_t gf = small_fact(g);
        uint32_t kg = k % gf;
        k /= gf;
        uint32_t avail = (1u << g) - 1u, i = 0;
#pragma unroll
        for (int u = t; u < N; u++) {
            if (((rk >> (6 * u)) & 7u) != lo) continue;
            const uint32_t f = small_fact(g - 1u - i);
            uint32_t d = kg / f;
            kg -= d * f;
            uint32_t m = avail;
            for (; d; d--) m &= m - 1u;
            const uint32_t pos = (uint32_t)__builtin_ctz(m);
            avail &= ~(1u << pos);
            img |= (lo + pos) << (3 * u);
            i++;
        }
    }
    return img;
}
// H_f at one permutation (packed as coset_img): sum over the content matrix C(f, t, j) (diagonal:
// own word) of the position constant K(f, pi(t), pi(j))
template <int N, class FC, class FK>
__device__ __forceinline__ ulonglong2 hash_at(uint32_t img, FC C, FK K) {
    uint64_t h0 = 0, h1 = 0;
#pragma unroll
    for (int t = 0; t < N; t++) {
        const uint32_t it = (img >> (3 * t)) & 7u;
#pragma unroll
        for (int j = 0; j < N; j++) {
            const uint32_t ij = (img >> (3 * j)) & 7u;
            h0 += C(0, t, j) * K(0, it, ij);
            h1 += C(1, t, j) * K(1, it, ij);
        }
    }
    return make_ulonglong2(h0, h1);
}
__device__ __forceinline__ bool lex_less(ulonglong2 a, ulonglong2 b) {  // (h1, h0) order
    return a.y < b.y || (a.y == b.y && a.x < b.x);
}

// Per-server and per-pair inputs of the content matrix, from the words of one row.
template <int N>
__device__ __forceinline__ uint64_t own_word(uint32_t vfw, uint32_t ctw, uint32_t rolew, uint32_t ciw, uint32_t llw,
                                             uint32_t lw, uint32_t mirow, uint32_t nirow, uint32_t i) {
    const uint32_t vf = nib(vfw, i);
    const uint32_t vrel = vf == VF_NONE ? 0u : (vf == i ? 1u : 2u);
    const uint32_t own = vrel | (nib(ctw, i) << 2) | (nib(rolew, i) << 6) | (nib(ciw, i) << 10) |
                         (nib(llw, i) << 14) | (nib(mirow, i) << 18) | (nib(nirow, i) << 22);
    return ((uint64_t)lw << 32) | own;
}
__device__ __forceinline__ uint64_t pair_small(uint32_t mirow, uint32_t nirow, uint32_t vf_i, uint32_t j) {
    return (uint64_t)(nib(mirow, j) | (nib(nirow, j) << 4) | ((vf_i == j) ? 256u : 0u));
}
// content C_f[t][j] of row t from its words and its message-hash sums toward j (Ms0/Ms1)
template <int N>
__device__ __forceinline__ uint64_t content(int f, uint32_t t, uint32_t j, const uint32_t *c, uint32_t lw_t,
                                            uint32_t mirow, uint32_t nirow, uint64_t Ms) {
    using Lo = Layout<N, 1>;
    if (t == j)
        return cmix_own(own_word<N>(c[Lo::W_VF], c[Lo::W_CT], c[Lo::W_ROLE], c[Lo::W_CI], c[Lo::W_LL], lw_t, mirow,
                                    nirow, t),
                        f);
    const uint64_t sm = pair_small(mirow, nirow, nib(c[Lo::W_VF], t), j);
    return cmix_pair(Ms ^ (sm * (f ? PAIR_K1 : PAIR_K0)), f);
}

// The fingerprint of a whole state: nibble core c, message-hash sums M_f[t * N + j] (src t, dst j).
template <int N, int V>
__device__ __forceinline__ ulonglong2 fingerprint(const uint32_t *c, const uint64_t *M0, const uint64_t *M1,
                                                  const Tables &t) {
    using Lo = Layout<N, V>;
    uint64_t C0[N * N], C1[N * N], sig[N];
#pragma unroll
    for (int i = 0; i < N; i++) {
        sig[i] = 0;
#pragma unroll
        for (int j = 0; j < N; j++) {
            C0[i * N + j] = content<N>(0, i, j, c, c[Lo::W_LOG + i], c[Lo::W_MI + i], c[Lo::W_NI + i], M0[i * N + j]);
            C1[i * N + j] = content<N>(1, i, j, c, c[Lo::W_LOG + i], c[Lo::W_MI + i], c[Lo::W_NI + i], M1[i * N + j]);
            sig[i] += C1[i * N + j];
        }
    }
    const uint32_t rk = t.np > 1 ? coset_ranks<N>(sig) : coset_ident<N>(), K = coset_size<N>(rk);
    ulonglong2 best = make_ulonglong2(~0ull, ~0ull);
    for (uint32_t k = 0; k < K; k++) {
        const ulonglong2 h = hash_at<N>(
            coset_img<N>(rk, k), [&](int f, int a, int b) { return f ? C1[a * N + b] : C0[a * N + b]; },
            [&](int f, uint32_t a, uint32_t b) { return t.seeds[f * SEEDS_PER_F + a * MAXN + b]; });
        if (lex_less(h, best)) best = h;
    }
    return make_ulonglong2(best.x | 1ull, best.y);
}
constexpr int factorial(int n) { return n <= 1 ? 1 : n * factorial(n - 1); }

// ---- expansion of one parent per wavefront ------------------------------------------------
template <int N, int V, int MR>
struct Wave {
    using S = Spec<N, V, MR>;
    using Lo = Layout<N, V>;
    uint32_t c[S::NW];   // parent core (wave-uniform), constant-index reads
    const uint32_t *lds; // same core in LDS [NW] + vpcnt [N]: runtime-indexed reads
    uint32_t nm;
    uint64_t idw;        // ring position of the parent's first message-id word
    uint32_t id[MR];     // message id owned by this lane per round (0xFFFF = none)
    uint32_t inf[MR];
    const uint32_t *bm;  // LDS bitmap of the parent's message ids (msg_bitmap)
};

// The wave's parent's ids as a bitmap in LDS (bmw words): cleared, then one LDS OR per message.
template <int N, int V, int MR>
__device__ __forceinline__ void msg_bitmap(uint32_t *bm, uint32_t bmw, const Wave<N, V, MR> &W, int lane) {
    for (uint32_t i = (uint32_t)lane; i < bmw; i += 64) bm[i] = 0u;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MR; r++)
        if ((uint32_t)(r * 64 + lane) < W.nm) atomicOr(&bm[W.id[r] >> 5], 1u << (W.id[r] & 31u));
    __syncthreads();
}

// ---- message-id lookups of the actions, issued before any branch -------------------------------
// An action that sends a message looks its id up in nat2id; done inside the divergent action
// branches, every branch the wave takes paid its own round trip.  These compute the same table
// indices under the same guards as eval_msg / eval_slot, and the loads go out together for the
// whole wave (one round trip), their values passed in.
constexpr uint32_t NAT_NONE = 0xFFFFFFFFu;

// the message lane's lookup (round r): ResponseVote's VoteResp, FollowerAccept/RejectEntry's AppendResp
template <int N, int V, int MR>
__device__ __forceinline__ uint32_t msg_nat(const KParams &P, const Wave<N, V, MR> &W, int r, int lane) {
    using Lo = Layout<N, V>;
    const uint32_t k = (uint32_t)(r * 64 + lane);
    if (k >= W.nm) return NAT_NONE;
    const uint32_t m = W.inf[r];
    const uint32_t s = mi_dst(m), typ = mi_type(m), mt = mi_term(m), src = mi_src(m);
    const uint32_t ct = nib(W.c[Lo::W_CT], s), role = nib(W.c[Lo::W_ROLE], s);
    if (mt != ct || role != FOL) return NAT_NONE;
    if (typ == VREQ) return nat_vresp(P.d, s, src, mt);
    if (typ != AREQ) return NAT_NONE;
    const uint32_t ll = nib(W.c[Lo::W_LL], s), lw = W.lds[Lo::W_LOG + s];
    const uint32_t pli = mi_x1(m), plt = mi_x2(m), ent = mi_ent(m);
    const bool match = pli <= ll && plt == lw_term(lw, pli);  // LogMatch tla:271-273
    return match ? nat_aresp(P.d, s, src, mt, pli + ent, 1) : nat_aresp(P.d, s, src, mt, pli, 0);
}

// the slot lane's lookups: BecomeCandidate's VoteReqs to the N - 1 peers, LeaderAppendEntry's AppendReq
template <int N, int V, int MR>
__device__ __forceinline__ void slot_nats(const KParams &P, const Wave<N, V, MR> &W, int lane, uint32_t (&nat)[N - 1]) {
    using Lo = Layout<N, V>;
    using S = Spec<N, V, MR>;
#pragma unroll
    for (int i = 0; i < N - 1; i++) nat[i] = NAT_NONE;
    if (lane >= N * S::SLOTS_PER_SERVER) return;
    const uint32_t s = (uint32_t)lane / S::SLOTS_PER_SERVER, t = (uint32_t)lane % S::SLOTS_PER_SERVER;
    const uint32_t role = nib(W.c[Lo::W_ROLE], s), ct = nib(W.c[Lo::W_CT], s), ll = nib(W.c[Lo::W_LL], s);
    const uint32_t lw = W.lds[Lo::W_LOG + s];
    if (t == 0) {  // BecomeCandidate's guards (eval_slot)
        if (!((int)(W.c[Lo::W_MISC] & 15u) < P.E) || !(role == FOL || role == CAN)) return;
        const uint32_t term = ct + 1, llt = lw_term(lw, ll);
        // nat[i] = the i-th peer's VoteReq: peer i below s, i + 1 from s on (constant indices only)
#pragma unroll
        for (int i = 0; i < N - 1; i++) {
            const uint32_t p = (uint32_t)i < s ? (uint32_t)i : (uint32_t)i + 1u;
            nat[i] = nat_vreq(P.d, s, p, term, ll, llt);
        }
        return;
    }
    if (t >= 2 + (uint32_t)V && t < 2 + (uint32_t)V + (N - 1)) {  // LeaderAppendEntry's guards (eval_slot)
        const uint32_t q = t - 2 - V;
        const uint32_t dst = q < s ? q : q + 1;
        if (role != LEA) return;
        const uint32_t ni = nib(W.lds[Lo::W_NI + s], dst);
        if (!(ni <= ll + 1)) return;
        if ((W.c[Lo::W_PEND] >> (s * N + dst)) & 1u) return;
        const uint32_t pli = ni - 1, plt = lw_term(lw, pli);
        const uint32_t ent = ni <= ll ? 1u : 0u;
        const uint32_t eb = ent ? lw_byte(lw, ni) : 0u;
        nat[0] = nat_areq(P.d, s, dst, ct, pli, plt, ent, eb & 15u, eb >> 4, nib(W.c[Lo::W_CI], s));
    }
}

__device__ __forceinline__ uint32_t nat_lookup(const KParams &P, uint32_t nat) {
    return nat != NAT_NONE ? (uint32_t)P.t.nat2id[nat] : 0u;
}

// Evaluate the message lane (round r) -> at most one successor.
// BFV (the tla:420 variant): ob gets the lane's BecomeFollower successor (tla:190-229) -- a second
// candidate per message; with BFV false ob is not touched.
template <int N, int V, int MR, bool BFV = false>
__device__ __forceinline__ void eval_msg(const KParams &P, const Wave<N, V, MR> &W, int r, int lane,
                         Succ<N, V, MR> &o, Succ<N, V, MR> &ob, uint32_t &assert_key, uint32_t *ainf, uint32_t pid) {
    // pid: the id msg_nat looked up for this lane (the only one its action may send)
    using Lo = Layout<N, V>;
    o.key = KEY_NONE;
    o.nadd = 0;
    o.s = 0;
#pragma unroll
    for (int a = 0; a < Spec<N, V, MR>::NADD; a++) o.add[a] = 0;
    if (BFV) {
        ob.key = KEY_NONE;
        ob.nadd = 0;
        ob.s = 0;
        ob.self = false;
#pragma unroll
        for (int a = 0; a < Spec<N, V, MR>::NADD; a++) ob.add[a] = 0;
    }
    o.self = false;
    const uint32_t k = (uint32_t)(r * 64 + lane);
    if (k >= W.nm) return;
    const uint32_t m = W.inf[r];
    const uint32_t s = mi_dst(m), typ = mi_type(m), mt = mi_term(m), src = mi_src(m);
    const uint32_t ct = nib(W.c[Lo::W_CT], s), role = nib(W.c[Lo::W_ROLE], s);
#pragma unroll
    for (int w = 0; w < Lo::NW; w++) o.c[w] = W.c[w];
    o.s = s;
    o.lw = W.lds[Lo::W_LOG + s];
    o.mirow = W.lds[Lo::W_MI + s];
    o.nirow = W.lds[Lo::W_NI + s];
    if (BFV) {
        // FollowerUpdateTerm (tla:191-197: votedFor, role kept), CandidateToFollower (tla:200-212),
        // LeaderToFollower (tla:215-223): role[s] picks one; msgs unchanged
        const bool up = mt > ct, step = mt == ct && typ == AREQ && role == CAN;
        if (up || step) {
#pragma unroll
            for (int w = 0; w < Lo::NW; w++) ob.c[w] = W.c[w];
            ob.s = s;
            ob.lw = o.lw;
            ob.mirow = o.mirow;
            ob.nirow = o.nirow;
            if (up) ob.c[Lo::W_CT] = setnib(ob.c[Lo::W_CT], s, mt);
            if (role != FOL) {
                ob.c[Lo::W_ROLE] = setnib(ob.c[Lo::W_ROLE], s, FOL);
                if (up) ob.c[Lo::W_VF] = setnib(ob.c[Lo::W_VF], s, VF_NONE);
            }
            ob.key = slot_key(s, BF, k);
        }
    }
    if (mt > ct) {  // UpdateTerm, first disjunct (tla:178-182)
        o.c[Lo::W_ROLE] = setnib(o.c[Lo::W_ROLE], s, FOL);
        o.c[Lo::W_CT] = setnib(o.c[Lo::W_CT], s, mt);
        o.c[Lo::W_VF] = setnib(o.c[Lo::W_VF], s, VF_NONE);
        o.key = slot_key(s, UT, k);
        return;
    }
    if (mt != ct) return;
    if (typ == AREQ && role != FOL) {  // UpdateTerm, second disjunct (tla:183-188)
        if (role == LEA) { assert_key = slot_key(s, UT, 0); return; }  // Assert(role[s] # Leader) tla:185
        o.c[Lo::W_ROLE] = setnib(o.c[Lo::W_ROLE], s, FOL);
        o.key = slot_key(s, UT, k);
        return;
    }
    const uint32_t ll = nib(W.c[Lo::W_LL], s);
    const uint32_t lw = W.lds[Lo::W_LOG + s];
    if (typ == VREQ && role == FOL) {  // ResponseVote tla:132-155
        const uint32_t vf = nib(W.c[Lo::W_VF], s);
        if (!(vf == VF_NONE || vf == src)) return;
        const uint32_t llt = lw_term(lw, ll), mlli = mi_x1(m), mllt = mi_x2(m);
        if (!(mllt > llt || (mllt == llt && mlli >= ll))) return;
        const uint32_t g = pid;  // nat2id[nat_vresp(s, src, mt)]
        if (in_msgs(W.bm, g)) return;
        o.c[Lo::W_VF] = setnib(o.c[Lo::W_VF], s, src);
        o.add[0] = g; o.nadd = 1;
        if (ainf) ainf[0] = minfo(VRESP, s, src, mt, 0, 0, 0, 0, 0, 0);
        o.key = slot_key(s, RV, k);
        return;
    }
    if (typ == AREQ && role == FOL) {  // FollowerAcceptEntry / FollowerRejectEntry tla:275-321
        const uint32_t pli = mi_x1(m), plt = mi_x2(m), lc = mi_x3(m), ent = mi_ent(m);
        const bool match = pli <= ll && plt == lw_term(lw, pli);  // LogMatch tla:271-273
        if (match) {
            const uint32_t nl = pli + ent;
            const bool append_new = nl > ll;
            const uint32_t eb = mi_et(m) | (mi_ev(m) << 4);
            const bool truncated = nl <= ll && ent && lw_byte(lw, nl) != eb;
            const uint32_t mn = (lc < nl || (P.quirks & 2u)) ? lc : nl;  // (RaftCommitPastLog: no Min)
            const uint32_t ci = nib(W.c[Lo::W_CI], s);
            const uint32_t nci = ci > mn ? ci : mn;
            const uint32_t resp = pid;  // nat2id[nat_aresp(s, src, mt, pli + ent, TRUE)]
            o.c[Lo::W_CI] = setnib(o.c[Lo::W_CI], s, nci);
            if (truncated || append_new) {
                // newLog == SubSeq(logs[s], 1, prevLogIndex) \o entries   (tla:291)
                uint32_t keep = pli >= 2 ? (pli - 1) * 8 : 0;  // bytes of indices 2..pli
                uint32_t nlw = keep >= 32 ? lw : (lw & ((1u << keep) - 1u));
                if (ent) nlw |= eb << (8 * (nl - 2));
#pragma unroll
                for (int q = 0; q < N; q++) o.c[Lo::W_LOG + q] = ((uint32_t)q == s) ? nlw : o.c[Lo::W_LOG + q];
                o.lw = nlw;
                o.c[Lo::W_LL] = setnib(o.c[Lo::W_LL], s, nl);
            }
            const bool has = in_msgs(W.bm, resp);
            if (!has) {
                o.add[0] = resp; o.nadd = 1;
                if (ainf) ainf[0] = minfo(ARESP, s, src, mt, pli + ent, 1, 0, 0, 0, 0);
            }
            o.self = has && !(truncated || append_new) && nci == ci;  // (the parent itself)
            o.key = slot_key(s, FAE, k);
        } else {
            const uint32_t resp = pid;  // nat2id[nat_aresp(s, src, mt, pli, FALSE)]
            if (in_msgs(W.bm, resp)) return;
            o.add[0] = resp; o.nadd = 1;
            if (ainf) ainf[0] = minfo(ARESP, s, src, mt, pli, 0, 0, 0, 0, 0);
            o.key = slot_key(s, FRE, k);
        }
        return;
    }
    if (typ == ARESP && role == LEA) {  // HandleAppendResp tla:374-396
        const uint32_t pend = W.c[Lo::W_PEND];
        const uint32_t pb = s * N + src;
        if (!((pend >> pb) & 1u)) return;
        const uint32_t pli = mi_x1(m);
        const uint32_t mirow = W.lds[Lo::W_MI + s], nirow = W.lds[Lo::W_NI + s];
        const uint32_t mi = nib(mirow, src), ni = nib(nirow, src);
        uint32_t nmi = mirow, nni = nirow;
        if (mi_x2(m)) {
            if (!(mi < pli)) return;
            nmi = setnib(mirow, src, pli);
            nni = setnib(nirow, src, pli + 1);
        } else {
            if (!(pli + 1 == ni)) return;
            if (!(pli > mi)) return;
            nni = setnib(nirow, src, pli);
        }
#pragma unroll
        for (int q = 0; q < N; q++) {
            o.c[Lo::W_MI + q] = ((uint32_t)q == s) ? nmi : o.c[Lo::W_MI + q];
            o.c[Lo::W_NI + q] = ((uint32_t)q == s) ? nni : o.c[Lo::W_NI + q];
        }
        o.mirow = nmi;
        o.nirow = nni;
        o.c[Lo::W_PEND] = pend & ~(1u << pb);
        o.key = slot_key(s, HAR, k);
        return;
    }
}

// Evaluate the non-message slot owned by this lane (last round).
template <int N, int V, int MR>
__device__ __forceinline__ void eval_slot(const KParams &P, const Wave<N, V, MR> &W, int lane,
                          Succ<N, V, MR> &o, uint32_t *ainf, const uint32_t (&sid)[N - 1]) {
    // sid: the ids slot_nats looked up for this lane
    using Lo = Layout<N, V>;
    using S = Spec<N, V, MR>;
    o.key = KEY_NONE;
    o.nadd = 0;
    o.s = 0;
    o.self = false;
#pragma unroll
    for (int a = 0; a < S::NADD; a++) o.add[a] = 0;
    if (lane >= N * S::SLOTS_PER_SERVER) return;
    const uint32_t s = (uint32_t)lane / S::SLOTS_PER_SERVER, t = (uint32_t)lane % S::SLOTS_PER_SERVER;
    const uint32_t role = nib(W.c[Lo::W_ROLE], s), ct = nib(W.c[Lo::W_CT], s), ll = nib(W.c[Lo::W_LL], s);
    const uint32_t ci = nib(W.c[Lo::W_CI], s);
    const uint32_t lw = W.lds[Lo::W_LOG + s];
    const uint32_t misc = W.c[Lo::W_MISC];
#pragma unroll
    for (int w = 0; w < Lo::NW; w++) o.c[w] = W.c[w];
    o.s = s;
    o.lw = lw;
    o.mirow = W.lds[Lo::W_MI + s];
    o.nirow = W.lds[Lo::W_NI + s];
    if (t == 0) {  // BecomeCandidate tla:107-130
        const uint32_t ec = misc & 15u;
        if (!((int)ec < P.E)) return;
        if (!(role == FOL || role == CAN)) return;
        const uint32_t term = ct + 1, llt = lw_term(lw, ll);
        o.c[Lo::W_CT] = setnib(o.c[Lo::W_CT], s, term);
        o.c[Lo::W_ROLE] = setnib(o.c[Lo::W_ROLE], s, CAN);
        o.c[Lo::W_VF] = setnib(o.c[Lo::W_VF], s, s);
        o.c[Lo::W_MISC] = (misc & ~15u) | (ec + 1);
        uint32_t na = 0;
#pragma unroll
        for (int p = 0; p < N; p++) {
            if ((uint32_t)p == s) continue;
            // sid[p < s ? p : p - 1] = nat2id[nat_vreq(s, p, term, ll, llt)] (selects: no runtime index)
            const int ix = p < (int)s ? p : p - 1;
            uint32_t id = 0;
#pragma unroll
            for (int i = 0; i < N - 1; i++) id = i == ix ? sid[i] : id;
            if (!in_msgs(W.bm, id)) {
#pragma unroll
                for (int a = 0; a < S::NADD; a++) o.add[a] = ((uint32_t)a == na) ? id : o.add[a];
                if (ainf) ainf[na] = minfo(VREQ, s, (uint32_t)p, term, ll, llt, 0, 0, 0, 0);
                na++;
            }
        }
        o.nadd = na;
        o.key = slot_key(s, BC, 0);
        return;
    }
    if (t == 1) {  // BecomeLeader tla:157-173
        if (role != CAN) return;
        const uint32_t vp = W.lds[Lo::NW + s];
        if (!(vp + 1 >= ((P.quirks & 1u) ? 1u : (uint32_t)(N / 2 + 1)))) return;  // (RaftSplitBrain: quorum 1)
        uint32_t mirow = 0, nirow = 0;
#pragma unroll
        for (int u = 0; u < N; u++) {
            mirow = setnib(mirow, u, (uint32_t)u != s ? 1u : ll);
            nirow = setnib(nirow, u, ll + 1);
        }
#pragma unroll
        for (int q = 0; q < N; q++) {
            o.c[Lo::W_MI + q] = ((uint32_t)q == s) ? mirow : o.c[Lo::W_MI + q];
            o.c[Lo::W_NI + q] = ((uint32_t)q == s) ? nirow : o.c[Lo::W_NI + q];
        }
        o.mirow = mirow;
        o.nirow = nirow;
        o.c[Lo::W_PEND] = W.c[Lo::W_PEND] & ~(((1u << N) - 1u) << (s * N));
        o.c[Lo::W_ROLE] = setnib(o.c[Lo::W_ROLE], s, LEA);
        o.key = slot_key(s, BL, 0);
        return;
    }
    if (t < 2 + (uint32_t)V) {  // ClientReq tla:233-240, witness v
        const uint32_t v = t - 2;
        if (role != LEA) return;
        if ((misc >> (8 + v)) & 1u) return;  // valSent[v] # None
        o.c[Lo::W_MISC] = misc | (1u << (8 + v));
        const uint32_t nlw = lw | ((ct | (v << 4)) << (8 * (ll + 1 - 2)));
        const uint32_t mirow = setnib(W.lds[Lo::W_MI + s], s, ll + 1);
#pragma unroll
        for (int q = 0; q < N; q++) {
            o.c[Lo::W_LOG + q] = ((uint32_t)q == s) ? nlw : o.c[Lo::W_LOG + q];
            o.c[Lo::W_MI + q] = ((uint32_t)q == s) ? mirow : o.c[Lo::W_MI + q];
        }
        o.lw = nlw;
        o.mirow = mirow;
        o.c[Lo::W_LL] = setnib(o.c[Lo::W_LL], s, ll + 1);
        o.key = slot_key(s, CR, v);
        return;
    }
    if (t < 2 + (uint32_t)V + (N - 1)) {  // LeaderAppendEntry tla:242-269, witness dst
        const uint32_t q = t - 2 - V;
        const uint32_t dst = q < s ? q : q + 1;
        if (role != LEA) return;
        const uint32_t ni = nib(W.lds[Lo::W_NI + s], dst);
        if (!(ni <= ll + 1)) return;
        const uint32_t pb = s * N + dst;
        if ((W.c[Lo::W_PEND] >> pb) & 1u) return;
        const uint32_t pli = ni - 1, plt = lw_term(lw, pli);
        const uint32_t ent = ni <= ll ? 1u : 0u;
        const uint32_t eb = ent ? lw_byte(lw, ni) : 0u;
        const uint32_t id = sid[0];  // nat2id[nat_areq(s, dst, ct, pli, plt, ent, eb, ci)]
        if (in_msgs(W.bm, id)) return;  // m \notin msgs
        o.c[Lo::W_PEND] = W.c[Lo::W_PEND] | (1u << pb);
        o.add[0] = id;
        o.nadd = 1;
        if (ainf) ainf[0] = minfo(AREQ, s, dst, ct, pli, plt, ci, ent, eb & 15u, eb >> 4);
        o.key = slot_key(s, LAE, dst);
        return;
    }
    if (t == 2 + (uint32_t)V + (N - 1)) {  // LeaderCanCommit tla:398-407
        if (role != LEA) return;
        const uint32_t thr = P.seeded ? (uint32_t)N : (uint32_t)(N / 2 + 1);
        const uint32_t med = median_row<N>(W.lds[Lo::W_MI + s], thr);
        if (!(med > ci)) return;
        o.c[Lo::W_CI] = setnib(o.c[Lo::W_CI], s, med);
        o.key = slot_key(s, LCC, 0);
        return;
    }
    {  // Restart tla:409-414
        const uint32_t rc = (misc >> 4) & 15u;
        if (role != LEA || !((int)rc < P.R)) return;
        o.c[Lo::W_ROLE] = setnib(o.c[Lo::W_ROLE], s, FOL);
        o.c[Lo::W_MISC] = (misc & ~0xF0u) | ((rc + 1) << 4);
        o.key = slot_key(s, RS, 0);
    }
}

// Read a packed core (wave-uniform) at ring position `start` and decode it to the nibble layout.
template <int N, int V>
__device__ __forceinline__ void load_core(const uint32_t *ring, uint64_t start, uint64_t rcap, int lane, uint32_t *c,
                                          uint32_t *packed) {
    constexpr int CCW = Codec<N, V>::CCW;
    const uint32_t mine = lane < CCW ? ring_word(ring, start, (uint32_t)lane, rcap) : 0u;
#pragma unroll
    for (int k = 0; k < CCW; k++) packed[k] = rdlane(mine, k);
    decode_core<N, V>(packed, c);
}

// Load a state record into the wave: uniform core (+ an LDS copy), per-lane message ids and info
// words, the per-(src,dst) message hash sums.
// The whole record in one round trip: lane k holds record word k (and 64 + k); the core is read
// across lanes, each lane's message ids are shuffled to it by load_parent -- no second dependent
// load for the ids (words past the record's end are read but never used).  k_expand issues this
// for its next parent while it works on the current one.
template <int MR, int RECW_MAX>
__device__ __forceinline__ void fetch_record(const KParams &P, uint64_t start, int lane, uint32_t &rw0, uint32_t &rw1) {
    rw0 = lane < RECW_MAX ? ring_word(P.front, start, (uint32_t)lane, P.rcap) : 0u;
    rw1 = (MR > 1 && 64 + lane < RECW_MAX) ? ring_word(P.front, start, 64u + (uint32_t)lane, P.rcap) : 0u;
}

// load_parent on a record already fetched (fetch_record)
template <int N, int V, int MR, bool SUMS>
__device__ __forceinline__ void load_parent_words(const KParams &P, uint64_t start, uint32_t rw0, uint32_t rw1, int lane,
                                                  Wave<N, V, MR> &W, uint64_t *M0, uint64_t *M1, uint32_t *pcore) {
    using Lo = Layout<N, V>;
    using S = Spec<N, V, MR>;
    uint32_t packed[S::CCW];
#pragma unroll
    for (int k = 0; k < S::CCW; k++) packed[k] = rdlane(rw0, k);
    decode_core<N, V>(packed, W.c);
    if (lane == 0) {  // uniform values: one lane writes the LDS copy (no runtime-indexed register array)
#pragma unroll
        for (int w = 0; w < Lo::NW; w++) pcore[w] = W.c[w];
    }
    W.lds = pcore;
    W.nm = (W.c[Lo::W_MISC] >> 16) & 0xFFu;
    W.idw = ring_wrap(start + S::CCW, P.rcap);
    if (SUMS && lane < N * N) { M0[lane] = 0; M1[lane] = 0; }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MR; r++) {
        const uint32_t k = (uint32_t)(r * 64 + lane);
        const uint32_t wi = (uint32_t)S::CCW + (k >> 1);  // record word holding id k
        const uint32_t a = __shfl(rw0, (int)(wi & 63u), 64);
        const uint32_t b = MR > 1 ? __shfl(rw1, (int)(wi & 63u), 64) : 0u;
        const uint32_t word = wi < 64u ? a : b;
        uint32_t id = 0xFFFFu, inf = 0;
        if (k < W.nm) {
            id = (word >> ((k & 1u) * 16u)) & 0xFFFFu;
            inf = P.t.info[id];
            if (SUMS) {
                const ulonglong2 g = P.t.gmsg[id];
                const uint32_t pr = mi_src(inf) * N + mi_dst(inf);
                atomicAdd((unsigned long long *)&M0[pr], (unsigned long long)g.x);
                atomicAdd((unsigned long long *)&M1[pr], (unsigned long long)g.y);
            }
        }
        W.id[r] = id;
        W.inf[r] = inf;
    }
#pragma unroll
    for (int s = 0; s < N; s++) {
        const uint32_t ct = nib(W.c[Lo::W_CT], s);
        uint32_t cnt = 0;
#pragma unroll
        for (int r = 0; r < MR; r++) {
            const uint32_t m = W.inf[r];
            const bool hit = (uint32_t)(r * 64 + lane) < W.nm && mi_type(m) == VRESP && mi_dst(m) == (uint32_t)s &&
                             mi_term(m) == ct;
            cnt += (uint32_t)__popcll(__ballot(hit));
        }
        if (lane == 0) pcore[Lo::NW + s] = cnt;
    }
    __syncthreads();
}

// The message-table words of a fetched record (info word + hash pair per message), issued ahead of
// use: k_expand loads them for its next parent while it hashes the current one, which takes the
// table round trip off the start of every parent.
template <int MR>
struct MsgPre {
    uint32_t id[MR], inf[MR];
    ulonglong2 g[MR];
};

template <int N, int V, int MR>
__device__ __forceinline__ void fetch_msgs(const KParams &P, uint32_t rw0, uint32_t rw1, int lane, MsgPre<MR> &pm) {
    using Lo = Layout<N, V>;
    using S = Spec<N, V, MR>;
    uint32_t packed[S::CCW], c[Lo::NW];
#pragma unroll
    for (int k = 0; k < S::CCW; k++) packed[k] = rdlane(rw0, k);
    decode_core<N, V>(packed, c);
    const uint32_t nm = (c[Lo::W_MISC] >> 16) & 0xFFu;
#pragma unroll
    for (int r = 0; r < MR; r++) {
        const uint32_t k = (uint32_t)(r * 64 + lane);
        const uint32_t wi = (uint32_t)S::CCW + (k >> 1);
        const uint32_t a = __shfl(rw0, (int)(wi & 63u), 64);
        const uint32_t b = MR > 1 ? __shfl(rw1, (int)(wi & 63u), 64) : 0u;
        const uint32_t word = wi < 64u ? a : b;
        uint32_t id = 0xFFFFu, inf = 0;
        ulonglong2 g = make_ulonglong2(0ull, 0ull);
        if (k < nm) {
            id = (word >> ((k & 1u) * 16u)) & 0xFFFFu;
            inf = P.t.info[id];
            g = P.t.gmsg[id];
        }
        pm.id[r] = id;
        pm.inf[r] = inf;
        pm.g[r] = g;
    }
}

// load_parent_words with the message-table words already fetched (fetch_msgs)
template <int N, int V, int MR>
__device__ __forceinline__ void load_parent_pre(const KParams &P, uint64_t start, uint32_t rw0, int lane,
                                                Wave<N, V, MR> &W, uint64_t *M0, uint64_t *M1, uint32_t *pcore,
                                                const MsgPre<MR> &pm) {
    using Lo = Layout<N, V>;
    using S = Spec<N, V, MR>;
    uint32_t packed[S::CCW];
#pragma unroll
    for (int k = 0; k < S::CCW; k++) packed[k] = rdlane(rw0, k);
    decode_core<N, V>(packed, W.c);
    if (lane == 0) {
#pragma unroll
        for (int w = 0; w < Lo::NW; w++) pcore[w] = W.c[w];
    }
    W.lds = pcore;
    W.nm = (W.c[Lo::W_MISC] >> 16) & 0xFFu;
    W.idw = ring_wrap(start + S::CCW, P.rcap);
    if (lane < N * N) { M0[lane] = 0; M1[lane] = 0; }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MR; r++) {
        const uint32_t k = (uint32_t)(r * 64 + lane);
        if (k < W.nm) {
            const uint32_t pr = mi_src(pm.inf[r]) * N + mi_dst(pm.inf[r]);
            atomicAdd((unsigned long long *)&M0[pr], (unsigned long long)pm.g[r].x);
            atomicAdd((unsigned long long *)&M1[pr], (unsigned long long)pm.g[r].y);
        }
        W.id[r] = pm.id[r];
        W.inf[r] = pm.inf[r];
    }
#pragma unroll
    for (int s = 0; s < N; s++) {
        const uint32_t ct = nib(W.c[Lo::W_CT], s);
        uint32_t cnt = 0;
#pragma unroll
        for (int r = 0; r < MR; r++) {
            const uint32_t m = W.inf[r];
            const bool hit = (uint32_t)(r * 64 + lane) < W.nm && mi_type(m) == VRESP && mi_dst(m) == (uint32_t)s &&
                             mi_term(m) == ct;
            cnt += (uint32_t)__popcll(__ballot(hit));
        }
        if (lane == 0) pcore[Lo::NW + s] = cnt;
    }
    __syncthreads();
}

template <int N, int V, int MR, bool SUMS>
__device__ __forceinline__ void load_parent(const KParams &P, uint64_t start, int lane, Wave<N, V, MR> &W, uint64_t *M0,
                                            uint64_t *M1, uint32_t *pcore) {
    using S = Spec<N, V, MR>;
    uint32_t rw0, rw1;
    fetch_record<MR, S::RECW_MAX>(P, start, lane, rw0, rw1);
    load_parent_words<N, V, MR, SUMS>(P, start, rw0, rw1, lane, W, M0, M1, pcore);
}

// hash row of the acting server: parent sums + the messages this successor adds
template <int N, int V, int MR>
__device__ __forceinline__ void succ_row_at(uint32_t s, uint32_t nadd, const uint64_t *M0, const uint64_t *M1,
                                            const uint32_t *ainf, uint64_t *row0, uint64_t *row1) {
#pragma unroll
    for (int j = 0; j < N; j++) { row0[j] = M0[s * N + j]; row1[j] = M1[s * N + j]; }
#pragma unroll
    for (int a = 0; a < Spec<N, V, MR>::NADD; a++) {
        if ((uint32_t)a >= nadd) break;
        // the added message's hash from its info word, built where it was generated: no
        // dependent table loads after the id lookup
        const uint32_t inf = ainf[a];
        const uint32_t dst = mi_dst(inf);
        const MsgHash g = msg_hash(inf);
#pragma unroll
        for (int j = 0; j < N; j++) {
            row0[j] += ((uint32_t)j == dst) ? g.x : 0ull;
            row1[j] += ((uint32_t)j == dst) ? g.y : 0ull;
        }
    }
}

// Merge the parent's sorted ids (per lane: id[r] = id r*64+lane, 0xFFFF past nm) with a
// successor's added ids into a record's id list at ring position `idw` (whole wave).
template <int N, int V, int MR>
__device__ __forceinline__ void write_ids(uint32_t *ring, uint64_t idw, uint64_t rcap, const uint32_t *id, uint32_t nm,
                                          const uint32_t *add, uint32_t nadd, int lane) {
    using S = Spec<N, V, MR>;
#pragma unroll
    for (int r = 0; r < MR; r++) {
        const uint32_t k = (uint32_t)(r * 64 + lane);
        if (k < nm) {
            uint32_t pos = k;
#pragma unroll
            for (int a = 0; a < S::NADD; a++) pos += ((uint32_t)a < nadd && add[a] < id[r]) ? 1u : 0u;
            ring_put_id(ring, idw, pos, rcap, id[r]);
        }
    }
#pragma unroll
    for (int a = 0; a < S::NADD; a++) {
        if ((uint32_t)a >= nadd) break;
        uint32_t less = 0;
#pragma unroll
        for (int r = 0; r < MR; r++)
            less += (uint32_t)__popcll(__ballot((uint32_t)(r * 64 + lane) < nm && id[r] < add[a]));
#pragma unroll
        for (int b = 0; b < S::NADD; b++) less += ((uint32_t)b < nadd && add[b] < add[a]) ? 1u : 0u;
        if (lane == 0) ring_put_id(ring, idw, less, rcap, add[a]);
    }
    if (lane == 0 && ((nm + nadd) & 1u)) ring_put_id(ring, idw, nm + nadd, rcap, 0u);  // pad half-word
}

// Write the successor held by lane t (round r) as a fixed-stride record at rec_out (whole wave).
template <int N, int V, int MR>
__device__ __forceinline__ void write_record(const Wave<N, V, MR> &W, const Succ<N, V, MR> &o, int t, int lane, uint32_t *rec_out) {
    using Lo = Layout<N, V>;
    using S = Spec<N, V, MR>;
    const uint32_t nadd = rdlane(o.nadd, t);
    uint32_t add[S::NADD];
#pragma unroll
    for (int a = 0; a < S::NADD; a++) add[a] = rdlane(o.add[a], t);
    uint32_t c[Lo::NW], packed[S::CCW];
#pragma unroll
    for (int w = 0; w < Lo::NW; w++) c[w] = rdlane(o.c[w], t);
    c[Lo::W_MISC] = (c[Lo::W_MISC] & ~0xFF0000u) | ((W.nm + nadd) << 16);
    encode_core<N, V>(c, packed);
    if (lane < S::CCW) rec_out[lane] = sel<S::CCW>(packed, lane);
    write_ids<N, V, MR>(rec_out, S::CCW, ~0ull, W.id, W.nm, add, nadd, lane);
}

// ---- seen set -----------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t t_index(const ulonglong2 f, uint64_t mask) {
    return (f.y ^ (f.y >> 29) ^ (f.x >> 23)) & mask;
}

// The compact table is bucketed: TB = 8 slots of 8 B per 64-B bucket, a fingerprint x in the first bucket
// from its home (linear over buckets) that had a free slot when it was inserted -- a probe reads one
// bucket in one round trip (four 16-B loads issued together) where single-slot linear probing took a
// dependent load per slot of the run.  Slots are only ever filled, so a bucket with a free slot ends a
// probe: a fingerprint inserted earlier would have found that slot (or one before it) free.
constexpr uint64_t TB = 8;
// Home bucket: multiply-shift of a remixed word (any bucket count).  The remix matters: y is a minimum
// over Permutations(Servers), so its high bits are far from uniform (the smallest of 6 -- or 120 --
// hashes), and multiply-shift reads the high bits.
__device__ __forceinline__ uint64_t t_home_c(const ulonglong2 f, uint64_t nbk) {
    uint64_t z = (f.y ^ (f.x >> 17)) * 0x9e3779b97f4a7c15ull;
    z ^= z >> 29;
    return __umul64hi(z, nbk);
}

// the eight slots of bucket b, loaded together
__device__ __forceinline__ void bucket_load(const unsigned long long *Tc, uint64_t b, unsigned long long e[TB]) {
    const ulonglong2 *p = reinterpret_cast<const ulonglong2 *>(Tc + b * TB);
    const ulonglong2 a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
    e[0] = a0.x; e[1] = a0.y; e[2] = a1.x; e[3] = a1.y; e[4] = a2.x; e[5] = a2.y; e[6] = a3.x; e[7] = a3.y;
}

__device__ __forceinline__ bool seen_contains(const Seen &S, ulonglong2 f) {
    if (S.Tc) {
        const uint64_t nbk = S.cap / TB;
        uint64_t b = t_home_c(f, nbk);
        for (;;) {
            unsigned long long e[TB];
            bucket_load(S.Tc, b, e);
            bool hit = false, free_ = false;
#pragma unroll
            for (uint64_t k = 0; k < TB; k++) {
                hit |= e[k] == f.x;
                free_ |= e[k] == 0ull;
            }
            if (hit) return true;
            if (free_) return false;
            b = (b + 1 == nbk) ? 0 : b + 1;
        }
    }
    uint64_t h = t_index(f, S.mask);
    for (;;) {
        const ulonglong2 e = S.T[h];
        // both words now: one 16-B load per probe (left alone, the compiler loads y only once x
        // has matched -- a second dependent round trip on every hit and on every collision)
        asm volatile("" ::"v"(e.x), "v"(e.y));
        if (e.x == 0ull) return false;
        if (e.x == f.x && e.y == f.y) return true;
        h = (h + 1) & S.mask;
    }
}

// keys inserted are never already present (winners are new, rehash moves distinct keys)
__device__ __forceinline__ void seen_insert(const Seen &S, ulonglong2 f) {
    if (S.Tc) {
        const uint64_t nbk = S.cap / TB;
        uint64_t b = t_home_c(f, nbk);
        for (;;) {
            unsigned long long e[TB];
            bucket_load(S.Tc, b, e);
            // the bucket's free slots in order; a slot another insert took first fails its CAS
            for (uint64_t k = 0; k < TB; k++)
                if (e[k] == 0ull && atomicCAS(&S.Tc[b * TB + k], 0ull, (unsigned long long)f.x) == 0ull) return;
            b = (b + 1 == nbk) ? 0 : b + 1;
        }
    }
    uint64_t h = t_index(f, S.mask);
    for (;;) {
        unsigned long long prev = atomicCAS((unsigned long long *)&S.T[h].x, 0ull, (unsigned long long)f.x);
        if (prev == 0ull) { S.T[h].y = f.y; return; }
        h = (h + 1) & S.mask;
    }
}

__device__ __forceinline__ uint64_t l_index(const ulonglong2 f, uint64_t mask) {
    return (f.x ^ (f.x >> 31) ^ (f.y >> 7)) & mask;
}
// sharded run: owner(fp) = high bits of fp.y mod W -- independent of the seen-set and election index bits
__device__ __forceinline__ uint32_t fp_owner(const ulonglong2 f, uint32_t W) {
    return (uint32_t)((f.y >> 40) % W);
}

// ---- in-launch election (fused single-GPU level) -------------------------------------------
// The first successor in TLC order (smallest slot q) per new fingerprint wins.  Election slot g
// holds the fingerprint in E[g].x / .y -- both words carry the chunk's 16-bit tag in their low bits,
// so slots of earlier chunks read as free and the table is never cleared (the host clears it
// once every 65535 epochs) -- and the election word E[g].k = elect_key(epoch, smallest q, its e), in the
// same 32-B sector.
// The word of a newer epoch is smaller than any older one (and than the all-ones initial value),
// so every candidate just takes the minimum.  All accesses are agent-scope atomics on the slot's
// own words: a claimer CASes x then stores y; a candidate that finds x equal but y not yet
// tagged retries the same slot on its next iteration (never spinning in place, so a claimer
// in the same wave always gets to its store).
__device__ __forceinline__ uint32_t elect_tag(uint32_t epoch) { return epoch % 0xFFFFu + 1u; }
// e = the record words a winner adds beyond CCW + floor(|parent msgs| / 2): ceil((nadd + (nm & 1)) / 2)
__device__ __forceinline__ unsigned long long elect_key(uint32_t epoch, uint64_t q, uint32_t e) {
    return ((unsigned long long)(0xFFFFFFFFu - epoch) << 32) | ((unsigned long long)(uint32_t)q << 2) | e;
}
__device__ __forceinline__ uint32_t elect_q(unsigned long long w) { return (uint32_t)w >> 2; }

// The candidate that becomes a slot's minimum adds one winner (and its e extra words) to its
// parent's packed count wacc = winners | extra << 12, and takes the displaced candidate's (the old
// minimum the atomic returns) off its parent: once the launch is done, wacc per parent is exact
// (the packed sum of adds and subtracts is exact mod 2^32 whatever their order).
template <int MAXS>
__device__ __forceinline__ uint32_t elect_slot(ESlot *E, uint32_t *wacc, uint64_t mask,
                                               uint32_t epoch, const ulonglong2 f, uint64_t q, uint32_t e, uint64_t g,
                                               unsigned long long v) {
    // g = l_index(f, mask) and v = its x word, loaded by the caller together with the seen-set probe
    const unsigned long long tag = elect_tag(epoch);
    const unsigned long long xk = (f.x & ~0xFFFFull) | tag, yk = (f.y & ~0xFFFFull) | tag;
    for (;;) {
        unsigned long long *px = &E[g].x, *py = &E[g].y;
        if ((v & 0xFFFFull) != tag) {
            const unsigned long long prev = atomicCAS(px, v, xk);
            if (prev == v) {
#ifdef RMC_RACE_PROBE
                if ((q & 7u) == 0u) race_delay(2);  // x claimed, y not yet visible
#endif
                __hip_atomic_store(py, yk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            v = prev;
            if ((v & 0xFFFFull) != tag) continue;
        }
        if (v == xk) {
            const unsigned long long y = __hip_atomic_load(py, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((y & 0xFFFFull) != tag) {  // the claimer's y is not visible yet: this slot again
                v = __hip_atomic_load(px, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                continue;
            }
            if (y == yk) break;
        }
        g = (g + 1) & mask;
        v = __hip_atomic_load(&E[g].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const unsigned long long mine = elect_key(epoch, q, e);
    const unsigned long long old = atomicMin(&E[g].k, mine);
    if (old > mine) {
        atomicAdd(&wacc[q / MAXS], 1u + (e << 12));
        if ((old >> 32) == (mine >> 32)) atomicSub(&wacc[elect_q(old) / MAXS], 1u + ((uint32_t)(old & 3u) << 12));
    }
    return (uint32_t)g;
}

// Staging of one successor: the acting server's row and the words an action may change
// (tla:107-414: every action assigns only votedFor[s], currentTerm[s], role[s], commitIndex[s],
// logs[s], matchIndex[s], nextIndex[s], pendingResponse, the aux counters and msgs):
//   w0 = votedFor[s] | currentTerm[s] << 4 | role[s] << 8 | commitIndex[s] << 12 | Len(logs[s]) << 16 | s << 20
//   w1 = logs[s] word  w2 = matchIndex[s] row  w3 = nextIndex[s] row  w4 = pendingResponse  w5 = misc (|msgs| set)
//   w6 = key | nadd << 16  w7 = add0 | add1 << 16  [w8 = add2 | add3 << 16]
template <int N, int V, int MR>
__device__ __forceinline__ void stage_succ(const Succ<N, V, MR> &o, uint32_t nm, uint4 *dst) {
    using Lo = Layout<N, V>;
    using S = Spec<N, V, MR>;
    const uint32_t s = o.s;
    const uint32_t w0 = nib(o.c[Lo::W_VF], s) | (nib(o.c[Lo::W_CT], s) << 4) | (nib(o.c[Lo::W_ROLE], s) << 8) |
                        (nib(o.c[Lo::W_CI], s) << 12) | (nib(o.c[Lo::W_LL], s) << 16) | (s << 20);
    const uint32_t w5 = (o.c[Lo::W_MISC] & ~0xFF0000u) | ((nm + o.nadd) << 16);
    uint32_t a01, a23;
    succ_adds(o, &a01, &a23);
    dst[0] = make_uint4(w0, o.lw, o.mirow, o.nirow);
    dst[1] = make_uint4(o.c[Lo::W_PEND], w5, o.key | (o.nadd << 16), a01);
    if (S::SW4 > 2) dst[2] = make_uint4(a23, 0u, 0u, 0u);
}

// parent nibble core pc + staged row -> the successor's nibble core c
template <int N, int V>
__device__ __forceinline__ void unstage_core(const uint32_t *pc, const uint4 a, const uint4 b, uint32_t *c) {
    using Lo = Layout<N, V>;
#pragma unroll
    for (int w = 0; w < Lo::NW; w++) c[w] = pc[w];
    const uint32_t s = a.x >> 20;
    c[Lo::W_VF] = setnib(c[Lo::W_VF], s, a.x & 15u);
    c[Lo::W_CT] = setnib(c[Lo::W_CT], s, (a.x >> 4) & 15u);
    c[Lo::W_ROLE] = setnib(c[Lo::W_ROLE], s, (a.x >> 8) & 15u);
    c[Lo::W_CI] = setnib(c[Lo::W_CI], s, (a.x >> 12) & 15u);
    c[Lo::W_LL] = setnib(c[Lo::W_LL], s, (a.x >> 16) & 15u);
#pragma unroll
    for (int q = 0; q < N; q++) {
        c[Lo::W_LOG + q] = ((uint32_t)q == s) ? a.y : c[Lo::W_LOG + q];
        c[Lo::W_MI + q] = ((uint32_t)q == s) ? a.z : c[Lo::W_MI + q];
        c[Lo::W_NI + q] = ((uint32_t)q == s) ? a.w : c[Lo::W_NI + q];
    }
    c[Lo::W_PEND] = b.x;
    c[Lo::W_MISC] = b.y;
}

// Words of a split chunk's hash context per parent (M_SPLIT -> k_hash_probe): the packed core
// (padded to 16 B), then per ordered server pair (t, j), t != j, its message-hash sums
// {M_0 lo, hi, M_1 lo, hi}.
template <int N, int V>
constexpr int ctx_words() { return ((Codec<N, V>::CCW + 3) / 4) * 4 + 4 * N * (N - 1); }
constexpr int pair_index(int N, int t, int j) { return t * (N - 1) + (j < t ? j : j - 1); }

// one family's half of msg_hash (rmc_spec.h)
__device__ __forceinline__ uint64_t msg_hash_half(uint32_t info, int f) {
    const uint64_t body = (uint64_t)info & ~0xFCull;
    return f ? mix64(body * 0xc2b2ae3d27d4eb4fULL + (SEED_MSG + 0x632be59bd9b4e019ULL))
             : mix64(body * 0x9e3779b97f4a7c15ULL + SEED_MSG);
}

// A staged successor's fingerprint (rmc_spec.h): its content matrix rebuilt from the parent's decoded
// core pc, the parent's message-hash sums per server pair (mp(pi) = {M_0, M_1} of pair pi) and the
// staged row (sa, sb, sc: the acting server's row and the added messages), then the coset minimum
// (ai(a, id): the info word of added message a, id its message id)
template <int N, int V, int MR, class FM, class FA>
__device__ __forceinline__ ulonglong2 staged_fp(const KParams &P, const uint32_t *pc, FM mp, FA ai, const uint4 sa,
                                                const uint4 sb, const uint4 sc, const uint64_t (*sK)[N * N]) {
    using S = Spec<N, V, MR>;
    using Lo = Layout<N, V>;
    uint32_t c[Lo::NW];
    unstage_core<N, V>(pc, sa, sb, c);
    const uint32_t sv = sa.x >> 20, nadd = sb.z >> 16;
    // the added messages' hashes toward each destination (all from the acting server)
    uint64_t ad0[N], ad1[N];
#pragma unroll
    for (int j = 0; j < N; j++) { ad0[j] = 0; ad1[j] = 0; }
    const uint32_t aid[4] = {sb.w & 0xFFFFu, sb.w >> 16, sc.x & 0xFFFFu, sc.x >> 16};
#pragma unroll
    for (int a = 0; a < S::NADD; a++) {
        if ((uint32_t)a >= nadd) break;
        const uint32_t inf = ai(a, aid[a]);
        const uint64_t g0 = msg_hash_half(inf, 0), g1 = msg_hash_half(inf, 1);  // (= the table's gmsg)
        const uint32_t d = mi_dst(inf);
#pragma unroll
        for (int j = 0; j < N; j++) {
            ad0[j] += (uint32_t)j == d ? g0 : 0ull;
            ad1[j] += (uint32_t)j == d ? g1 : 0ull;
        }
    }
    // the successor's content matrix and its servers' signatures
    uint64_t C0[N * N], C1[N * N], sig[N];
#pragma unroll
    for (int t = 0; t < N; t++) {
        sig[t] = 0;
#pragma unroll
        for (int j = 0; j < N; j++) {
            uint64_t m0 = 0, m1 = 0;
            if (t != j) {
                const ulonglong2 m = mp(pair_index(N, t, j));
                m0 = m.x + ((uint32_t)t == sv ? ad0[j] : 0ull);
                m1 = m.y + ((uint32_t)t == sv ? ad1[j] : 0ull);
            }
            C0[t * N + j] = content<N>(0, t, j, c, c[Lo::W_LOG + t], c[Lo::W_MI + t], c[Lo::W_NI + t], m0);
            C1[t * N + j] = content<N>(1, t, j, c, c[Lo::W_LOG + t], c[Lo::W_MI + t], c[Lo::W_NI + t], m1);
            sig[t] += C1[t * N + j];
        }
    }
    const uint32_t rk = P.t.np > 1 ? coset_ranks<N>(sig) : coset_ident<N>(), K = coset_size<N>(rk);
    ulonglong2 best = make_ulonglong2(~0ull, ~0ull);
    for (uint32_t k = 0; k < K; k++) {
        const ulonglong2 h = hash_at<N>(
            coset_img<N>(rk, k), [&](int f, int a, int b) { return f ? C1[a * N + b] : C0[a * N + b]; },
            [&](int f, uint32_t a, uint32_t b) { return sK[f][a * N + b]; });
        if (lex_less(h, best)) best = h;
    }
    return make_ulonglong2(best.x | 1ull, best.y);
}

// The fused election of a new fingerprint (the seen set is read-only in the launch): its slot q's
// verdict LS_SEEN, or the election slot it bid in.  e: the record words a winner adds (elect_key)
template <int MX>
__device__ __forceinline__ uint32_t probe_elect(const KParams &P, const ulonglong2 f, uint64_t q, uint32_t e,
                                                uint64_t Lmask) {
    // the election slot's first word goes out with the seen-set probe: one round trip fewer
    const uint64_t g = l_index(f, Lmask);
    const unsigned long long v0 = __hip_atomic_load(&P.ET[g].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return seen_contains(P.seen, f) ? LS_SEEN : elect_slot<MX>(P.ET, P.wacc, Lmask, P.epoch, f, q, e, g, v0);
}

template <int N, int MR, int MODE, bool BFV>
constexpr int expand_waves() {
    return (N <= 3 && MR == 1 && !BFV) ? RMC_N3_WAVES : ((BFV && N >= 4) ? 1 : RMC_WIDE_WAVES);
}

// BFV: the BecomeFollower variant (tla:420) -- MR more candidates (one per message lane) and MR * 64
// more successor slots per parent (MX)
template <int N, int V, int MR, int MODE, bool BFV = false>
__global__ __launch_bounds__(64, (expand_waves<N, MR, MODE, BFV>())) void k_expand(KParams P) {
    using S = Spec<N, V, MR>;
    using Lo = Layout<N, V>;
    constexpr int MX = S::MAXS + (BFV ? S::MCAP : 0);   // successor slots per parent
    constexpr int NC = MR + 1 + (BFV ? MR : 0);         // candidates per lane: messages, slot, BecomeFollower
    constexpr int HX = MX;                              // per-successor hash inputs, by TLC rank
    constexpr int HB = N <= 3 ? 32 : 64;                // successors hashed per batch
    constexpr int FH = 64 / HB;                         // lanes per batch successor: one per half when 2
    __shared__ uint64_t M0[N * N], M1[N * N];           // the parent's message-hash sums per (src, dst)
    __shared__ uint32_t pcore[Lo::NW + N];
    __shared__ uint64_t sK[2][N * N];        // position constants K_f[a][b]
    __shared__ uint64_t pC[2][N * N];        // the parent's content matrix C_f[t][j]
    __shared__ uint64_t psig[N];             // ... and its servers' signatures
    // every successor's row inputs at its TLC rank: own word; matchIndex row | votedFor << 20;
    // nextIndex row; where its added messages' info words are (sAinf); acting server; |added|
    __shared__ uint64_t sUg[HX];
    __shared__ uint32_t sW1[HX], sW2[HX];
    __shared__ uint16_t sCa[HX];
    __shared__ uint8_t sS[HX], sNa[HX];
    // per batch successor: its acting row's contents, tie ranks, first task, running minimum;
    // per task lane: its partial minimum and successor
    __shared__ uint64_t sC[2][HB * N];
    __shared__ uint32_t sRk[HB], sKoff[HB], sTl[64];
    __shared__ ulonglong2 sBest[HB], sPart[64];
    __shared__ uint32_t sAinf[(MR + 1) * 64 * S::NADD];  // info words of the messages each candidate adds
    extern __shared__ uint32_t sBM[];                    // bitmap of the parent's message ids (P.t.bmw words)
    if (MODE == M_FUSED && !level_args(P)) return;
    // device loop: the levels committed so far go to the host as this level starts (the write to
    // host memory completes in the shadow of the expansion; see finish_level)
    if (MODE == M_FUSED && P.hloop && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(&P.hloop->done, P.done_levels, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // device-loop grids are sized on a bound of the level: blocks past it leave before the LDS setup
    if (MODE == M_FUSED && P.p_begin + blockIdx.x >= P.p_end) return;
    const int lane = threadIdx.x;
    if (lane < 2 * N * N) {
        const int f = lane / (N * N), a = (lane / N) % N, b = lane % N;
        sK[f][a * N + b] = P.t.seeds[f * SEEDS_PER_F + a * MAXN + b];
    }
    PHASE_DECL
    // software pipeline over the block's parents: the next parent's record offset goes out at the
    // top of an iteration and its record once this one's is consumed, so a block's second and later
    // parents start with their record in registers (offsets two parents ahead: an offset has a
    // whole iteration to land before its record is fetched).  One-round kernels also fetch the next
    // parent's message-table words once this one's actions are evaluated (the two-round n >= 4
    // expansion is at its register limit already).
    uint64_t p = P.p_begin + blockIdx.x, nstart = 0, nnstart = 0;
    uint32_t nrw0 = 0, nrw1 = 0;
    uint32_t route_self = 0;  // sharded round: the wave's self-loops (sum[SUM_SELF], one atomic per wave)
    constexpr bool PREM = MR == 1;
    MsgPre<MR> pm;
    if (p < P.p_end) {
        nstart = rec_start<S::RECW_MAX>(P, p);
        fetch_record<MR, S::RECW_MAX>(P, nstart, lane, nrw0, nrw1);
        if constexpr (PREM) fetch_msgs<N, V, MR>(P, nrw0, nrw1, lane, pm);
        if (p + gridDim.x < P.p_end) nnstart = rec_start<S::RECW_MAX>(P, p + gridDim.x);
    }
    for (; p < P.p_end; p += gridDim.x) {
        const uint64_t start = nstart;
        const bool more = p + gridDim.x < P.p_end;
        nstart = nnstart;
        if (p + 2ull * gridDim.x < P.p_end) nnstart = rec_start<S::RECW_MAX>(P, p + 2ull * gridDim.x);
        Wave<N, V, MR> W;
        if constexpr (PREM) {
            load_parent_pre<N, V, MR>(P, start, nrw0, lane, W, M0, M1, pcore, pm);
            if (more) fetch_record<MR, S::RECW_MAX>(P, nstart, lane, nrw0, nrw1);
        } else {
            load_parent_words<N, V, MR, true>(P, start, nrw0, nrw1, lane, W, M0, M1, pcore);
        }
        msg_bitmap<N, V, MR>(sBM, P.t.bmw, W, lane);
        W.bm = sBM;
        PHASE(0);
        Succ<N, V, MR> cand[NC];
        uint32_t akey = KEY_NONE;
        // the lane index, opaque to the compiler here: what the evaluation derives from it is
        // recomputed per parent instead of hoisted out of the loop (and spilled)
        int ln = lane;
        asm volatile("" : "+v"(ln));
        // every id lookup of the actions in one round trip (msg_nat / slot_nats)
        uint32_t mid[MR], sid[N - 1];
        {
            uint32_t snat[N - 1];
            slot_nats<N, V, MR>(P, W, ln, snat);
#pragma unroll
            for (int r = 0; r < MR; r++) mid[r] = nat_lookup(P, msg_nat<N, V, MR>(P, W, r, ln));
#pragma unroll
            for (int i = 0; i < N - 1; i++) sid[i] = nat_lookup(P, snat[i]);
        }
#pragma unroll
        for (int r = 0; r < MR; r++)
            eval_msg<N, V, MR, BFV>(P, W, r, ln, cand[r], cand[BFV ? MR + 1 + r : r], akey,
                                    &sAinf[(r * 64 + ln) * S::NADD], mid[r]);
        eval_slot<N, V, MR>(P, W, ln, cand[MR], &sAinf[(MR * 64 + ln) * S::NADD], sid);
        if constexpr (PREM) {
            if (more) fetch_msgs<N, V, MR>(P, nrw0, nrw1, lane, pm);
        } else {
            if (more) fetch_record<MR, S::RECW_MAX>(P, nstart, lane, nrw0, nrw1);
        }
        PHASE(1);
        // rank of every enabled successor in TLC order
        uint64_t en[NC];
        uint32_t total = 0;
#pragma unroll
        for (int r = 0; r < NC; r++) {
            en[r] = __ballot(cand[r].key != KEY_NONE);
            total += (uint32_t)__popcll(en[r]);
        }
        uint32_t rank[NC];
#pragma unroll
        for (int r = 0; r < NC; r++) rank[r] = 0;
#pragma unroll
        for (int q = 0; q < NC; q++) {
            for (uint64_t m = en[q]; m; m &= m - 1) {
                const int t = __ffsll((unsigned long long)m) - 1;
                const uint32_t kt = rdlane(cand[q].key, t);
#pragma unroll
                for (int r = 0; r < NC; r++) rank[r] += kt < cand[r].key ? 1u : 0u;
            }
        }
        // a sharded round routes every successor's fingerprint to its owner, self-loops (the parent itself,
        // FollowerAcceptEntry changing nothing) too; they are counted for the level statistics only
        if (MODE == M_FUSED) {
#pragma unroll
            for (int r = 0; r < NC; r++) route_self += (uint32_t)__popcll(__ballot(cand[r].key != KEY_NONE && cand[r].self));
        }
        const uint64_t pl = p - P.p_begin;  // chunk-local parent index
        uint64_t am = 0;
        {
            bool ovf = false;
#pragma unroll
            for (int r = 0; r < NC; r++) ovf |= cand[r].key != KEY_NONE && W.nm + cand[r].nadd > (uint32_t)S::MCAP;
            if (__ballot(ovf) && lane == 0) atomicOr(&P.flags[0], 1u);
            am = __ballot(akey != KEY_NONE);
            if (am) {
                uint32_t best = KEY_NONE;
                for (uint64_t m = am; m; m &= m - 1) {
                    const uint32_t k = rdlane(akey, __ffsll((unsigned long long)m) - 1);
                    best = k < best ? k : best;
                }
                if (lane == 0) atomicMin(&P.err[ERR_ASSERT], (((unsigned long long)p << 16) | best) << 8);
            }
        }
        if (MODE != M_SINGLE && lane == 0) {
            P.cnt[pl] = total;
            P.pnm[pl] = W.nm;
            if (total == 0 && !am && P.check_deadlock) atomicMin(&P.err[ERR_DEADLOCK], ((unsigned long long)p << 16) << 8);
        }
        PHASE(2);
        if (MODE != M_SINGLE) {
            // stage every enabled successor at its slot q: the acting row and the added message ids
            // -- commit rebuilds the state from the parent's core and merges the ids
#pragma unroll
            for (int r = 0; r < NC; r++) {
                if (cand[r].key == KEY_NONE) continue;
                const uint64_t q = pl * (uint64_t)MX + rank[r];
                stage_succ<N, V, MR>(cand[r], W.nm, P.score + q * (uint64_t)S::SW4);
            }
        }
        PHASE(3);
        // ---- fingerprints (rmc_spec.h): content matrix, signature coset, minimum -----------------
        // (a) the parent's content matrix, a lane per (half, row, column)
        if (lane < 2 * N * N) {
            const int f = lane / (N * N), t = (lane / N) % N, j = lane % N;
            pC[f][t * N + j] = content<N>(f, (uint32_t)t, (uint32_t)j, W.c, pcore[Lo::W_LOG + t], pcore[Lo::W_MI + t],
                                          pcore[Lo::W_NI + t], f ? M1[t * N + j] : M0[t * N + j]);
        }
        // (b) every enabled successor's row inputs at its TLC rank
#pragma unroll
        for (int r = 0; r < NC; r++) {
            if (cand[r].key == KEY_NONE) continue;
            const Succ<N, V, MR> &o = cand[r];
            const uint32_t g = rank[r];
            const uint32_t vfs = nib(o.c[Lo::W_VF], o.s);
            sUg[g] = own_word<N>(o.c[Lo::W_VF], o.c[Lo::W_CT], o.c[Lo::W_ROLE], o.c[Lo::W_CI], o.c[Lo::W_LL], o.lw,
                                 o.mirow, o.nirow, o.s);
            sW1[g] = o.mirow | (vfs << 20);  // rows of N <= 5 nibbles
            sW2[g] = o.nirow;
            // (BecomeFollower candidates, r > MR, add no messages: their info words are never read)
            sCa[g] = (uint16_t)(((r <= MR ? r : 0) * 64 + lane) * S::NADD);
            sS[g] = (uint8_t)o.s;
            sNa[g] = (uint8_t)o.nadd;
        }
        __syncthreads();
        if (lane < N) {
            uint64_t sg = 0;
#pragma unroll
            for (int j = 0; j < N; j++) sg += pC[1][lane * N + j];
            psig[lane] = sg;
        }
        PHASE(4);
        auto emit = [&](uint32_t lo, ulonglong2 best) {
            const ulonglong2 f = make_ulonglong2(best.x | 1ull, best.y);
            if (MODE == M_FUSED) {
                P.fp[pl * (uint64_t)MX + lo] = f;  // sharded round: the fingerprint's owner probes and elects
            } else {
                P.fp[lo] = f;
            }
        };
        // (c) per batch of HB successors (by TLC rank)
        for (uint32_t b0 = 0; b0 < total; b0 += (uint32_t)HB) {
            const uint32_t nb = total - b0 < (uint32_t)HB ? total - b0 : (uint32_t)HB;
            {  // (c1) the acting row's contents: lane (half, successor) when FH == 2, else both halves
                const uint32_t l = (uint32_t)lane % HB, g = b0 + l;
                if (l < nb) {
                    const uint32_t sv = sS[g], w1 = sW1[g], na = sNa[g];
                    const uint32_t mirow = w1 & 0xFFFFFu, vfs = w1 >> 20, nirow = sW2[g];
                    const uint64_t u = sUg[g];
                    const uint32_t *ai = &sAinf[sCa[g]];
#pragma unroll
                    for (int fi = 0; fi < 3 - FH; fi++) {
                        const int f = FH == 2 ? lane / HB : fi;
                        uint64_t row[N];
#pragma unroll
                        for (int j = 0; j < N; j++) row[j] = f ? M1[sv * N + j] : M0[sv * N + j];
#pragma unroll
                        for (int a = 0; a < S::NADD; a++) {
                            if ((uint32_t)a >= na) break;
                            const uint32_t inf = ai[a];
                            const uint32_t dst = mi_dst(inf);
                            const uint64_t h = msg_hash_half(inf, f);
#pragma unroll
                            for (int j = 0; j < N; j++) row[j] += ((uint32_t)j == dst) ? h : 0ull;
                        }
                        sC[f][l * N + sv] = cmix_own(u, f);
#pragma unroll
                        for (int j = 0; j < N; j++) {
                            if ((uint32_t)j == sv) continue;
                            const uint64_t sm = pair_small(mirow, nirow, vfs, (uint32_t)j);
                            sC[f][l * N + j] = cmix_pair(row[j] ^ (sm * (f ? PAIR_K1 : PAIR_K0)), f);
                        }
                    }
                }
            }
            __syncthreads();
            PHASE(4);
            if ((uint32_t)lane < nb) {  // (c2) signatures, tie ranks and coset size per successor
                const uint32_t l = (uint32_t)lane, sv = sS[b0 + l];
                uint64_t rs = 0;
#pragma unroll
                for (int j = 0; j < N; j++) rs += sC[1][l * N + j];
                uint64_t sig[N];
#pragma unroll
                for (int t = 0; t < N; t++) sig[t] = (uint32_t)t == sv ? rs : psig[t];
                const uint32_t rk = P.t.np > 1 ? coset_ranks<N>(sig) : coset_ident<N>();
                sRk[l] = rk;
                sKoff[l] = coset_size<N>(rk);
                sBest[l] = make_ulonglong2(~0ull, ~0ull);
            }
            __syncthreads();
            uint32_t ntask = 0;
            {
                const uint32_t l = (uint32_t)lane;
                uint32_t rt;
                const uint32_t ex = wave_excl_scan(l < nb ? sKoff[l] : 0u, lane, &rt);
                if (l < nb) sKoff[l] = ex;
                ntask = rt;
            }
            __syncthreads();
            PHASE(5);
            // (c3) one task per (successor, allowed permutation), 64 per round; a successor's tasks
            //      are consecutive, so the first lane of each run folds the run into its minimum
            for (uint32_t tb = 0; tb < ntask; tb += 64) {
                const uint32_t ti = tb + (uint32_t)lane;
                uint32_t l = 0xFFFFFFFFu;
                ulonglong2 h = make_ulonglong2(~0ull, ~0ull);
                if (ti < ntask) {
                    uint32_t a = 0, b = nb;  // sKoff[a] <= ti < sKoff[b]
                    while (b - a > 1) {
                        const uint32_t m = (a + b) >> 1;
                        if (sKoff[m] <= ti) a = m; else b = m;
                    }
                    l = a;
                    const uint32_t imgw = coset_img<N>(sRk[l], ti - sKoff[l]);
                    const uint32_t sv = sS[b0 + l];
                    // a row per iteration (not unrolled: the LDS operands of every row at once
                    // would spill); the acting row from the batch, the others from the parent
                    uint64_t h0 = 0, h1 = 0;
#pragma unroll 1
                    for (uint32_t t = 0; t < (uint32_t)N; t++) {
                        const uint32_t it = (imgw >> (3 * t)) & 7u;
                        const uint64_t *r0 = t == sv ? &sC[0][l * N] : &pC[0][t * N];
                        const uint64_t *r1 = t == sv ? &sC[1][l * N] : &pC[1][t * N];
#pragma unroll
                        for (int j = 0; j < N; j++) {
                            const uint32_t ij = (imgw >> (3 * j)) & 7u;
                            h0 += r0[j] * sK[0][it * N + ij];
                            h1 += r1[j] * sK[1][it * N + ij];
                        }
                    }
                    h = make_ulonglong2(h0, h1);
                }
                sPart[lane] = h;
                sTl[lane] = l;
                __syncthreads();
                if (ti < ntask && (lane == 0 || sTl[lane - 1] != l)) {
                    ulonglong2 best = sBest[l];
                    for (int j = lane; j < 64 && sTl[j] == l; j++)
                        if (lex_less(sPart[j], best)) best = sPart[j];
                    sBest[l] = best;
                }
                __syncthreads();
            }
            PHASE(6);
            if ((uint32_t)lane < nb) emit(b0 + (uint32_t)lane, sBest[lane]);
            __syncthreads();
            PHASE(7);
        }
        asm volatile("" ::"v"(nnstart));  // the offset two parents ahead is in by now: keep its load up top
        if (MODE == M_FUSED) continue;
        // SINGLE: every successor, in TLC order
#pragma unroll
        for (int r = 0; r < NC; r++) {
            const bool win = cand[r].key != KEY_NONE;
            const uint64_t out = rank[r];
            if (win) P.out_keys[out] = cand[r].key;
            for (uint64_t m = __ballot(win); m; m &= m - 1) {
                const int t = __ffsll((unsigned long long)m) - 1;
                const uint64_t ot = rdlane64(out, t);
                write_record<N, V, MR>(W, cand[r], t, lane, P.next + ot * (uint64_t)S::RECW_MAX);
            }
        }
        if (lane == 0) *P.out_count = total;
    }
    if (MODE == M_FUSED && P.route && lane == 0 && route_self) atomicAdd(&P.sum[SUM_SELF], (unsigned long long)route_self);
    PHASE_FLUSH;
}

// ---- split chunk expansion, a lane per (parent, item) -------------------------------------------
// k_expand<..., M_SPLIT> gives every parent a 64-lane wave: the wave decodes the parent's core on all
// 64 lanes, builds a bitmap of its message ids, then lane k evaluates message k's receive action and
// lanes 0 .. N * SLOTS_PER_SERVER - 1 the non-message slots -- about 26 + 24 busy lanes of 128 at
// Raft.cfg's depth, every message type's branch run one after another, and the TLC-order ranks by
// a loop over the enabled lanes.  Here a 256-thread block takes 64 consecutive parents at a time:
//   (a) their records -- consecutive in the frontier ring -- are copied into LDS in one coalesced
//       pass; a lane per parent decodes its core once into LDS and lists its *items*: one per
//       message (UpdateTerm tla:175, ResponseVote tla:132, FollowerAccept/RejectEntry tla:275/302,
//       HandleAppendResp tla:374 -- at most one is enabled per message; with the tla:420 variant also
//       BecomeFollower) and one per non-message slot the server's role can enable (a follower only
//       BecomeCandidate tla:107, a candidate also BecomeLeader tla:157, a leader ClientReq tla:233 per
//       value, LeaderAppendEntry tla:242 per peer, LeaderCanCommit tla:398 and Restart tla:409);
//   (b) a lane per message adds its hashes into the parent's per-pair sums (the hash context
//       k_hash_probe reads) and counts the votes BecomeLeader needs (tla:160-164), LDS atomics;
//   (c) the items of whole parents, up to 256 at a time, a lane each: the action on the acting
//       server's row only (every action of tla:107-414 changes only votedFor / currentTerm / role /
//       commitIndex / logs / matchIndex / nextIndex of its server s, pendingResponse, the aux
//       counters and msgs), `m \notin msgs` by a binary search of the parent's sorted ids in LDS;
//   (d) each enabled successor's rank in TLC order (slot keys increase in TLC order, Next tla:416-430)
//       from the parent's list of enabled keys, and its staged row at slot hoff[pl] + rank (a dense
//       split chunk: each round's parents take a range of the chunk's slots with one atomic) or
//       pl * MX + rank (fused levels, sharded rounds) -- the slots k_hash_probe and the commits read.
#ifndef RMC_ITEMS_PB
#define RMC_ITEMS_PB 64
#endif
constexpr int XB_PARENTS = RMC_ITEMS_PB;  // parents per batch (<= 64: a lane of wave 0 each)
// ... of a fused level: levels of a few thousand parents (configs[1]) need more blocks than 64-parent
// batches make to fill 256 CUs
#ifndef RMC_FUSED_PB
#define RMC_FUSED_PB 16
#endif
constexpr int XF_PARENTS = RMC_FUSED_PB;
#ifndef RMC_FUSED_CPB
#define RMC_FUSED_CPB RMC_FUSED_PB  // ... and per block of their commit
#endif
constexpr int XC_PARENTS = RMC_FUSED_CPB;
#ifndef RMC_FUSED_WAVES
#define RMC_FUSED_WAVES 4  // n <= 3: registers cut for 4 waves per SIMD, 4 blocks per CU (the compiler's choice: 3;
                           // n >= 4 would spill)
#endif
constexpr int XB_THREADS = 256;  // threads per block = items per evaluation round at most
#ifndef RMC_ITEMS_NT  // ... of the split expansion where a parent's items fit that many (else 256)
#define RMC_ITEMS_NT 256
#endif
template <int N, int V, int MR, bool FUSE>
constexpr int items_threads() {
    return (!FUSE && Spec<N, V, MR>::MCAP + N * Spec<N, V, MR>::SLOTS_PER_SERVER <= RMC_ITEMS_NT) ? RMC_ITEMS_NT : XB_THREADS;
}

// votedFor, currentTerm, role, commitIndex, Len(logs) of server s and s itself: staging word 0
__device__ __forceinline__ uint32_t row_w0(uint32_t vf, uint32_t ct, uint32_t role, uint32_t ci, uint32_t ll,
                                           uint32_t s) {
    return vf | (ct << 4) | (role << 8) | (ci << 12) | (ll << 16) | (s << 20);
}

// g \in msgs of a parent whose sorted ids are ids[0 .. nm) (LDS): branch-free lower bound (a two-step search --
// the first id of every block of eight, then the block's eight -- issues twice the LDS reads and measured slower)
template <int MCAP>
__device__ __forceinline__ bool ids_contain(const uint16_t *ids, uint32_t nm, uint32_t g) {
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t st = (uint32_t)MCAP; st; st >>= 1)
        if (pos + st <= nm && (uint32_t)ids[pos + st - 1] < g) pos += st;
    return pos < nm && (uint32_t)ids[pos] == g;
}

// one successor candidate of an item: the acting server's staged row (stage_succ's layout)
template <int NADD>
struct RowSucc {
    uint32_t w0, lw, mirow, nirow, pend, misc;
    uint32_t key;  // KEY_NONE: disabled
    uint32_t nadd;
    uint32_t add[NADD];
    uint32_t ainf[NADD];  // the added messages' info words (a fused level hashes them; dead code in a split chunk)
    bool self;     // the successor is the parent itself (FollowerAcceptEntry changing nothing)
};

template <int NADD>
__device__ __forceinline__ void row_stage(const RowSucc<NADD> &o, uint32_t nm, int sw4, uint4 *dst) {
    uint32_t a[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < NADD; k++) a[k] = o.add[k];
    const uint32_t misc = (o.misc & ~0xFF0000u) | ((nm + o.nadd) << 16);
    dst[0] = make_uint4(o.w0, o.lw, o.mirow, o.nirow);
    dst[1] = make_uint4(o.pend, misc, o.key | (o.nadd << 16), a[0] | (a[1] << 16));
    if (sw4 > 2) dst[2] = make_uint4(a[2] | (a[3] << 16), 0u, 0u, 0u);
}

// The message item k (info word m) of a parent whose nibble core is pc (LDS) -> at most one successor
// o (and with BFV the BecomeFollower one, ob).  The same guards and updates as eval_msg, on the row of
// s = m.dst; pid is the id of the one message the action may send (looked up before any branch).
template <int N, int V, int MR, bool BFV>
__device__ __forceinline__ void item_msg(const KParams &P, const uint32_t *pc, const uint16_t *ids, uint32_t nm,
                                         uint32_t k, uint32_t m, uint32_t pid, RowSucc<Spec<N, V, MR>::NADD> &o,
                                         RowSucc<Spec<N, V, MR>::NADD> &ob, uint32_t &akey) {
    using Lo = Layout<N, V>;
    using S = Spec<N, V, MR>;
    const uint32_t s = mi_dst(m), typ = mi_type(m), mt = mi_term(m), src = mi_src(m);
    uint32_t vf = nib(pc[Lo::W_VF], s), ct = nib(pc[Lo::W_CT], s), role = nib(pc[Lo::W_ROLE], s);
    uint32_t ci = nib(pc[Lo::W_CI], s), ll = nib(pc[Lo::W_LL], s);
    const uint32_t lw = pc[Lo::W_LOG + s], mirow = pc[Lo::W_MI + s], nirow = pc[Lo::W_NI + s];
    const uint32_t pend = pc[Lo::W_PEND], misc = pc[Lo::W_MISC];
    o.key = KEY_NONE;
    o.nadd = 0;
    o.self = false;
#pragma unroll
    for (int a = 0; a < S::NADD; a++) o.add[a] = 0;
    o.lw = lw; o.mirow = mirow; o.nirow = nirow; o.pend = pend; o.misc = misc;
    o.w0 = row_w0(vf, ct, role, ci, ll, s);
    if (BFV) {
        // FollowerUpdateTerm / CandidateToFollower / LeaderToFollower (tla:190-229); msgs unchanged
        ob = o;
        const bool up = mt > ct, step = mt == ct && typ == AREQ && role == CAN;
        if (up || step) {
            const uint32_t bct = up ? mt : ct, brole = role != FOL ? (uint32_t)FOL : role;
            const uint32_t bvf = (role != FOL && up) ? VF_NONE : vf;
            ob.w0 = row_w0(bvf, bct, brole, ci, ll, s);
            ob.key = slot_key(s, BF, k);
        }
    }
    if (mt > ct) {  // UpdateTerm, first disjunct (tla:178-182)
        o.w0 = row_w0(VF_NONE, mt, FOL, ci, ll, s);
        o.key = slot_key(s, UT, k);
        return;
    }
    if (mt != ct) return;
    if (typ == AREQ && role != FOL) {  // UpdateTerm, second disjunct (tla:183-188)
        if (role == LEA) { akey = slot_key(s, UT, 0); return; }  // Assert(role[s] # Leader) tla:185
        o.w0 = row_w0(vf, ct, FOL, ci, ll, s);
        o.key = slot_key(s, UT, k);
        return;
    }
    if (typ == VREQ && role == FOL) {  // ResponseVote tla:132-155
        if (!(vf == VF_NONE || vf == src)) return;
        const uint32_t llt = lw_term(lw, ll), mlli = mi_x1(m), mllt = mi_x2(m);
        if (!(mllt > llt || (mllt == llt && mlli >= ll))) return;
        if (ids_contain<S::MCAP>(ids, nm, pid)) return;
        o.w0 = row_w0(src, ct, role, ci, ll, s);
        o.add[0] = pid; o.nadd = 1;
        o.ainf[0] = minfo(VRESP, s, src, mt, 0, 0, 0, 0, 0, 0);
        o.key = slot_key(s, RV, k);
        return;
    }
    if (typ == AREQ && role == FOL) {  // FollowerAcceptEntry / FollowerRejectEntry tla:275-321
        const uint32_t pli = mi_x1(m), plt = mi_x2(m), lc = mi_x3(m), ent = mi_ent(m);
        const bool match = pli <= ll && plt == lw_term(lw, pli);  // LogMatch tla:271-273
        if (match) {
            const uint32_t nl = pli + ent;
            const bool append_new = nl > ll;
            const uint32_t eb = mi_et(m) | (mi_ev(m) << 4);
            const bool truncated = nl <= ll && ent && lw_byte(lw, nl) != eb;
            const uint32_t mn = (lc < nl || (P.quirks & 2u)) ? lc : nl;  // (RaftCommitPastLog: no Min)
            const uint32_t nci = ci > mn ? ci : mn;
            uint32_t nll = ll;
            if (truncated || append_new) {
                // newLog == SubSeq(logs[s], 1, prevLogIndex) \o entries   (tla:291)
                const uint32_t keep = pli >= 2 ? (pli - 1) * 8 : 0;  // bytes of indices 2..pli
                uint32_t nlw = keep >= 32 ? lw : (lw & ((1u << keep) - 1u));
                if (ent) nlw |= eb << (8 * (nl - 2));
                o.lw = nlw;
                nll = nl;
            }
            o.w0 = row_w0(vf, ct, role, nci, nll, s);
            const bool has = ids_contain<S::MCAP>(ids, nm, pid);
            if (!has) { o.add[0] = pid; o.nadd = 1; }
            o.ainf[0] = minfo(ARESP, s, src, mt, pli + ent, 1, 0, 0, 0, 0);
            // (no new entry, no truncation, no commit, the response already sent: the parent itself)
            o.self = has && !(truncated || append_new) && nci == ci;
            o.key = slot_key(s, FAE, k);
        } else {
            if (ids_contain<S::MCAP>(ids, nm, pid)) return;
            o.add[0] = pid; o.nadd = 1;
            o.ainf[0] = minfo(ARESP, s, src, mt, pli, 0, 0, 0, 0, 0);
            o.key = slot_key(s, FRE, k);
        }
        return;
    }
    if (typ == ARESP && role == LEA) {  // HandleAppendResp tla:374-396
        const uint32_t pb = s * N + src;
        if (!((pend >> pb) & 1u)) return;
        const uint32_t pli = mi_x1(m);
        const uint32_t mi = nib(mirow, src), ni = nib(nirow, src);
        uint32_t nmi = mirow, nni = nirow;
        if (mi_x2(m)) {
            if (!(mi < pli)) return;
            nmi = setnib(mirow, src, pli);
            nni = setnib(nirow, src, pli + 1);
        } else {
            if (!(pli + 1 == ni)) return;
            if (!(pli > mi)) return;
            nni = setnib(nirow, src, pli);
        }
        o.mirow = nmi;
        o.nirow = nni;
        o.pend = pend & ~(1u << pb);
        o.key = slot_key(s, HAR, k);
    }
}

// the id of the one message a message item's action may send (ResponseVote's VoteResp, FollowerAccept /
// RejectEntry's AppendResp), or NAT_NONE -- msg_nat on the item's row
template <int N, int V>
__device__ __forceinline__ uint32_t item_msg_nat(const KParams &P, const uint32_t *pc, uint32_t m) {
    using Lo = Layout<N, V>;
    const uint32_t s = mi_dst(m), typ = mi_type(m), mt = mi_term(m), src = mi_src(m);
    if (mt != nib(pc[Lo::W_CT], s) || nib(pc[Lo::W_ROLE], s) != FOL) return NAT_NONE;
    if (typ == VREQ) return nat_vresp(P.d, s, src, mt);
    if (typ != AREQ) return NAT_NONE;
    const uint32_t ll = nib(pc[Lo::W_LL], s), lw = pc[Lo::W_LOG + s];
    const uint32_t pli = mi_x1(m), plt = mi_x2(m), ent = mi_ent(m);
    const bool match = pli <= ll && plt == lw_term(lw, pli);  // LogMatch tla:271-273
    return match ? nat_aresp(P.d, s, src, mt, pli + ent, 1) : nat_aresp(P.d, s, src, mt, pli, 0);
}

// The non-message slot t of server s (eval_slot's slots: 0 BecomeCandidate, 1 BecomeLeader, 2 .. 1 + V
// ClientReq, then LeaderAppendEntry per peer, LeaderCanCommit, Restart) -> at most one successor.
template <int N, int V, int MR>
__device__ __forceinline__ void item_slot(const KParams &P, const uint32_t *pc, const uint16_t *ids, uint32_t nm,
                                          uint32_t vp, uint32_t s, uint32_t t, RowSucc<Spec<N, V, MR>::NADD> &o) {
    using Lo = Layout<N, V>;
    using S = Spec<N, V, MR>;
    const uint32_t vf = nib(pc[Lo::W_VF], s), ct = nib(pc[Lo::W_CT], s), role = nib(pc[Lo::W_ROLE], s);
    const uint32_t ci = nib(pc[Lo::W_CI], s), ll = nib(pc[Lo::W_LL], s);
    const uint32_t lw = pc[Lo::W_LOG + s], mirow = pc[Lo::W_MI + s], nirow = pc[Lo::W_NI + s];
    const uint32_t pend = pc[Lo::W_PEND], misc = pc[Lo::W_MISC];
    o.key = KEY_NONE;
    o.nadd = 0;
    o.self = false;
#pragma unroll
    for (int a = 0; a < S::NADD; a++) o.add[a] = 0;
    o.lw = lw; o.mirow = mirow; o.nirow = nirow; o.pend = pend; o.misc = misc;
    o.w0 = row_w0(vf, ct, role, ci, ll, s);
    if (t == 0) {  // BecomeCandidate tla:107-130
        const uint32_t ec = misc & 15u;
        if (!((int)ec < P.E) || !(role == FOL || role == CAN)) return;
        const uint32_t term = ct + 1, llt = lw_term(lw, ll);
        uint32_t sid[N - 1];  // the VoteReqs to the N - 1 peers, looked up together
#pragma unroll
        for (int i = 0; i < N - 1; i++) {
            const uint32_t p = (uint32_t)i < s ? (uint32_t)i : (uint32_t)i + 1u;
            sid[i] = (uint32_t)P.t.nat2id[nat_vreq(P.d, s, p, term, ll, llt)];
        }
        uint32_t na = 0;
#pragma unroll
        for (int i = 0; i < N - 1; i++) {
            if (!ids_contain<S::MCAP>(ids, nm, sid[i])) {
                const uint32_t p = (uint32_t)i < s ? (uint32_t)i : (uint32_t)i + 1u;
                const uint32_t inf = minfo(VREQ, s, p, term, ll, llt, 0, 0, 0, 0);
#pragma unroll
                for (int a = 0; a < S::NADD; a++) {
                    o.add[a] = ((uint32_t)a == na) ? sid[i] : o.add[a];
                    o.ainf[a] = ((uint32_t)a == na) ? inf : o.ainf[a];
                }
                na++;
            }
        }
        o.nadd = na;
        o.w0 = row_w0(s, term, CAN, ci, ll, s);
        o.misc = (misc & ~15u) | (ec + 1);
        o.key = slot_key(s, BC, 0);
        return;
    }
    if (t == 1) {  // BecomeLeader tla:157-173
        if (role != CAN) return;
        if (!(vp + 1 >= ((P.quirks & 1u) ? 1u : (uint32_t)(N / 2 + 1)))) return;  // (RaftSplitBrain: quorum 1)
        uint32_t mr = 0, nr = 0;
#pragma unroll
        for (int u = 0; u < N; u++) {
            mr = setnib(mr, u, (uint32_t)u != s ? 1u : ll);
            nr = setnib(nr, u, ll + 1);
        }
        o.mirow = mr;
        o.nirow = nr;
        o.pend = pend & ~(((1u << N) - 1u) << (s * N));
        o.w0 = row_w0(vf, ct, LEA, ci, ll, s);
        o.key = slot_key(s, BL, 0);
        return;
    }
    if (role != LEA) return;
    if (t < 2 + (uint32_t)V) {  // ClientReq tla:233-240, witness v
        const uint32_t v = t - 2;
        if ((misc >> (8 + v)) & 1u) return;  // valSent[v] # None
        o.misc = misc | (1u << (8 + v));
        o.lw = lw | ((ct | (v << 4)) << (8 * (ll + 1 - 2)));
        o.mirow = setnib(mirow, s, ll + 1);
        o.w0 = row_w0(vf, ct, role, ci, ll + 1, s);
        o.key = slot_key(s, CR, v);
        return;
    }
    if (t < 2 + (uint32_t)V + (N - 1)) {  // LeaderAppendEntry tla:242-269, witness dst
        const uint32_t q = t - 2 - V;
        const uint32_t dst = q < s ? q : q + 1;
        const uint32_t ni = nib(nirow, dst);
        if (!(ni <= ll + 1)) return;
        const uint32_t pb = s * N + dst;
        if ((pend >> pb) & 1u) return;
        const uint32_t pli = ni - 1, plt = lw_term(lw, pli);
        const uint32_t ent = ni <= ll ? 1u : 0u;
        const uint32_t eb = ent ? lw_byte(lw, ni) : 0u;
        const uint32_t id = P.t.nat2id[nat_areq(P.d, s, dst, ct, pli, plt, ent, eb & 15u, eb >> 4, ci)];
        if (ids_contain<S::MCAP>(ids, nm, id)) return;  // m \notin msgs
        o.pend = pend | (1u << pb);
        o.add[0] = id;
        o.ainf[0] = minfo(AREQ, s, dst, ct, pli, plt, ci, ent, eb & 15u, eb >> 4);
        o.nadd = 1;
        o.key = slot_key(s, LAE, dst);
        return;
    }
    if (t == 2 + (uint32_t)V + (N - 1)) {  // LeaderCanCommit tla:398-407
        const uint32_t thr = P.seeded ? (uint32_t)N : (uint32_t)(N / 2 + 1);
        const uint32_t med = median_row<N>(mirow, thr);
        if (!(med > ci)) return;
        o.w0 = row_w0(vf, ct, role, med, ll, s);
        o.key = slot_key(s, LCC, 0);
        return;
    }
    {  // Restart tla:409-414
        const uint32_t rc = (misc >> 4) & 15u;
        if (!((int)rc < P.R)) return;
        o.w0 = row_w0(vf, ct, FOL, ci, ll, s);
        o.misc = (misc & ~0xF0u) | ((rc + 1) << 4);
        o.key = slot_key(s, RS, 0);
    }
}

// the non-message slots a server's role can enable: first slot and count, 4 bits each, per server
template <int N, int V>
__device__ __forceinline__ uint32_t slot_range(uint32_t role, uint32_t ec, uint32_t rc, int E, int R) {
    constexpr uint32_t SPS = 4 + V + (N - 1);
    if (role == LEA) return 2u | ((SPS - 2u - ((int)rc < R ? 0u : 1u)) << 4);  // ClientReq .. LeaderCanCommit (+ Restart)
    const uint32_t bc = (int)ec < E ? 1u : 0u;                              // BecomeCandidate while elections remain
    if (role == CAN) return (bc ? 0u : 1u) | ((bc + 1u) << 4);               // (+ BecomeLeader)
    return bc << 4;
}

#ifndef RMC_ITEMS_WAVES  // waves per SIMD the item-parallel expansion's registers are cut for (0: the compiler's)
#define RMC_ITEMS_WAVES 0
#endif
// Item classes: the action an item can take, from its message and its server's term and role alone
// (the first guards of eval_msg / eval_slot) -- a round's items are evaluated class by class, so the
// lanes of a wave take one action's branch, and messages no action can receive (an older term than
// their destination's, a VoteResp) are never items at all.
enum ItemClass : uint32_t {
    IC_UT = 0,  // m.term > currentTerm[s]: UpdateTerm's first disjunct (+ BecomeFollower)        tla:178-182
    IC_UT2,     // = term, AppendReq, s not a follower: UpdateTerm's second (Assert tla:185) (+ BF)  tla:183-188
    IC_RV,      // = term, VoteReq, s a follower: ResponseVote                                      tla:132-155
    IC_AE,      // = term, AppendReq, s a follower: FollowerAcceptEntry / FollowerRejectEntry       tla:275-321
    IC_HAR,     // = term, AppendResp, s a leader: HandleAppendResp                                 tla:374-396
    IC_BC, IC_BL, IC_CR, IC_LAE, IC_LCC, IC_RS,  // the non-message slots (eval_slot)
    IC_N,
    IC_DEAD = 0xFF
};
__device__ __forceinline__ uint32_t msg_class(uint32_t m, uint32_t ct, uint32_t role) {
    const uint32_t mt = mi_term(m), typ = mi_type(m);
    if (mt > ct) return IC_UT;
    if (mt < ct) return IC_DEAD;
    if (typ == AREQ) return role != FOL ? IC_UT2 : IC_AE;
    if (typ == VREQ) return role == FOL ? IC_RV : IC_DEAD;
    if (typ == ARESP) return role == LEA ? IC_HAR : IC_DEAD;
    return IC_DEAD;  // VoteResp: only counted (BecomeLeader)
}
template <int N, int V>
__device__ __forceinline__ uint32_t slot_class(uint32_t t) {
    return t == 0 ? IC_BC : t == 1 ? IC_BL : t < 2 + (uint32_t)V ? IC_CR : t < 2 + (uint32_t)V + (N - 1) ? IC_LAE
         : t == 2 + (uint32_t)V + (N - 1) ? IC_LCC : IC_RS;
}

// (the fused BecomeFollower kernel is not cut to RMC_FUSED_WAVES: at 4 waves per SIMD it spills 23 VGPRs, and with
// the message-parent notes that build gave wrong BecomeFollower n3 counts while the uncut one matches the oracle --
// profiles/r06_ab_message_parents.txt)
template <int N, int V, int MR, bool BFV, bool FUSE, int PB>
__global__ __launch_bounds__((items_threads<N, V, MR, FUSE>()), FUSE ? ((N <= 3 && !BFV) ? RMC_FUSED_WAVES : 0) : RMC_ITEMS_WAVES) void k_expand_items(KParams P) {
    using S = Spec<N, V, MR>;
    using Lo = Layout<N, V>;
    constexpr int NT = items_threads<N, V, MR, FUSE>();
    static_assert(PB >= 2 && PB <= 64 && (PB & (PB - 1)) == 0, "parents per batch: a power of two, a lane of wave 0 each");
    constexpr int CCW = S::CCW, RECW = S::RECW_MAX, NW = Lo::NW, NWP = (NW + 3) / 4 * 4;
    constexpr int MX = S::MAXS + (BFV ? S::MCAP : 0);
    constexpr int NCI = BFV ? 2 : 1;  // candidates of a message item
    constexpr int NPR = N * (N - 1);
    constexpr int CTXW = ctx_words<N, V>(), CC = ((CCW + 3) / 4) * 4;
    constexpr int RC = FUSE ? 1 : 4;  // record words per lane in flight in the batch's copy (a fused batch: one)
    static_assert(S::MCAP + N * S::SLOTS_PER_SERVER <= NT, "a parent's items fit one evaluation round");
    static_assert(S::MCAP <= 128 && PB <= 64, "item codes: parent << 8 | slot bit << 7 | message index or s << 4 | t");
    __shared__ uint32_t sRec[PB * RECW];           // the batch's records, as in the ring
    __shared__ uint32_t sCore[PB * NWP];           // their nibble cores
    __shared__ uint8_t sMI[PB * S::MCAP];          // per message of the batch: its class (15: none)
    __shared__ uint8_t sMJ[PB * S::MCAP];          // ... and its parent (the class lists' item codes)
    __shared__ uint32_t sInf[FUSE ? PB * S::MCAP : 1];  // fused level: ... and its info word (one round trip less)
    __shared__ uint32_t sVp[PB * N];               // per parent and server: VoteResps to it in its term (tla:160-164)
    __shared__ uint32_t sOff[PB];                  // record's first word in sRec
    __shared__ uint32_t sItm[PB + 1], sMsc[PB + 1];  // items / messages: exclusive scans over the batch
    __shared__ uint32_t sLive[PB];                 // per parent: messages some action may receive
    __shared__ unsigned long long sSlot[PB];       // slot_range per server, 8 bits each
    __shared__ uint32_t sCnt[PB], sAk[PB];         // enabled successors (self-loops apart), smallest Assert key
    __shared__ uint32_t sHo[FUSE ? 1 : PB];        // dense split chunk: each parent's first successor slot -- the
    __shared__ uint32_t sAlloc;                    // batch's successors packed from the start of its parents' sparse
                                                   // range (b0 * MX ..), each round's after the last (sAlloc used)
    __shared__ uint32_t sSelf[PB];                 // self-loops (P.hcnt: staged nowhere, never fingerprinted)
    __shared__ uint32_t sCc[IC_N];                 // the round's items per class
    // the batch's hash sums (until the hash context is written), then the rounds' item lists and keys
    // (a fused level keeps the sums to the end: its lanes fingerprint their successors themselves)
    constexpr int UM = FUSE ? 0 : 2 * PB * NPR * 8, UQ = IC_N * NT * 2 + NT * NCI * 2;
    __shared__ __attribute__((aligned(16))) unsigned char sU[UM > UQ ? UM : UQ];
    __shared__ unsigned long long sMh[FUSE ? 2 * PB * NPR : 1];
    __shared__ uint64_t sK[2][FUSE ? N * N : 1];   // fused level: position constants K_f[a][b]
    unsigned long long *sM0 = FUSE ? sMh : reinterpret_cast<unsigned long long *>(sU), *sM1 = sM0 + PB * NPR;
    uint16_t *sQ = reinterpret_cast<uint16_t *>(sU);   // [IC_N][NT] item codes by class
    uint16_t *sKey = sQ + IC_N * NT;                    // [NT * NCI] the round's enabled keys, per parent at its items' offset
    __shared__ uint32_t sSpan;
    __shared__ uint32_t sSelfN;                    // fused level: the block's self-loops (finish_level adds them up)
    __shared__ uint32_t sHfp;                      // sparse split chunk: the block's successors to fingerprint (SUM_HFP)
    const int tid = threadIdx.x;
    if (tid == 0) {
        sSelfN = 0u;
        sHfp = 0u;
    }
    if constexpr (FUSE) {
        // device loop: the level from the control block, the levels committed so far to the host as
        // this one starts (as k_expand<M_FUSED>); grids are sized on a bound of the level
        if (!level_args(P)) return;
        if (P.hloop && blockIdx.x == 0 && tid == 0)
            __hip_atomic_store(&P.hloop->done, P.done_levels, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (tid < 2 * N * N) {  // (read after the batch loop's first barrier)
            const int f = tid / (N * N), a = (tid / N) % N, b = tid % N;
            sK[f][a * N + b] = P.t.seeds[f * SEEDS_PER_F + a * MAXN + b];
        }
    }
    const uint64_t np = P.p_end - P.p_begin;
    PHASE_DECL
    for (uint64_t b0 = (uint64_t)blockIdx.x * PB; b0 < np; b0 += (uint64_t)gridDim.x * PB) {
        const uint32_t nb = (uint32_t)(np - b0 < (uint64_t)PB ? np - b0 : (uint64_t)PB);
        // (a) the batch's records: consecutive in the ring (every level is laid out in parent order)
        if (tid < 64) {  // wave 0: a lane per parent
            if (tid == 0) sAlloc = 0u;
            const uint64_t o = (uint32_t)tid < nb ? P.foff[P.p_begin + b0 + tid] : 0ull;
            const uint64_t first = rdlane64(o, 0);
            const uint64_t last = rdlane64(o, (int)nb - 1);
            if ((uint32_t)tid < nb) sOff[tid] = (uint32_t)(o - first);
            if (tid == 0) {
                uint64_t span = last - first + RECW;
                if (span > (uint64_t)PB * RECW) {  // not consecutive: never the case (see the commits)
                    atomicOr(&P.flags[0], 2u);
                    span = (uint64_t)PB * RECW;
                }
                sSpan = (uint32_t)span;
            }
        }
        __syncthreads();
        {
            const uint64_t f0 = P.foff[P.p_begin + b0];
            const uint64_t start = ring_wrap(P.fbase + f0, P.rcap);
            const uint32_t span = sSpan;
            // (RC words per lane in flight at once: the loads go out together, then the LDS stores)
            for (uint32_t w0 = (uint32_t)tid; w0 < span; w0 += RC * NT) {
                uint32_t v[RC];
#pragma unroll
                for (int k = 0; k < RC; k++)
                    if (w0 + k * NT < span) v[k] = ring_word(P.front, start, w0 + k * NT, P.rcap);
#pragma unroll
                for (int k = 0; k < RC; k++)
                    if (w0 + k * NT < span) sRec[w0 + k * NT] = v[k];
            }
        }
        __syncthreads();
        PHASE(0);
        // a lane per parent: core, slots, counters; the message scan in wave 0
        if (tid < 64) {
            uint32_t nmj = 0;
            if ((uint32_t)tid < nb) {
                const uint32_t *rec = sRec + sOff[tid];
                uint32_t pk[CCW], c[NW];
#pragma unroll
                for (int k = 0; k < CCW; k++) pk[k] = rec[k];
                decode_core<N, V>(pk, c);
                nmj = (c[Lo::W_MISC] >> 16) & 0xFFu;
                if (nmj > (uint32_t)S::MCAP) {  // never a real record (commits flag the overflow): a
                    // corrupted one stops the level with the msg_cap error instead of overrunning LDS
                    atomicOr(&P.flags[0], 1u);
                    nmj = S::MCAP;
                    c[Lo::W_MISC] = (c[Lo::W_MISC] & ~0xFF0000u) | (nmj << 16);
                }
#pragma unroll
                for (int w = 0; w < NW; w++) sCore[tid * NWP + w] = c[w];
                const uint32_t ec = c[Lo::W_MISC] & 15u, rc = (c[Lo::W_MISC] >> 4) & 15u;
                unsigned long long sl = 0;
#pragma unroll
                for (int s = 0; s < N; s++)
                    sl |= (unsigned long long)slot_range<N, V>(nib(c[Lo::W_ROLE], s), ec, rc, P.E, P.R) << (8 * s);
                sSlot[tid] = sl;
#pragma unroll
                for (int s = 0; s < N; s++) sVp[tid * N + s] = 0u;
#pragma unroll
                for (int k = 0; k < NPR; k++) { sM0[tid * NPR + k] = 0ull; sM1[tid * NPR + k] = 0ull; }
                sCnt[tid] = 0u;
                sSelf[tid] = 0u;
                sAk[tid] = KEY_NONE;
                sLive[tid] = 0u;
            }
            uint32_t tm;
            const uint32_t xm = wave_excl_scan(nmj, tid, &tm);
            if ((uint32_t)tid < nb) sMsc[tid] = xm;
            if (tid == 0) sMsc[nb] = tm;
            // each message's parent, for the message pass and the class lists (no search per message; round 6:
            // expansion -5.7 %, profiles/r06_ab_message_parents.txt)
            for (uint32_t k = 0; k < nmj; k++) sMJ[xm + k] = (uint8_t)tid;
        }
        __syncthreads();
        PHASE(1);
        // (b) a lane per message: hash sums per server pair, votes per server, its class
        const uint32_t tmsg = sMsc[nb];
        for (uint32_t m = (uint32_t)tid; m < tmsg; m += NT) {
            const uint32_t j = sMJ[m];  // its parent
            const uint32_t k = m - sMsc[j];
            const uint32_t id = reinterpret_cast<const uint16_t *>(sRec + sOff[j] + CCW)[k];
            const uint32_t inf = P.t.info[id];
            const ulonglong2 g = P.t.gmsg[id];
            const uint32_t src = mi_src(inf), dst = mi_dst(inf);
            const int pi = pair_index(N, (int)src, (int)dst);
            atomicAdd(&sM0[j * NPR + pi], (unsigned long long)g.x);
            atomicAdd(&sM1[j * NPR + pi], (unsigned long long)g.y);
            const uint32_t *pc = sCore + j * NWP;
            const uint32_t ct = nib(pc[Lo::W_CT], dst);
            if (mi_type(inf) == VRESP && mi_term(inf) == ct) atomicAdd(&sVp[j * N + dst], 1u);
            const uint32_t c = msg_class(inf, ct, nib(pc[Lo::W_ROLE], dst));
            sMI[m] = (uint8_t)(c == IC_DEAD ? 15u : c);
            if constexpr (FUSE) sInf[m] = inf;
            if (c != IC_DEAD) atomicAdd(&sLive[j], 1u);
        }
        __syncthreads();
        PHASE(2);
        // the batch's hash contexts (k_hash_probe): packed core padded to 16 B, then per server pair its
        // sums {M_0 lo, hi, M_1 lo, hi}; the batch's parents are consecutive, so one coalesced range
        for (uint32_t w = (uint32_t)tid; !FUSE && w < nb * (uint32_t)CTXW; w += NT) {
            const uint32_t j = w / CTXW, k = w % CTXW;
            uint32_t v = 0u;
            if (k < (uint32_t)CC) {
                v = k < (uint32_t)CCW ? sRec[sOff[j] + k] : 0u;
            } else {
                const uint32_t pi = (k - CC) >> 2, part = k & 3u;
                const unsigned long long mm = (part >> 1) ? sM1[j * NPR + pi] : sM0[j * NPR + pi];
                v = (part & 1u) ? (uint32_t)(mm >> 32) : (uint32_t)mm;
            }
            P.hctx[(b0 + j) * (uint64_t)CTXW + k] = v;
        }
        // items per parent: its live messages and its slots; their scan (wave 0)
        if (tid < 64) {
            uint32_t ni = 0;
            if ((uint32_t)tid < nb) {
                const unsigned long long sl = sSlot[tid];
                ni = sLive[tid];
#pragma unroll
                for (int u = 0; u < N; u++) ni += (uint32_t)(sl >> (8 * u + 4)) & 15u;
            }
            uint32_t ti;
            const uint32_t xi = wave_excl_scan(ni, tid, &ti);
            if ((uint32_t)tid < nb) sItm[tid] = xi;
            if (tid == 0) sItm[nb] = ti;
        }
        if (tid < IC_N) sCc[tid] = 0u;
        __syncthreads();  // (also: the hash sums are read; sQ / sKey may reuse their words)
        PHASE(3);
        // (c) + (d): rounds of whole parents, up to NT items each
        for (uint32_t a = 0; a < nb;) {
            const uint32_t ibase = sItm[a];
            uint32_t b = a;  // the last parent b with sItm[b] <= ibase + NT: parents a .. b - 1 fit
#pragma unroll
            for (uint32_t st = PB; st; st >>= 1) b = (b + st <= nb && sItm[b + st] <= ibase + NT) ? b + st : b;
            b = b > a ? b : a + 1;  // (a parent's items always fit a round: MCAP + N * SLOTS_PER_SERVER <= NT)
            const uint32_t nI = sItm[b] - ibase < (uint32_t)NT ? sItm[b] - ibase : (uint32_t)NT;
            // the round's items into their class lists: live messages (each one's parent noted with the message
            // scan: no search), then each parent's slots, a server's positions all taken before any is written so its
            // LDS atomics are in flight together (round 6: expansion -8 %, profiles/r06_ab_class_lists.txt); one LDS
            // atomic per item -- appending a wave's items per class with ballots and one atomic per class, or
            // finding the parent by a two-step search, measured slower (profiles/r06_ab_expansion.txt)
            for (uint32_t m = sMsc[a] + (uint32_t)tid; m < sMsc[b]; m += NT) {
                const uint32_t c = sMI[m];
                if (c == 15u) continue;
                const uint32_t j = sMJ[m];
                sQ[c * NT + atomicAdd(&sCc[c], 1u)] = (uint16_t)((j << 8) | (m - sMsc[j]));
            }
            for (uint32_t q = (uint32_t)tid; q < (b - a) * (uint32_t)N; q += NT) {  // a lane per (parent, server)
                const uint32_t j = a + q / N, u = q % N;
                const uint32_t rg = (uint32_t)(sSlot[j] >> (8 * u)) & 0xFFu, n = rg >> 4, t0 = rg & 15u;
                uint32_t pos[S::SLOTS_PER_SERVER];
#pragma unroll
                for (uint32_t r = 0; r < (uint32_t)S::SLOTS_PER_SERVER; r++)
                    if (r < n) pos[r] = atomicAdd(&sCc[slot_class<N, V>(t0 + r)], 1u);
#pragma unroll
                for (uint32_t r = 0; r < (uint32_t)S::SLOTS_PER_SERVER; r++)
                    if (r < n) sQ[slot_class<N, V>(t0 + r) * NT + pos[r]] = (uint16_t)((j << 8) | 0x80u | (u << 4) | (t0 + r));
            }
            __syncthreads();
            PHASE(7);
            RowSucc<S::NADD> o, ob;
            o.key = KEY_NONE;
            ob.key = KEY_NONE;
            uint32_t j = 0, nmj = 0;
            if ((uint32_t)tid < nI) {
                // this lane's item: class lists concatenated in class order
                uint32_t pre = 0, code = 0;
#pragma unroll
                for (uint32_t c = 0; c < IC_N; c++) {
                    const uint32_t n = sCc[c], t = (uint32_t)tid - pre;
                    if (t < n) code = sQ[c * NT + t];
                    pre += n;
                }
                j = code >> 8;
                const uint32_t *pc = sCore + j * NWP;
                const uint16_t *ids = reinterpret_cast<const uint16_t *>(sRec + sOff[j] + CCW);
                nmj = (pc[Lo::W_MISC] >> 16) & 0xFFu;
                uint32_t akey = KEY_NONE;
                if (!(code & 0x80u)) {
                    const uint32_t k = code & 0x7Fu;
                    const uint32_t inf = FUSE ? sInf[sMsc[j] + k] : P.t.info[ids[k]];
                    const uint32_t nat = item_msg_nat<N, V>(P, pc, inf);
                    const uint32_t pid = nat != NAT_NONE ? (uint32_t)P.t.nat2id[nat] : 0u;
                    item_msg<N, V, MR, BFV>(P, pc, ids, nmj, k, inf, pid, o, ob, akey);
                } else {
                    const uint32_t s = (code >> 4) & 7u, t = code & 15u;
                    item_slot<N, V, MR>(P, pc, ids, nmj, sVp[j * N + s], s, t, o);
                }
                if (akey != KEY_NONE) atomicMin(&sAk[j], akey);
                const uint32_t kb = (sItm[j] - ibase) * NCI;  // the parent's key list
                if (!FUSE && o.key != KEY_NONE && o.self && P.hcnt) atomicAdd(&sSelf[j], 1u);
                else if (o.key != KEY_NONE) sKey[kb + atomicAdd(&sCnt[j], 1u)] = (uint16_t)o.key;
                if (BFV && ob.key != KEY_NONE) sKey[kb + atomicAdd(&sCnt[j], 1u)] = (uint16_t)ob.key;
                if ((o.key != KEY_NONE && nmj + o.nadd > (uint32_t)S::MCAP)) atomicOr(&P.flags[0], 1u);
            }
            __syncthreads();
            PHASE(4);
            // per parent: successor count, |msgs|, Assert and deadlock keys (level-local index p); a dense split
            // chunk's slots for the round's parents: wave 0 scans their counts, the round's slots follow the batch's
            // earlier rounds' from the start of the batch's sparse range (an LDS counter: a global atomic per round
            // on the critical path cost the expansion 14 %, profiles/r06_ab_expansion.txt)
            if (tid < 64) {
                const uint32_t jj = a + (uint32_t)tid;
                const bool in = (uint32_t)tid < b - a;
                if (in) {
                    const uint64_t pl = b0 + jj, p = P.p_begin + pl;
                    const uint32_t total = sCnt[jj] + sSelf[jj], ak = sAk[jj];
                    P.cnt[pl] = total;
                    if (P.hcnt) P.hcnt[pl] = sCnt[jj];
                    if (!FUSE && sCnt[jj]) atomicAdd(&sHfp, sCnt[jj]);
                    P.pnm[pl] = (sCore[jj * NWP + Lo::W_MISC] >> 16) & 0xFFu;
                    if (ak != KEY_NONE) atomicMin(&P.err[ERR_ASSERT], (((unsigned long long)p << 16) | ak) << 8);
                    else if (total == 0 && P.check_deadlock)
                        atomicMin(&P.err[ERR_DEADLOCK], ((unsigned long long)p << 16) << 8);
                }
                if (!FUSE && P.hoff) {
                    uint32_t tot;
                    const uint32_t x = wave_excl_scan(in ? sCnt[jj] : 0u, tid, &tot);
                    const uint32_t b32 = (uint32_t)(b0 * (uint64_t)MX) + sAlloc + x;
                    if (in) {
                        sHo[jj] = b32;
                        P.hoff[b0 + jj] = b32;
                    }
                    if (tid == 0) sAlloc += tot;
                }
            }
            if (tid < IC_N) sCc[tid] = 0u;  // (every lane has read its item: the sync above)
            __syncthreads();
            PHASE(6);
            // each enabled successor's rank in TLC order and its slot (the next round's class lists touch neither
            // the key lists nor these parents' counts: no barrier before them)
            if ((uint32_t)tid < nI) {
                const uint32_t kb = (sItm[j] - ibase) * NCI, cn = sCnt[j];
                const uint64_t pl = b0 + j;
                const uint64_t q0 = (!FUSE && P.hoff) ? (uint64_t)sHo[j] : pl * (uint64_t)MX;  // the parent's first slot
#pragma unroll
                for (int c = 0; c < NCI; c++) {
                    const RowSucc<S::NADD> &x = c ? ob : o;
                    if (x.key == KEY_NONE || (!FUSE && x.self && P.hcnt)) continue;
                    uint32_t rank = 0;
                    for (uint32_t e = 0; e < cn; e++) rank += (uint32_t)sKey[kb + e] < x.key ? 1u : 0u;
                    const uint64_t q = q0 + rank;
                    if constexpr (FUSE) {
                        // a fused level: a self-loop takes its slot as seen (the parent is in the seen set);
                        // any other successor is staged for the commit, fingerprinted from the parent's core
                        // and hash sums in LDS, probed and elected right here (k_hash_probe's work)
                        if (x.self) {
                            P.lslot[q] = LS_SEEN;
                            atomicAdd(&sSelfN, 1u);
                            continue;
                        }
                        uint4 st4[S::SW4];
                        row_stage<S::NADD>(x, nmj, S::SW4, st4);
                        uint4 *dst = P.score + q * (uint64_t)S::SW4;
#pragma unroll
                        for (int w = 0; w < S::SW4; w++) dst[w] = st4[w];
                        const unsigned long long *m0 = sM0 + j * NPR, *m1 = sM1 + j * NPR;
                        const ulonglong2 f = staged_fp<N, V, MR>(
                            P, sCore + j * NWP, [&](int pi) { return make_ulonglong2(m0[pi], m1[pi]); },
                            [&](int a, uint32_t) { return x.ainf[a]; }, st4[0], st4[1],
                            S::SW4 > 2 ? st4[S::SW4 > 2 ? 2 : 0] : make_uint4(0u, 0u, 0u, 0u), sK);
                        P.fp[q] = f;
                        P.lslot[q] = probe_elect<MX>(P, f, q, (x.nadd + (nmj & 1u) + 1u) >> 1, P.Lmask);
                    } else {
                        row_stage<S::NADD>(x, nmj, S::SW4, P.score + q * (uint64_t)S::SW4);
                    }
                }
            }
            PHASE(5);
            a = b;
        }
    }
    __syncthreads();
    if constexpr (FUSE) {
        if (tid == 0 && sSelfN)
            atomicAdd(&P.sum[SUM_SELF_STRIPE + SELF_STRIDE * (blockIdx.x % SELF_STRIPES)], (unsigned long long)sSelfN);
    } else {
        if (tid == 0 && sHfp) atomicAdd(&P.sum[SUM_HFP], (unsigned long long)sHfp);
    }
    PHASE_FLUSH;
}

// Every successor slot of a split chunk, a lane each: a wave takes 64 consecutive parents, their
// successor counts are scanned across the wave and successor i of the group goes to lane i % 64 of
// round i / 64 (its parent found by a binary search over the scan); f(parent pl, rank r, its slot sq):
// sq = pl * MX + r in the sparse layout, P.hoff[pl] + r in a dense split chunk's.
template <int MX, class F>
__device__ __forceinline__ void each_successor(const KParams &P, F &&f) {
    const int lane = threadIdx.x & 63;
    const uint64_t np = P.p_end - P.p_begin;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t g0 = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64; g0 < np;
         g0 += nwaves * 64) {
        const uint64_t pl = g0 + (uint64_t)lane;
        const uint32_t t = pl < np ? (P.hcnt ? P.hcnt : P.cnt)[pl] : 0u;  // (a split chunk: its self-loops are not visited)
        const uint32_t h0 = (pl < np && P.hoff) ? P.hoff[pl] : 0u;
        uint32_t tot;
        const uint32_t ex = wave_excl_scan(t, lane, &tot);
        for (uint32_t b0 = 0; b0 < tot; b0 += 64) {
            const uint32_t i = b0 + (uint32_t)lane;
            // the last lane j with ex[j] <= i: ex[j + 1] = ex[j] + t[j] > i, so t[j] > 0
            int j = 0;
#pragma unroll
            for (int st = 32; st; st >>= 1) {
                const uint32_t v = (uint32_t)__shfl(ex, j + st, 64);
                j = v <= i ? j + st : j;
            }
            const uint32_t exj = (uint32_t)__shfl(ex, j, 64);
            const uint32_t hj = (uint32_t)__shfl(h0, j, 64);
            const uint64_t pj = g0 + (uint64_t)j;
            if (i < tot) f(pj, i - exj, P.hoff ? (uint64_t)hj + (i - exj) : pj * (uint64_t)MX + (i - exj));
        }
    }
}

// ---- sharded round: the owner's election table (k_hash_probe, k_local_elect, k_owner_elect) ----
// A fingerprint already in the seen set loses; otherwise it takes (or finds) its slot in the
// round's election table and bids its key.  The table is cleared only every 65533 rounds
// (owner_table): `round` counts the rounds since, and both words of a slot carry its 16-bit tag
// round + 1 in their low bits, so a slot of an earlier round reads as free, and a key word is the
// round's key below ((0xFFFF - tag) << 48) -- smaller than any earlier round's -- so every bid just
// takes the minimum (OT: fingerprint, OK: smallest tagged key; the same protocol as the fused
// election).  key = ((parent's global index in the level << 10 | rank) << 2) | e: TLC's order of the level,
// and in its two low bits the record words a winner adds (elect_key's e; 0 in a received item's key).
__device__ __forceinline__ unsigned long long owner_key(uint32_t tag, uint64_t key) {
    return ((unsigned long long)(0xFFFFu - tag) << 48) | key;  // key < 2^48
}
__device__ __forceinline__ uint64_t owner_order(uint64_t gparent, uint32_t rank, uint32_t e) {
    return (((gparent << 10) | rank) << 2) | e;
}
// the same successor: the keys without e
__device__ __forceinline__ bool owner_same(unsigned long long k, unsigned long long want) { return (k | 3ull) == (want | 3ull); }
// The shard's own parents of the round (global indices g0 .. g0 + np - 1) and their winner accumulator:
// a bid that becomes its slot's minimum counts on its parent if the parent is one of these, and takes the
// displaced bid off its parent if that one is -- so the winners per parent are exact once every bid is in
// (the fused election's wacc protocol), and no pass over the own successors' verdicts has to count them.
struct OwnerLocal {
    uint32_t *wacc;
    uint64_t g0, np;
};
__device__ __forceinline__ uint32_t owner_bid(ESlot *OT, uint64_t mask, uint32_t tag32,
                                              const ulonglong2 f, uint64_t key, const OwnerLocal &loc) {
    const unsigned long long tag = tag32;
    const unsigned long long xk = (f.x & ~0xFFFFull) | tag, yk = (f.y & ~0xFFFFull) | tag;
    // one exit at the bottom (no break): a claimer stores its y inside the loop, in the same
    // iteration as its CAS, before any lane of its wave waits for that y (a divergent break
    // lets the compiler defer the claimer's store until every lane has left the loop)
    uint64_t g = l_index(f, mask);
    unsigned long long v = __hip_atomic_load(&OT[g].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool done = false;
    while (!done) {
        bool next = false;
        if ((v & 0xFFFFull) != tag) {  // free, or an earlier round's: claim it
            const unsigned long long prev = atomicCAS(&OT[g].x, v, xk);
            if (prev == v) {
#ifdef RMC_RACE_PROBE
                if ((key & 7u) == 0u) race_delay(2);  // x claimed, y not yet visible
#endif
                __hip_atomic_store(&OT[g].y, yk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                done = true;
            } else {
                v = prev;
            }
        }
        if (!done && (v & 0xFFFFull) == tag) {
            if (v == xk) {
                const unsigned long long y = __hip_atomic_load(&OT[g].y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (y == yk) done = true;
                else if ((y & 0xFFFFull) == tag) next = true;
                else v = __hip_atomic_load(&OT[g].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // y not visible yet
            } else {
                next = true;
            }
        }
        if (next) {
            g = (g + 1) & mask;
            v = __hip_atomic_load(&OT[g].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    const unsigned long long nk = owner_key(tag32, key);
    const unsigned long long old = atomicMin(&OT[g].k, nk);
    if (loc.wacc && nk < old) {
        const uint64_t gp = key >> 12;
        if (gp - loc.g0 < loc.np) atomicAdd(&loc.wacc[gp - loc.g0], 1u + ((uint32_t)(key & 3u) << 12));
        if ((old >> 48) == (unsigned long long)(0xFFFFu - tag32)) {  // a bid of this round displaced
            const uint64_t ok = old & ((1ull << 48) - 1ull), op = ok >> 12;
            if (op - loc.g0 < loc.np) atomicSub(&loc.wacc[op - loc.g0], 1u + ((uint32_t)(ok & 3u) << 12));
        }
    }
    return (uint32_t)g;
}

// Split chunk: every successor's fingerprint, seen-set probe and election, a lane per successor.
// The expansion (M_SPLIT) left each parent's hash context (its packed core and its message-hash
// sums per server pair, ctx_words) and each successor's staged row; the successor's content
// matrix is rebuilt from those (rmc_spec.h), its coset minimum taken, and the fingerprint probed
// and elected with the fused pass's protocol (elect_slot) -- 64 independent chains per wave instead
// of the ~5 of one parent, and the hash at full lane occupancy.  A sharded round (P.route) only
// needs the fingerprints: its owners probe and elect.
#ifndef RMC_PROBE_WAVES  // waves per SIMD the probe pass's registers are cut for (0: the compiler's choice)
#define RMC_PROBE_WAVES 0
#endif
template <int N, int V, int MR, int MX>
__global__ __launch_bounds__(256, RMC_PROBE_WAVES) void k_hash_probe(KParams P) {
    using S = Spec<N, V, MR>;
    using Lo = Layout<N, V>;
    constexpr int CTXW = ctx_words<N, V>(), CC4 = (S::CCW + 3) / 4;
    __shared__ uint64_t sK[2][N * N];
    __shared__ uint32_t sOwn[64];  // sharded round: the block's successors per owner (P.ocnt)
    if (threadIdx.x < 2 * N * N) {
        const int f = threadIdx.x / (N * N), a = (threadIdx.x / N) % N, b = threadIdx.x % N;
        sK[f][a * N + b] = P.t.seeds[f * SEEDS_PER_F + a * MAXN + b];
    }
    if (threadIdx.x < 64) sOwn[threadIdx.x] = 0u;
    // The election table of the chunk: twice its successors to fingerprint (counted by the expansion), not
    // the host's bound of MAXS per parent -- ~35x fewer slots at Raft.cfg's depth, so the elections' random
    // lines stay in the caches far more often (every slot of the table is free for this chunk's tag, so any
    // prefix of it serves)
    uint64_t Lmask = P.Lmask;
    if (!P.route) {
        const unsigned long long nf = __hip_atomic_load(&P.sum[SUM_HFP], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t want = nf < 512ull ? 1024ull : 1ull << (64 - __clzll((long long)(2 * nf - 1)));
        Lmask = want - 1 < Lmask ? want - 1 : Lmask;
    }
    __syncthreads();
    each_successor<MX>(P, [&](uint64_t pl, uint32_t r, uint64_t sq) {
        const uint64_t q = pl * (uint64_t)MX + r;  // TLC's order (the election key); sq: the slot
        const uint4 *cx = reinterpret_cast<const uint4 *>(P.hctx + pl * (uint64_t)CTXW);
        const uint4 *st = P.score + sq * (uint64_t)S::SW4;
        const uint4 sa = st[0], sb = st[1];
        const uint4 sc = S::SW4 > 2 ? st[2] : make_uint4(0u, 0u, 0u, 0u);
        uint32_t pk[CC4 * 4];
#pragma unroll
        for (int k = 0; k < CC4; k++) {
            const uint4 v = cx[k];
            pk[4 * k] = v.x; pk[4 * k + 1] = v.y; pk[4 * k + 2] = v.z; pk[4 * k + 3] = v.w;
        }
        uint4 mp[N * (N - 1)];
#pragma unroll
        for (int k = 0; k < N * (N - 1); k++) mp[k] = cx[CC4 + k];
        uint32_t pc[Lo::NW];
        decode_core<N, V>(pk, pc);
        const ulonglong2 f = staged_fp<N, V, MR>(P, pc, [&](int pi) {
            const uint4 m = mp[pi];
            return make_ulonglong2((uint64_t)m.y << 32 | m.x, (uint64_t)m.w << 32 | m.z);
        }, [&](int, uint32_t id) { return P.t.info[id]; }, sa, sb, sc, sK);
        const uint32_t nadd = sb.z >> 16;
        P.fp[sq] = f;
        if (P.route) {  // the owners probe and elect; the round's counts per owner (k_route_count's)
            const uint32_t o = fp_owner(f, P.nown);
            if (P.ocnt) atomicAdd(&sOwn[o], 1u);
            // the shard's own successors bid in its owner table right here (k_local_elect's work;
            // the others are marked for the exchange)
            if (P.OT) {
                const uint32_t nm = (pc[Lo::W_MISC] >> 16) & 0xFFu;
                P.lslot[sq] = o != P.self ? LS_ELECT
                              : seen_contains(P.seen, f)
                                  ? LS_SEEN
                                  : owner_bid(P.OT, P.ot_mask, P.ot_round + 1u, f,
                                              owner_order(P.gblk + pl, r, (nadd + (nm & 1u) + 1u) >> 1),
                                              OwnerLocal{P.wacc, P.gblk, P.p_end - P.p_begin});
            }
            return;
        }
        const uint32_t nm = (pc[Lo::W_MISC] >> 16) & 0xFFu;
        P.lslot[sq] = probe_elect<MX>(P, f, q, (nadd + (nm & 1u) + 1u) >> 1, Lmask);
    });
    if (P.route && P.ocnt) {
        __syncthreads();
        if (threadIdx.x < P.nown && sOwn[threadIdx.x]) atomicAdd(&P.ocnt[threadIdx.x], sOwn[threadIdx.x]);
    }
}

// Split chunk, once the election is over: every winner's fingerprint into the seen set, a lane per
// successor, and every candidate's verdict in its slot (LS_WIN / LS_SEEN, as the owners' verdicts of a
// sharded round) -- the commit then reads neither the election words nor inserts: both were
// dependent round trips per parent with winners
template <int MX>
__global__ __launch_bounds__(256) void k_insert_winners(KParams P) {
    each_successor<MX>(P, [&](uint64_t pl, uint32_t r, uint64_t sq) {
        const uint64_t q = pl * (uint64_t)MX + r;
        const uint32_t g = P.lslot[sq];
        if (g >= LS_ELECT) return;
        const bool w = elect_q(P.ET[g].k) == (uint32_t)q;
        if (w) seen_insert(P.seen, P.fp[sq]);
        if (P.split & 4) P.lslot[sq] = w ? LS_WIN : LS_SEEN;  // the verdict: the commit needs no election word
    });
}

// fingerprints of whole states (Init, test hooks): one wave per state
template <int N, int V, int MR>
__global__ __launch_bounds__(64) void k_fp_states(KParams P, uint64_t n) {
    using S = Spec<N, V, MR>;
    __shared__ uint64_t M0[N * N], M1[N * N];
    __shared__ uint32_t pcore[Layout<N, V>::NW + N];
    const int lane = threadIdx.x;
    for (uint64_t p = blockIdx.x; p < n; p += gridDim.x) {
        Wave<N, V, MR> W;
        load_parent<N, V, MR, true>(P, rec_start<S::RECW_MAX>(P, p), lane, W, M0, M1, pcore);
        const ulonglong2 f = fingerprint<N, V>(W.c, M0, M1, P.t);
        if (lane == 0) P.fp[p] = f;
    }
}

template <int N, int V, int MR>
__global__ __launch_bounds__(64) void k_inv_states(KParams P, uint64_t n, int32_t *out) {
    using S = Spec<N, V, MR>;
    using Lo = Layout<N, V>;
    const uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    const uint64_t start = rec_start<S::RECW_MAX>(P, i);
    uint32_t packed[S::CCW], c[Lo::NW];
#pragma unroll
    for (int k = 0; k < S::CCW; k++) packed[k] = ring_word(P.front, start, (uint32_t)k, P.rcap);
    decode_core<N, V>(packed, c);
    const MsgView mv{P.front, ring_wrap(start + S::CCW, P.rcap), P.rcap, (c[Lo::W_MISC] >> 16) & 0xFFu, 0u, 0u, 0u,
                     P.t.info};
    for (int b = 0; b < 7; b++) out[i * 7 + b] = inv_eval<N, V>(c, b, mv);
}

// ---- fused level: winner counts, commit --------------------------------------------------------
// Exclusive scan of one value per thread over a 1024-thread block (16 waves); *total gets the
// block's sum.  ws holds 16 words of LDS.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *ws, uint32_t *total) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    __syncthreads();
    if (lane == 63) ws[wv] = x;
    __syncthreads();
    uint32_t base = 0, all = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; k++) {
        const uint32_t w = ws[k];
        base += k < wv ? w : 0u;
        all += w;
    }
    *total = all;
    return base + x - v;
}

// One 1024-thread block per WTILE-parent tile, thread per parent: winners per parent (wcnt, as the
// election counted them in wacc) and their record words, the exclusive scans of both inside the
// tile (wpos, wposw), and per tile the winners (bw), words (bww) and successors generated (bg).
// The last block to finish scans the tile totals into boff / boffw and writes {generated, winners,
// words} to the chunk summary -- the only values the host needs before commit.
template <int N, int V, int MR>
__global__ __launch_bounds__(1024) void k_wincount(KParams P) {
    constexpr uint32_t CCW = (uint32_t)Spec<N, V, MR>::CCW;
    __shared__ uint32_t ws[16];
    __shared__ uint32_t flag;
    if (!level_args(P)) return;
    const uint64_t np = P.p_end - P.p_begin;
    const uint32_t ntiles = (uint32_t)((np + WTILE - 1) / WTILE);
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t pl = (uint64_t)tile * WTILE + threadIdx.x;
        uint32_t w = 0, t = 0, wd = 0;
        if (pl < np) {
            // winners per parent were counted by the election itself; the accumulator is
            // re-armed for the next chunk here
            t = P.cnt[pl];
            const uint32_t wa = P.wacc[pl], nm = P.pnm[pl];
            P.wacc[pl] = 0u;
            w = wa & 0xFFFu;
            wd = w * (CCW + (nm >> 1)) + (wa >> 12);
        }
        uint32_t wt, gt, dt;
        const uint32_t x = block_excl_scan(w, ws, &wt);
        (void)block_excl_scan(t, ws, &gt);
        const uint32_t xd = block_excl_scan(wd, ws, &dt);
        if (pl < np) {
            P.wcnt[pl] = w;
            P.wpos[pl] = x;
            P.wposw[pl] = xd;
        }
        // parents with winners in the tile (for k_nzlist)
        const uint32_t nt = P.plist ? (uint32_t)__syncthreads_count(w != 0u) : 0u;
        if (P.hcnt) {  // the tile's self-loops (set apart by the split expansion) for the level's statistics
            uint32_t st;
            (void)block_excl_scan(pl < np ? t - P.hcnt[pl] : 0u, ws, &st);
            if (threadIdx.x == 0 && st) atomicAdd(&P.sum[SUM_SELF], (unsigned long long)st);
        }
        if (ntiles == 1) {  // one tile (small levels): its totals are the chunk's, no arrival round trips
            if (threadIdx.x == 0) {
                P.boff[0] = 0u;
                P.boffw[0] = 0u;
                P.sum[0] = gt;
                P.sum[1] = wt;
                P.sum[SUM_WORDS] = dt;
                if (P.plist) {
                    P.bn[0] = nt;
                    P.boffn[0] = 0u;
                    P.sum[SUM_NZ] = nt;
                }
            }
            return;
        }
        if (threadIdx.x == 0) {
            // write-through (sc1) stores: the last block reads them with sc1 loads, no fences
            __hip_atomic_store(&P.bw[tile], wt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&P.bg[tile], gt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&P.bww[tile], dt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (P.plist) __hip_atomic_store(&P.bn[tile], nt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // arrivals: only the nb blocks that had a tile (MI355X guide: sc1 payload, drained, then an
    // agent-scope atomic add; the last adder reads the payload with sc1 loads)
    const uint32_t nb = ntiles < gridDim.x ? (ntiles ? ntiles : 1u) : gridDim.x;
    if (blockIdx.x >= nb) return;
#ifdef RMC_RACE_PROBE
    if (blockIdx.x == 0 && nb > 1) race_delay(8);  // block 0 arrives last
#endif
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t a = __hip_atomic_fetch_add(&P.tickets[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = a == nb - 1;
        if (last) __hip_atomic_store(&P.tickets[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag = last ? 1u : 0u;
    }
    __syncthreads();
    if (!flag) return;
    // tile offsets (ntiles <= WTILES_MAX: thread i takes tiles TPT i .. TPT i + TPT - 1) and the
    // chunk totals
    constexpr uint32_t TPT = WTILES_MAX / 1024;
    static_assert(TPT * 1024 == WTILES_MAX, "whole tiles per thread of the 1024-thread block");
    uint32_t wv[TPT], gv[TPT], dv[TPT], wtot, gtot, dtot, ws_ = 0, gs_ = 0, ds_ = 0;
    const uint32_t i = threadIdx.x;
#pragma unroll
    for (uint32_t k = 0; k < TPT; k++) {
        const uint32_t tl = TPT * i + k;
        wv[k] = gv[k] = dv[k] = 0u;
        if (tl < ntiles) {
            wv[k] = __hip_atomic_load(&P.bw[tl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            gv[k] = __hip_atomic_load(&P.bg[tl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            dv[k] = __hip_atomic_load(&P.bww[tl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        ws_ += wv[k];
        gs_ += gv[k];
        ds_ += dv[k];
    }
    uint32_t o = block_excl_scan(ws_, ws, &wtot);
    (void)block_excl_scan(gs_, ws, &gtot);
    uint32_t od = block_excl_scan(ds_, ws, &dtot);
#pragma unroll
    for (uint32_t k = 0; k < TPT; k++) {
        const uint32_t tl = TPT * i + k;
        if (tl < ntiles) {
            P.boff[tl] = o;
            P.boffw[tl] = od;
        }
        o += wv[k];
        od += dv[k];
    }
    if (i == 0) {
        P.sum[0] = gtot;
        P.sum[1] = wtot;
        P.sum[SUM_WORDS] = dtot;
    }
    if (P.plist) {  // parents with winners: tile offsets and the chunk's count
        uint32_t nv[TPT], ns_ = 0, ntot;
#pragma unroll
        for (uint32_t k = 0; k < TPT; k++) {
            const uint32_t tl = TPT * i + k;
            nv[k] = tl < ntiles ? __hip_atomic_load(&P.bn[tl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
            ns_ += nv[k];
        }
        uint32_t on = block_excl_scan(ns_, ws, &ntot);
#pragma unroll
        for (uint32_t k = 0; k < TPT; k++) {
            const uint32_t tl = TPT * i + k;
            if (tl < ntiles) P.boffn[tl] = on;
            on += nv[k];
        }
        if (i == 0) P.sum[SUM_NZ] = ntot;
    }
}

// The chunk-local indices of the parents with winners, in order (one 1024-thread block per tile of
// the winner count: its parents' winner counts, scanned, at the tile's offset).  A split chunk's
// commit visits only these: at Raft.cfg's wide levels most parents' successors are all seen.
__global__ __launch_bounds__(1024) void k_nzlist(KParams P) {
    __shared__ uint32_t ws[16];
    const uint64_t np = P.p_end - P.p_begin;
    const uint32_t ntiles = (uint32_t)((np + WTILE - 1) / WTILE);
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t pl = (uint64_t)tile * WTILE + threadIdx.x;
        const uint32_t w = pl < np ? P.wcnt[pl] : 0u;
        uint32_t tot;
        const uint32_t x = block_excl_scan(w ? 1u : 0u, ws, &tot);
        if (w) P.plist[P.boffn[tile] + x] = (uint32_t)pl;
    }
}

// the commit's arrival counters (last_commit_block): CTICK_SUB sub-counters and a top one, each on its own line
constexpr uint32_t CTICK_SUB = 32, CTICK_STRIDE = 32;

// Chunk summary, by the last block of the commit pass (one wave): {generated, winners, words} (from the
// winner count pass), the error keys and flags (then re-armed).  In device-loop mode it also
// records the level and advances the control block to the next one -- or stops the loop.
template <int MAXS, int RECW_MAX>
__device__ void finish_level(const KParams &P) {
    // one wave, everything it reads in flight at once: lanes 0..3 take the error slots, lane 4
    // the flags, lane 0 the summary and the control block
    // (the summary words and the control block, which this launch does not write, go out with the
    // exchanges: one round trip)
    const int lane = threadIdx.x;
    unsigned long long *sm = P.sum;
    unsigned long long G = 0, Wn = 0, Ww = 0;
    LevelCtl c{};
#ifdef RMC_RACE_PROBE
    // when the last arriver gets here every block of the launch has arrived and every counter has
    // re-armed itself (a sub-counter's last re-arms it before it arrives at the top one): a counter
    // left off by an arrival from another level (the late-block race) shows here
    if (lane == 0 && P.ctick) {
        uint32_t off = 0;
        for (uint32_t i = 0; i <= CTICK_SUB; i++)
            off |= __hip_atomic_load(P.ctick + i * CTICK_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (off) atomicOr(&P.flags[0], 4u);
    }
#endif
    if (lane == 0) {
        G = sm[0];
        Wn = sm[1];
        Ww = sm[SUM_WORDS];
        if (P.ctl) c = *ctl_cur(P);
    }
    // the fused expansion's self-loops, striped over SELF_STRIPES lines (one atomic per block each):
    // into the level's record (device loop) or the chunk's sum[SUM_SELF] (host-driven), re-armed
    unsigned long long Sf = 0;
    if (lane < SELF_STRIPES) {
        Sf = __hip_atomic_exchange(&sm[SUM_SELF_STRIPE + SELF_STRIDE * lane], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int o = SELF_STRIPES / 2; o; o >>= 1) Sf += __shfl_xor(Sf, o, SELF_STRIPES);
        if (lane == 0 && !P.ctl && Sf) atomicAdd(&sm[SUM_SELF], Sf);
    }
    unsigned long long e = 0;
    if (lane < ERR_NSLOTS)
        e = __hip_atomic_exchange(&P.err[lane], ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (lane == ERR_NSLOTS)
        e = __hip_atomic_exchange(&P.flags[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool bad = __ballot(lane < ERR_NSLOTS ? e != ~0ull : (lane == ERR_NSLOTS && e != 0)) != 0;
    if (lane <= ERR_NSLOTS) sm[2 + lane] = e;
    if (lane != 0) return;
    if (!P.ctl) return;
    if (bad) {  // the host reports the error from this level's buffers
        c.stop = CTL_ERROR;  // the erroring level's block, not advanced, into both (see below)
        *ctl_nxt(P) = c;
        *ctl_cur(P) = c;
        if (P.hloop) {
            c.stop = CTL_ERROR;
            P.hloop->ctl = c;
            __hip_atomic_store(&P.hloop->stop, (uint32_t)CTL_ERROR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;
    }
    if (c.done_levels < (uint32_t)LREC_CAP) {
        LevelRec r;
        r.expanded = c.cur_n;
        r.generated = G;
        r.new_states = Wn;
        r.words = Ww;
        r.self_loops = Sf;
        P.lrec[c.done_levels] = r;
        if (P.hloop) P.hloop->rec[c.done_levels] = r;
    }
    c.done_levels++;
    c.gid_cur += c.cur_n;
    c.cur_n = Wn;
    c.cur_wbase = ring_wrap(c.cur_wbase + c.cur_words, c.rcap);
    c.cur_words = Ww;
    c.T_count += Wn;
    c.level++;
    c.epoch++;
    const unsigned long long Gub = Wn * (unsigned long long)MAXS;
    unsigned long long lc = 1;
    while (lc < 2 * Gub) lc <<= 1;
    c.Lmask = (lc < c.Lcap_max ? lc : c.Lcap_max) - 1;
    if (Wn == 0)
        c.stop = CTL_DONE;
    else if (c.done_levels >= c.batch || c.done_levels >= (uint32_t)LREC_CAP || Wn > c.chunk_parents ||
             Gub > c.off_cap || Ww + Gub * RECW_MAX > c.rcap || c.gid_cur + Wn + Gub - c.trace_base > c.trace_cap ||
             2 * (c.T_count + Gub) > c.T_cap)
        c.stop = CTL_HOST;  // the next level is not known to fit the buffers: the host grows them
    // into the other block of the pair: a late block of this launch (one with no parent, which
    // leaves without arriving) still reads this level's block, never the next level's
    // A stopped loop's block goes into both: the no-op launches after it read either.
    *ctl_nxt(P) = c;
    if (c.stop != CTL_RUN) *ctl_cur(P) = c;
#ifdef RMC_RACE_PROBE
    // (the probe's late block polls `level`: the block's words visible device-wide first)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_store(&ctl_nxt(P)->level, c.level, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
    // The loop's stop goes to the host here, with the control block (read after the drain); the
    // running loop's progress is reported by the next level's expansion as it starts (k_expand):
    // a write to host memory at the end of this kernel would hold the next launch ~5.6 us.
    if (P.hloop && c.stop != CTL_RUN) {
        P.hloop->ctl = c;
        __hip_atomic_store(&P.hloop->done, c.done_levels, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&P.hloop->stop, c.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// True in the last one-wave block of the commit pass to get here, among the nb blocks that had a
// parent (the others leave without arriving).  Arrivals go to CTICK_SUB counters (block b to
// b % CTICK_SUB, each on its own 128-B line) and the last arriver of each to one top counter, so
// no counter sees more than nb / CTICK_SUB atomics.  No fence: the last
// block reads nothing that this launch wrote except the error words, and those are atomics that
// every wave has completed (vmcnt(0)) before its arrival.  Counters re-arm themselves.
__device__ __forceinline__ bool last_commit_block(uint32_t *tick, uint32_t nb) {
    if (blockIdx.x >= nb) return false;
#ifdef RMC_RACE_PROBE
    if (blockIdx.x == 0 && nb > 1) race_delay(8);  // block 0 arrives last
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t last = 0;
    if (threadIdx.x == 0 && nb <= CTICK_SUB) {  // few blocks: straight to the top counter
        uint32_t *top = tick + CTICK_SUB * CTICK_STRIDE;
        if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nb - 1) {
            __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = 1;
        }
    } else if (threadIdx.x == 0) {
        const uint32_t g = nb, b = blockIdx.x, sub = b % CTICK_SUB;
        const uint32_t nsub = g < CTICK_SUB ? g : CTICK_SUB;
        const uint32_t expect = (g - sub + CTICK_SUB - 1) / CTICK_SUB;  // blocks with b % CTICK_SUB == sub
        uint32_t *c = tick + sub * CTICK_STRIDE, *top = tick + CTICK_SUB * CTICK_STRIDE;
        if (__hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == expect - 1) {
            __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsub - 1) {
                __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last = 1;
            }
        }
    }
    return __builtin_amdgcn_readfirstlane(last) != 0;
}

// One wave per parent with winners: rebuild each winner (in TLC order) from the parent's core and
// its staged row, check the INVARIANTs (Raft.cfg:33) on it, append it to the next level (record
// at the scanned word offset, its offset in noff), insert its fingerprint, record its parent
// pointer and slot key.
template <int N, int V, int MR, bool BFV = false>
__global__ __launch_bounds__(64, (N <= 3 && MR == 1) ? RMC_N3_COMMIT_WAVES : 1) void k_commit(KParams P) {
    using S = Spec<N, V, MR>;
    using Lo = Layout<N, V>;
    constexpr int MX = S::MAXS + (BFV ? S::MCAP : 0);  // successor slots per parent (k_expand)
#ifdef RMC_RACE_PROBE
    if (P.ctl) {  // the first block without a parent of this level reads its block after the level advanced
        const LevelCtl *c = ctl_cur(P);
        const uint32_t lv = c->level;
        if (c->stop == CTL_RUN && (uint64_t)blockIdx.x == c->cur_n) {
            race_wait(4000, [&] {
                return __hip_atomic_load(&ctl_nxt(P)->level, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == lv;
            });
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
    }
#endif
    if (!level_args(P)) return;
    const int lane = threadIdx.x;
    const uint64_t lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;
    // every load of a parent that depends on no other load goes out at once: its winner count,
    // offsets, successor count and first 64 election slots (read ahead of knowing whether they are
    // needed; all in bounds; commit always reads a ring level: foff is set).  The header's uniform
    // words travel in one VGPR: lane k loads word k (one load instruction for all of them, two
    // registers per header in flight instead of ten).  Software pipeline: the next parent's header
    // goes out with this parent's record, so its round trip overlaps this one's instead of starting
    // the next iteration.
    struct Hdr {
        uint32_t hw, g0;
    };
    auto header = [&](uint64_t p) {
        const uint64_t pl = p - P.p_begin;
        const uint32_t *src;
        switch (lane & 7) {
        case 0: src = (const uint32_t *)(P.foff + p); break;
        case 1: src = (const uint32_t *)(P.foff + p) + 1; break;
        case 2: src = P.wcnt + pl; break;
        case 3: src = P.boff + pl / WTILE; break;
        case 4: src = P.wpos + pl; break;
        case 5: src = P.cnt + pl; break;
        case 6: src = P.boffw + pl / WTILE; break;
        default: src = P.wposw + pl; break;
        }
        Hdr h;
        h.hw = lane < 8 ? *src : 0u;
        h.g0 = lane < MX ? P.lslot[pl * (uint64_t)MX + lane] : LS_SEEN;
        return h;
    };
    // the parents this pass visits: k-th -> level-local index (a split chunk: only those with winners)
    const uint64_t nvis = P.plist ? (uint64_t)P.sum[SUM_NZ] : P.p_end - P.p_begin;
    auto parent_at = [&](uint64_t k) -> uint64_t { return P.p_begin + (P.plist ? (uint64_t)P.plist[k] : k); };
    // pq: the parents of k, k + grid, k + 2 grid
    Hdr nh{};
    uint64_t pq[3] = {0, 0, 0};
#pragma unroll
    for (int j = 0; j < 3; j++)
        if (blockIdx.x + (uint64_t)j * gridDim.x < nvis) pq[j] = parent_at(blockIdx.x + (uint64_t)j * gridDim.x);
    if (blockIdx.x < nvis) nh = header(pq[0]);
    PHASE_DECL
    for (uint64_t k = blockIdx.x; k < nvis; k += gridDim.x) {
        const uint64_t p = pq[0];
        pq[0] = pq[1];
        pq[1] = pq[2];
        pq[2] = k + 3ull * gridDim.x < nvis ? parent_at(k + 3ull * gridDim.x) : 0ull;
        const uint64_t pl = p - P.p_begin;
        const Hdr h = nh;
        if (k + gridDim.x < nvis) nh = header(pq[0]);
        const uint32_t g0 = h.g0;
        const uint32_t wc = rdlane(h.hw, 2);
        PHASE(0);
        if (!wc) continue;
        const uint64_t foffp = ((uint64_t)rdlane(h.hw, 1) << 32) | rdlane(h.hw, 0);
        const uint32_t bo = rdlane(h.hw, 3), wp = rdlane(h.hw, 4), t = rdlane(h.hw, 5);
        const uint32_t bow = rdlane(h.hw, 6), wpw = rdlane(h.hw, 7);
        const uint64_t start = ring_wrap(P.fbase + foffp, P.rcap);
        // the parent's record in one round trip (as load_parent), and with it the election words
        // of the first 64 slots (their indices came with the first round trip)
        const uint32_t rw0 = lane < S::RECW_MAX ? ring_word(P.front, start, (uint32_t)lane, P.rcap) : 0u;
        const uint32_t rw1 =
            (MR > 1 && 64 + lane < S::RECW_MAX) ? ring_word(P.front, start, 64u + (uint32_t)lane, P.rcap) : 0u;
        // (slots past the parent's t successors hold a stale lslot from an earlier chunk: never an index)
        // (verdicts in lslot -- sharded round, or a split chunk after k_insert_winners -- need no election word)
        const bool verdict = P.route || (P.split & 4);
        const unsigned long long L0 = (!verdict && (uint32_t)lane < t && g0 < LS_ELECT) ? P.ET[g0].k : 0ull;
        // and the staged rows of the first 64 slots that may win (new fingerprints; in a sharded
        // round the owner's verdict is already known): a speculative read instead of a third round
        // trip once the election words are in
        uint4 xa = make_uint4(0u, 0u, 0u, 0u), xb = xa, xc = xa;
        if ((uint32_t)lane < t && (verdict ? g0 == LS_WIN : g0 < LS_ELECT)) {
            const uint4 *src = P.score + (pl * (uint64_t)MX + (uint32_t)lane) * (uint64_t)S::SW4;
            xa = src[0];
            xb = src[1];
            if (S::SW4 > 2) xc = src[2];
        }
        uint32_t pc[Lo::NW], ppk[S::CCW];
#pragma unroll
        for (int k = 0; k < S::CCW; k++) ppk[k] = rdlane(rw0, k);
        decode_core<N, V>(ppk, pc);
        const uint32_t nm = (pc[Lo::W_MISC] >> 16) & 0xFFu;
        const uint64_t idw = ring_wrap(start + S::CCW, P.rcap);
        uint32_t id[MR];
#pragma unroll
        for (int r = 0; r < MR; r++) {
            const uint32_t k = (uint32_t)(r * 64 + lane);
            const uint32_t wi = (uint32_t)S::CCW + (k >> 1);
            const uint32_t a = __shfl(rw0, (int)(wi & 63u), 64);
            const uint32_t b = MR > 1 ? __shfl(rw1, (int)(wi & 63u), 64) : 0u;
            id[r] = k < nm ? (((wi < 64u ? a : b) >> ((k & 1u) * 16u)) & 0xFFFFu) : 0xFFFFu;
        }
        PHASE(1);
        const uint32_t w0 = bo + wp;
        const uint64_t wd0 = P.next_wbase + bow + wpw;
        uint32_t done = 0;
        uint64_t done_w = 0;
        asm volatile("" ::"v"(xa.x), "v"(xa.y), "v"(xa.z), "v"(xa.w), "v"(xb.x), "v"(xb.y), "v"(xb.z), "v"(xb.w),
                     "v"(xc.x));  // issued with the record, not sunk into the winner branch
        for (uint32_t r0 = 0; r0 < t; r0 += 64) {
            const uint32_t r = r0 + (uint32_t)lane;
            const uint64_t q = pl * (uint64_t)MX + r;
            bool win = false;
            if (r < t) {
                const uint32_t g = r0 == 0 ? g0 : P.lslot[q];
                win = verdict ? g == LS_WIN : (g < LS_ELECT && elect_q(r0 == 0 ? L0 : P.ET[g].k) == (uint32_t)q);
            }
            const uint64_t m = __ballot(win);
            PHASE(2);
            if (!m) continue;
            uint32_t pk[S::CCW];
            uint4 sa = make_uint4(0u, 0u, 0u, 0u), sb = sa, sc = sa;
            uint32_t size = 0;
#pragma unroll
            for (int w = 0; w < S::CCW; w++) pk[w] = 0u;
            if (win) {
                if (r0 == 0) {
                    sa = xa;
                    sb = xb;
                    sc = xc;
                } else {
                    const uint4 *src = P.score + q * (uint64_t)S::SW4;
                    sa = src[0];
                    sb = src[1];
                    if (S::SW4 > 2) sc = src[2];
                }
                uint32_t c[Lo::NW];
                unstage_core<N, V>(pc, sa, sb, c);
                encode_core<N, V>(c, pk);
                const uint32_t key = sb.z & 0xFFFFu, nadd = sb.z >> 16;
                size = (uint32_t)S::CCW + ((nm + nadd + 1u) >> 1);
                const uint64_t out = P.next_base + w0 + done + (uint32_t)__popcll(m & lt_mask);
                if (P.route) {
                    // sharded round: the owner already inserted the fingerprint; the trace entry
                    // travels with the record to the state's next-level owner
                    const uint64_t pref = P.gid_parent_base + p;
                    P.xside[out] = make_uint4((uint32_t)pref, (uint32_t)(pref >> 32), key, size);
                } else {
                    const uint64_t gid = P.gid_next_base + out;
                    if (!(P.split & 2)) seen_insert(P.seen, P.fp[q]);  // (split chunk: k_insert_winners)
                    P.par[gid - P.trace_base] = P.gid_parent_base + p;
                    P.pslot[gid - P.trace_base] = (uint16_t)key;
                }
                int which = 0;
                const MsgView mv{P.front, idw, P.rcap, nm, sb.w, sc.x, nadd, P.t.info};
                const int iv = check_invs<N, V>(c, P.inv_order, &which, mv);
                if (iv != 1) {
                    const unsigned long long ek = ((((unsigned long long)p << 16) | key) << 8) | (unsigned long long)which;
                    atomicMin(&P.err[iv == 0 ? ERR_INV : ERR_EVAL], ek);
                }
            }
            PHASE(4);
            uint32_t wtot;
            const uint32_t wpre = wave_excl_scan(size, lane, &wtot);
            if (win) {
                const uint64_t out = P.next_base + w0 + done + (uint32_t)__popcll(m & lt_mask);
                P.noff[out] = wd0 + done_w + wpre;
            }
            // each winner's record (whole wave per record): packed core words + merged ids
            uint32_t i = 0;
            for (uint64_t mm = m; mm; mm &= mm - 1, i++) {
                const int tt = __ffsll((unsigned long long)mm) - 1;
                const uint64_t rstart = ring_wrap(P.nbase + wd0 + done_w + rdlane(wpre, tt), P.rcap);
                uint32_t v = 0;
#pragma unroll
                for (int w = 0; w < S::CCW; w++) {
                    const uint32_t x = rdlane(pk[w], tt);
                    v = (lane == w) ? x : v;
                }
                if (lane < S::CCW) P.next[ring_wrap(rstart + lane, P.rcap)] = v;
                const uint32_t nadd = rdlane(sb.z, tt) >> 16, ay = rdlane(sb.w, tt), az = rdlane(sc.x, tt);
                const uint32_t add[4] = {ay & 0xFFFFu, ay >> 16, az & 0xFFFFu, az >> 16};
                write_ids<N, V, MR>(P.next, ring_wrap(rstart + S::CCW, P.rcap), P.rcap, id, nm, add, nadd, lane);
            }
            done += (uint32_t)__popcll(m);
            done_w += wtot;
            PHASE(5);
        }
    }
    PHASE_FLUSH_AT(8);
    // the last block to leave finishes the level (finish_level)
    const uint64_t np = P.p_end - P.p_begin;
    const uint32_t nb = np < gridDim.x ? (np ? (uint32_t)np : 1u) : gridDim.x;
    if (last_commit_block(P.ctick, nb)) finish_level<MX, S::RECW_MAX>(P);
}

// ---- split chunk / sharded round commit: a lane per successor slot ------------------------------
// The wave-per-parent commit (k_commit) runs a parent's few winners on a few of its 64 lanes, and
// most of its time waits on one parent's chain of round trips.  Here a wave takes 64 consecutive
// parents with winners (plist), their successor counts scanned across the wave, and successor i of
// the group goes to lane i % 64 of round i / 64 (as each_successor); every lane whose slot won
// (lslot == LS_WIN: the split chunk's k_insert_winners verdict, or the owner's in a sharded round)
// rebuilds its state from the parent's record core and its staged row, encodes it, writes its record
// -- core words, then the parent's message ids merged with the ones its action added -- at its next-
// level word offset, its trace entry (or sidecar) and checks the INVARIANTs.  A parent's winners are
// consecutive lanes of a round (or run on into the next), so its winners' ordinals and word offsets
// are segmented scans across the wave plus what the parent's part of the previous round carried.
// The chunk summary follows in k_commit_finish.
template <int N, int V, int MR, int MX>
__global__ __launch_bounds__(256) void k_commit_split(KParams P) {
    using S = Spec<N, V, MR>;
    using Lo = Layout<N, V>;
    constexpr int CCW = S::CCW;
    const int lane = threadIdx.x & 63;
    const uint64_t lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;
    const uint64_t nvis = P.sum[SUM_NZ];
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t g0 = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64; g0 < nvis;
         g0 += nwaves * 64) {
        const uint64_t k = g0 + (uint64_t)lane;
        const uint32_t pl_l = k < nvis ? P.plist[k] : 0u;  // this lane's parent with winners (chunk-local)
        const uint32_t t = k < nvis ? (P.hcnt ? P.hcnt : P.cnt)[pl_l] : 0u;
        uint32_t tot;
        const uint32_t ex = wave_excl_scan(t, lane, &tot);
        uint32_t cw = 0, cs = 0;  // winners / record words the previous round gave the group's parent cj
        int cj = -1;
        for (uint32_t b0 = 0; b0 < tot; b0 += 64) {
            const uint32_t i = b0 + (uint32_t)lane;
            int j = 0;  // the last group entry j with ex[j] <= i
#pragma unroll
            for (int st = 32; st; st >>= 1) {
                const uint32_t v = (uint32_t)__shfl(ex, j + st, 64);
                j = v <= i ? j + st : j;
            }
            const uint32_t r = i - (uint32_t)__shfl(ex, j, 64);
            const uint32_t pl = (uint32_t)__shfl(pl_l, j, 64);
            const uint64_t q = (uint64_t)pl * MX + r;
            const bool win = i < tot && P.lslot[q] == LS_WIN;
            const uint64_t p = P.p_begin + pl;
            uint4 sa = make_uint4(0u, 0u, 0u, 0u), sb = sa, sc = sa;
            uint32_t pk[CCW], c[Lo::NW];
            uint32_t nm = 0, nadd = 0, size = 0;
            uint64_t start = 0;
            if (win) {
                const uint4 *src = P.score + q * (uint64_t)S::SW4;
                sa = src[0];
                sb = src[1];
                if (S::SW4 > 2) sc = src[2];
                start = ring_wrap(P.fbase + P.foff[p], P.rcap);
#pragma unroll
                for (int w = 0; w < CCW; w++) pk[w] = ring_word(P.front, start, (uint32_t)w, P.rcap);
                uint32_t pc[Lo::NW];
                decode_core<N, V>(pk, pc);
                unstage_core<N, V>(pc, sa, sb, c);
                encode_core<N, V>(c, pk);
                nm = (pc[Lo::W_MISC] >> 16) & 0xFFu;
                nadd = sb.z >> 16;
                size = (uint32_t)CCW + ((nm + nadd + 1u) >> 1);
            }
            // segmented (by parent) exclusive winner count and word offset, plus the carry
            const uint64_t wm = __ballot(win);
            const int j0 = __builtin_amdgcn_readfirstlane(j);
            const uint32_t r0 = __builtin_amdgcn_readfirstlane(r);
            const int seg = lane - (int)(j == j0 ? r - r0 : r);  // first lane of this lane's parent in the round
            uint32_t ord = (uint32_t)__popcll(wm & lt_mask & ~((1ull << seg) - 1ull));
            uint32_t szt;
            const uint32_t szx = wave_excl_scan(size, lane, &szt);
            uint32_t wofs = szx - (uint32_t)__shfl(szx, seg, 64);
            if (j == cj) {
                ord += cw;
                wofs += cs;
            }
            {  // what the round's last parent carries into the next round
                const int jl = __builtin_amdgcn_readlane(j, 63), sl = __builtin_amdgcn_readlane(seg, 63);
                const uint32_t szl = __builtin_amdgcn_readlane(szx, sl);
                const uint32_t w_in = (uint32_t)__popcll(wm & ~((1ull << sl) - 1ull));
                const bool cont = jl == cj;
                cw = w_in + (cont ? cw : 0u);
                cs = (szt - szl) + (cont ? cs : 0u);
                cj = jl;
            }
            if (!win) continue;
            const uint32_t tile = pl / WTILE;
            const uint64_t out = P.next_base + P.boff[tile] + P.wpos[pl] + ord;
            const uint64_t wd = P.next_wbase + P.boffw[tile] + P.wposw[pl] + wofs;  // level-relative
            const uint64_t rs = ring_wrap(P.nbase + wd, P.rcap);
            P.noff[out] = wd;
#pragma unroll
            for (int w = 0; w < CCW; w++) P.next[ring_wrap(rs + (uint32_t)w, P.rcap)] = pk[w];
            // the parent's sorted ids merged with the added ones (sorted here: BecomeCandidate adds
            // its VoteReqs in peer order), written a word at a time, the last half-word padded
            uint32_t add[4] = {sb.w & 0xFFFFu, sb.w >> 16, sc.x & 0xFFFFu, sc.x >> 16};
#pragma unroll
            for (int a = 0; a < S::NADD; a++)
#pragma unroll
                for (int b = 0; b + 1 < S::NADD - a; b++)
                    if ((uint32_t)(b + 1) < nadd && add[b + 1] < add[b]) {
                        const uint32_t x = add[b];
                        add[b] = add[b + 1];
                        add[b + 1] = x;
                    }
            const uint64_t pid = ring_wrap(start + CCW, P.rcap), oid = ring_wrap(rs + CCW, P.rcap);
            uint32_t kk = 0, a = 0, word = 0, pw = 0;
            const uint32_t tot_ids = nm + nadd;
            for (uint32_t o = 0; o < tot_ids; o++) {
                uint32_t next_add = 0xFFFFFFFFu;
#pragma unroll
                for (int b = 0; b < S::NADD; b++) next_add = (uint32_t)b == a ? add[b] : next_add;
                if (kk < nm && (kk & 1u) == 0u) pw = ring_word(P.front, pid, kk >> 1, P.rcap);
                const uint32_t pv = (pw >> ((kk & 1u) * 16u)) & 0xFFFFu;
                uint32_t id;
                if (a < nadd && (kk >= nm || next_add < pv)) {
                    id = next_add;
                    a++;
                } else {
                    id = pv;
                    kk++;
                }
                if (o & 1u) P.next[ring_wrap(oid + (o >> 1), P.rcap)] = word | (id << 16);
                else word = id;
            }
            if (tot_ids & 1u) P.next[ring_wrap(oid + (tot_ids >> 1), P.rcap)] = word;
            const uint32_t key = sb.z & 0xFFFFu;
            if (P.route) {
                // sharded round: the trace entry travels with the record to the state's next-level owner
                const uint64_t pref = P.gid_parent_base + p;
                P.xside[out] = make_uint4((uint32_t)pref, (uint32_t)(pref >> 32), key, size);
            } else {
                const uint64_t gid = P.gid_next_base + out;
                P.par[gid - P.trace_base] = P.gid_parent_base + p;
                P.pslot[gid - P.trace_base] = (uint16_t)key;
            }
            int which = 0;
            const MsgView mv{P.front, pid, P.rcap, nm, sb.w, sc.x, nadd, P.t.info};
            const int iv = check_invs<N, V>(c, P.inv_order, &which, mv);
            if (iv != 1) {
                const unsigned long long ek = ((((unsigned long long)p << 16) | key) << 8) | (unsigned long long)which;
                atomicMin(&P.err[iv == 0 ? ERR_INV : ERR_EVAL], ek);
            }
        }
    }
}

// a block's counts into one global counter: one atomic per block, not per wave (every block of a
// launch adds into the same word -- per-wave atomics on it cost ~0.7 s over Raft.cfg's rounds)
__device__ __forceinline__ void block_count_add(uint32_t mine, unsigned long long *total) {
    __shared__ uint32_t blk;
    if (threadIdx.x == 0) blk = 0u;
    __syncthreads();
    for (int d = 32; d >= 1; d >>= 1) mine += __shfl_xor(mine, d, 64);
    if ((threadIdx.x & 63) == 0 && mine) atomicAdd(&blk, mine);
    __syncthreads();
    if (threadIdx.x == 0 && blk) atomicAdd(total, (unsigned long long)blk);
}

// ---- split chunk / sharded round commit, records staged in LDS ------------------------------------
// k_commit_split gives each winner a lane but leaves it a chain of dependent global loads: its parent's
// record offset, then the core words, then -- one load per two ids -- the parent's message ids while it
// merges them with the ids its action added.  Here a 256-thread block takes 64 parents with winners
// (plist) at a time and copies their records into LDS first (a lane per record word); then, in rounds
// of whole parents of at most 256 successor slots, a lane per slot finds the winners (lslot == LS_WIN),
// stages each one's row in LDS and lists it on its parent, and a lane per winner -- dense, whatever the
// parents' successor counts -- takes its ordinal and word offset among its parent's winners from that
// list (TLC order = slot order), rebuilds the state from the LDS core, writes the record (core, then the
// parent's ids merged with the added ones, read from LDS), its trace entry (or sidecar) and checks the
// INVARIANTs.  Outputs are k_commit_split's, bit for bit; k_commit_finish follows.
// FUSE: a fused level's commit (device loop, chunks below the split size; k_commit's outputs): PB
// consecutive parents at a time, those without winners skipped, the level from the control block, and
// the last block to arrive finishes the level (finish_level).
template <int N, int V, int MR, int MX, bool FUSE, int PB>
__global__ __launch_bounds__(XB_THREADS) void k_commit_items(KParams P) {
    using S = Spec<N, V, MR>;
    using Lo = Layout<N, V>;
    constexpr int NT = XB_THREADS, CCW = S::CCW, RECW = S::RECW_MAX, SW4 = S::SW4;
    static_assert(MX <= NT, "a parent's successor slots fit one round");
    static_assert(PB >= 2 && PB <= 64 && (PB & (PB - 1)) == 0, "parents per batch: a power of two, a lane of wave 0 each");
    __shared__ uint32_t sRec[PB * RECW];        // the batch's parent records
    __shared__ uint32_t sOff[PB + 1];           // record offsets in sRec (exclusive scan of record words)
    __shared__ uint32_t sSl[PB + 1];            // successor slots: exclusive scan of cnt
    __shared__ uint32_t sPl[PB];                // chunk-local parent index
    __shared__ uint32_t sHo[PB];                // its first successor slot (dense split chunk: P.hoff; else pl * MX)
    __shared__ uint32_t sOut[PB];               // next-level index of the parent's first winner (chunk-relative)
    __shared__ uint32_t sWd[PB];                // ... and its record's first word (chunk-relative)
    __shared__ uint64_t sRs[PB];                // its record's first word in the ring
    __shared__ uint32_t sWc[PB];                // the round's winners per parent
    __shared__ uint32_t sWl[NT];                // per parent at its slots' round offset: (slot << 16) | record words
    __shared__ uint4 sSt[NT * SW4];             // the round's winners' staged rows, dense
    __shared__ uint32_t sWr[NT];                // ... and each one's parent | slot << 8
    __shared__ uint32_t sNW;
    __shared__ uint8_t sWj[FUSE ? 1 : PB * RECW];  // per record word of the batch: its parent
    __shared__ uint8_t sSj[FUSE ? 1 : PB * MX];    // per successor slot of the batch: its parent
    const int tid = threadIdx.x;
    uint32_t own_ins = 0;  // a split sharded round: its own winners this thread put into the seen set
    if constexpr (FUSE) {
#ifdef RMC_RACE_PROBE
        if (P.ctl) {  // the first block without a parent reads its block after the level advanced (k_commit)
            const LevelCtl *c = ctl_cur(P);
            const uint32_t lv = c->level;
            if (c->stop == CTL_RUN && (uint64_t)blockIdx.x == (c->cur_n + PB - 1) / PB) {
                race_wait(4000, [&] {
                    return __hip_atomic_load(&ctl_nxt(P)->level, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == lv;
                });
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            }
        }
#endif
        if (!level_args(P)) return;
    }
    // the parents visited: a split chunk's or sharded round's with winners (plist), a fused level's all
    const uint64_t nvis = FUSE ? P.p_end - P.p_begin : P.sum[SUM_NZ];
    const uint32_t nbat = (uint32_t)((nvis + PB - 1) / PB);
    for (uint64_t k0 = (uint64_t)blockIdx.x * PB; k0 < nvis; k0 += (uint64_t)gridDim.x * PB) {
        const uint32_t nb = (uint32_t)(nvis - k0 < (uint64_t)PB ? nvis - k0 : (uint64_t)PB);
        if (tid < 64) {  // wave 0: a lane per parent with winners
            uint32_t t = 0, words = 0;
            if ((uint32_t)tid < nb) {
                const uint32_t pl = FUSE ? (uint32_t)(k0 + tid) : P.plist[k0 + tid];
                const uint32_t tile = pl / WTILE;
                const bool has = !FUSE || P.wcnt[pl] != 0u;  // (a fused level: parents without winners copy nothing)
                t = has ? (P.hcnt ? P.hcnt : P.cnt)[pl] : 0u;  // (self-loops never win)
                t = t < (uint32_t)MX ? t : (uint32_t)MX;
                words = has ? (uint32_t)CCW + ((P.pnm[pl] + 1u) >> 1) : 0u;
                sPl[tid] = pl;
                sRs[tid] = words ? ring_wrap(P.fbase + P.foff[P.p_begin + pl], P.rcap) : 0ull;
                sHo[tid] = P.hoff ? P.hoff[pl] : pl * (uint32_t)MX;
                sOut[tid] = P.boff[tile] + P.wpos[pl];
                sWd[tid] = P.boffw[tile] + P.wposw[pl];
                sWc[tid] = 0u;
            }
            uint32_t ts, tw;
            const uint32_t xs = wave_excl_scan(t, tid, &ts), xw = wave_excl_scan(words, tid, &tw);
            if ((uint32_t)tid < nb) { sSl[tid] = xs; sOff[tid] = xw; }
            if (tid == 0) { sSl[nb] = ts; sOff[nb] = tw; sNW = 0u; }
            // each record word's and each successor slot's parent (the copy and the rounds: no search; a fused
            // level's 16-parent batches search -- the notes cost configs[1] 5 %, profiles/r06_ab_commit_parents.txt)
            if constexpr (!FUSE) {
                for (uint32_t k = 0; k < words; k++) sWj[xw + k] = (uint8_t)tid;
                for (uint32_t k = 0; k < t; k++) sSj[xs + k] = (uint8_t)tid;
            }
        }
        __syncthreads();
        // the records, a lane per word (its parent noted by wave 0, whose ring start wave 0 read once), RC words
        // per lane in flight at once (a fused batch of 16 parents is one pass of the block: RC = 1)
        constexpr int RC = FUSE ? 1 : 4;
        const uint32_t tw = sOff[nb];
        for (uint32_t w0 = (uint32_t)tid; w0 < tw; w0 += RC * NT) {
            uint32_t v[RC];
#pragma unroll
            for (int k = 0; k < RC; k++) {
                const uint32_t w = w0 + k * NT;
                if (w < tw) {
                    uint32_t j = 0;
                    if constexpr (FUSE) {
#pragma unroll
                        for (uint32_t st = PB / 2; st; st >>= 1) j = (j + st < nb && sOff[j + st] <= w) ? j + st : j;
                    } else {
                        j = sWj[w];
                    }
                    v[k] = ring_word(P.front, sRs[j], w - sOff[j], P.rcap);
                }
            }
#pragma unroll
            for (int k = 0; k < RC; k++)
                if (w0 + k * NT < tw) sRec[w0 + k * NT] = v[k];
        }
        __syncthreads();
        for (uint32_t a = 0; a < nb;) {
            const uint32_t sbase = sSl[a];
            uint32_t b = a;  // parents a .. b - 1: at most NT slots
#pragma unroll
            for (uint32_t st = PB; st; st >>= 1) b = (b + st <= nb && sSl[b + st] <= sbase + NT) ? b + st : b;
            b = b > a ? b : a + 1;  // (a parent's slots always fit a round: MX <= NT)
            const uint32_t nS = sSl[b] - sbase < (uint32_t)NT ? sSl[b] - sbase : (uint32_t)NT;
            // (a) a lane per slot: the winners, staged and listed on their parent
            if ((uint32_t)tid < nS) {
                const uint32_t i = sbase + (uint32_t)tid;
                uint32_t j = a;
                if constexpr (FUSE) {
#pragma unroll
                    for (uint32_t st = PB / 2; st; st >>= 1) j = (j + st < b && sSl[j + st] <= i) ? j + st : j;
                } else {
                    j = sSj[i];
                }
                const uint32_t r = i - sSl[j];
                const uint64_t q = (uint64_t)sPl[j] * MX + r, sq = (uint64_t)sHo[j] + r;  // TLC's order, the slot
                // the verdict (LS_WIN: k_insert_winners', an owner's), or -- no insert pass -- the election word; a
                // split sharded round's own candidates (their slot in the round's owner table) are decided here
                const uint32_t g = P.lslot[sq];
                const bool own = P.route && P.OT && g < LS_WIN;  // (a table slot; LS_WIN < LS_ELECT < LS_SEEN)
                const bool win = own ? owner_same(P.OT[g].k, owner_key(P.ot_round + 1u, owner_order(P.gblk + sPl[j], r, 0u)))
                               : (P.route || (P.split & 4)) ? g == LS_WIN
                                                            : (g < LS_ELECT && elect_q(P.ET[g].k) == (uint32_t)q);
                if (own) P.lslot[sq] = win ? LS_WIN : LS_SEEN;  // (the verdict, as k_local_flags leaves it: error counts)
                if (win) {
                    const uint4 *src = P.score + sq * (uint64_t)SW4;
                    uint4 st4[SW4];
#pragma unroll
                    for (int x = 0; x < SW4; x++) st4[x] = src[x];
                    const uint32_t w = atomicAdd(&sNW, 1u);
#pragma unroll
                    for (int x = 0; x < SW4; x++) sSt[w * SW4 + x] = st4[x];
                    sWr[w] = j | (r << 8) | (own ? 0x10000u : 0u);
                    const uint32_t words = (uint32_t)CCW + ((P.pnm[sPl[j]] + (st4[1].z >> 16) + 1u) >> 1);
                    sWl[(sSl[j] - sbase) + atomicAdd(&sWc[j], 1u)] = (r << 16) | words;
                }
            }
            __syncthreads();
            // (b) a lane per winner
            if ((uint32_t)tid < sNW) {
                const uint32_t e = sWr[tid], j = e & 0xFFu, r = (e >> 8) & 0xFFu;
                const uint32_t lb = sSl[j] - sbase, wc = sWc[j];
                uint32_t ord = 0, wofs = 0;
                for (uint32_t x = 0; x < wc; x++) {
                    const uint32_t l = sWl[lb + x];
                    if ((l >> 16) < r) { ord++; wofs += l & 0xFFFFu; }
                }
                const uint4 sa = sSt[tid * SW4], sb = sSt[tid * SW4 + 1];
                const uint4 sc = SW4 > 2 ? sSt[tid * SW4 + 2] : make_uint4(0u, 0u, 0u, 0u);
                const uint32_t *rec = sRec + sOff[j];
                uint32_t pk[CCW], pc[Lo::NW], c[Lo::NW];
#pragma unroll
                for (int w = 0; w < CCW; w++) pk[w] = rec[w];
                decode_core<N, V>(pk, pc);
                unstage_core<N, V>(pc, sa, sb, c);
                encode_core<N, V>(c, pk);
                const uint32_t nm = (pc[Lo::W_MISC] >> 16) & 0xFFu, nadd = sb.z >> 16;
                const uint32_t size = (uint32_t)CCW + ((nm + nadd + 1u) >> 1);
                const uint32_t pl = sPl[j];
                const uint64_t p = P.p_begin + pl;
                const uint64_t out = P.next_base + sOut[j] + ord;
                if ((!P.route && !(P.split & 2)) || (e & 0x10000u)) {  // (no insert pass; a sharded round's own winner)
                    seen_insert(P.seen, P.fp[(uint64_t)sHo[j] + r]);
                    own_ins++;
                }
                const uint64_t wd = P.next_wbase + sWd[j] + wofs;  // level-relative
                const uint64_t rs = ring_wrap(P.nbase + wd, P.rcap);
                P.noff[out] = wd;
#pragma unroll
                for (int w = 0; w < CCW; w++) P.next[ring_wrap(rs + (uint32_t)w, P.rcap)] = pk[w];
                // the parent's sorted ids (LDS) merged with the added ones (sorted here: BecomeCandidate
                // adds its VoteReqs in peer order), written a word at a time, the last half-word padded
                uint32_t add[4] = {sb.w & 0xFFFFu, sb.w >> 16, sc.x & 0xFFFFu, sc.x >> 16};
#pragma unroll
                for (int x = 0; x < S::NADD; x++)
#pragma unroll
                    for (int y = 0; y + 1 < S::NADD - x; y++)
                        if ((uint32_t)(y + 1) < nadd && add[y + 1] < add[y]) {
                            const uint32_t t = add[y];
                            add[y] = add[y + 1];
                            add[y + 1] = t;
                        }
                const uint16_t *pid = reinterpret_cast<const uint16_t *>(rec + CCW);
                const uint64_t oid = ring_wrap(rs + CCW, P.rcap);
                uint32_t kk = 0, ai = 0, word = 0;
                const uint32_t tot_ids = nm + nadd;
                for (uint32_t o = 0; o < tot_ids; o++) {
                    uint32_t next_add = 0xFFFFFFFFu;
#pragma unroll
                    for (int y = 0; y < S::NADD; y++) next_add = (uint32_t)y == ai ? add[y] : next_add;
                    const uint32_t pv = kk < nm ? (uint32_t)pid[kk] : 0xFFFFFFFFu;
                    uint32_t id;
                    if (ai < nadd && next_add < pv) {
                        id = next_add;
                        ai++;
                    } else {
                        id = pv;
                        kk++;
                    }
                    if (o & 1u) P.next[ring_wrap(oid + (o >> 1), P.rcap)] = word | (id << 16);
                    else word = id;
                }
                if (tot_ids & 1u) P.next[ring_wrap(oid + (tot_ids >> 1), P.rcap)] = word;
                const uint32_t key = sb.z & 0xFFFFu;
                if (P.route) {
                    // sharded round: the trace entry travels with the record to the state's next-level owner
                    const uint64_t pref = P.gid_parent_base + p;
                    P.xside[out] = make_uint4((uint32_t)pref, (uint32_t)(pref >> 32), key, size);
                } else {
                    const uint64_t gid = P.gid_next_base + out;
                    P.par[gid - P.trace_base] = P.gid_parent_base + p;
                    P.pslot[gid - P.trace_base] = (uint16_t)key;
                }
                int which = 0;
                // (only NoAllCommit, tla:451-481, reads the message set: the ring's copy of the parent's ids)
                const uint64_t mids = (P.inv_mask & 32u) ? ring_wrap(ring_wrap(P.fbase + P.foff[p], P.rcap) + CCW, P.rcap) : 0;
                const MsgView mv{P.front, mids, P.rcap, nm, sb.w, sc.x, nadd, P.t.info};
                const int iv = check_invs<N, V>(c, P.inv_order, &which, mv);
                if (iv != 1) {
                    const unsigned long long ek = ((((unsigned long long)p << 16) | key) << 8) | (unsigned long long)which;
                    atomicMin(&P.err[iv == 0 ? ERR_INV : ERR_EVAL], ek);
                }
            }
            __syncthreads();
            if (tid == 0) sNW = 0u;
            if ((uint32_t)tid < b - a) sWc[a + tid] = 0u;  // (parents of this round only: already zero beyond)
            __syncthreads();
            a = b;
        }
    }
    if constexpr (!FUSE) {
        if (P.route) block_count_add(own_ins, &P.sum[SUM_INS_COMMIT]);
    }
    if constexpr (FUSE) {
        // the last block to arrive finishes the level (k_commit's protocol); every wave's atomics and
        // stores are complete before its block's arrival (the barrier)
        __syncthreads();
        const uint32_t nbb = nbat < gridDim.x ? (nbat ? nbat : 1u) : gridDim.x;
        if (tid < 64 && last_commit_block(P.ctick, nbb)) finish_level<MX, S::RECW_MAX>(P);
    }
}

// the chunk summary after k_commit_split (one wave): finish_level
template <int MX, int RECW_MAX>
__global__ __launch_bounds__(64) void k_commit_finish(KParams P) {
    finish_level<MX, RECW_MAX>(P);
}


// ---- sharded round: the owner's election (W > 1, and the one-rank rehearsal) -------------------

// Owner's own successors (fingerprint owner == self), a lane each: they bid in the round's table
// straight from the expansion's slots -- no item through the exchange -- and the slot (or LS_SEEN)
// waits in lslot for k_local_flags.  Successors other shards own are marked LS_ELECT and left to
// the exchange (their verdicts arrive by k_scatter_win).
template <int MX, int SW4>
__global__ __launch_bounds__(256) void k_local_elect(KParams P, Seen seen, ESlot *OT,
                                                     uint64_t mask, uint32_t round, uint32_t W, uint32_t self,
                                                     uint64_t g0) {
    const OwnerLocal loc{P.wacc, g0, P.p_end - P.p_begin};
    each_successor<MX>(P, [&](uint64_t pl, uint32_t r, uint64_t q) {  // (sharded rounds: the sparse layout)
        const ulonglong2 f = P.fp[q];
        if (fp_owner(f, W) != self) {
            P.lslot[q] = LS_ELECT;
            return;
        }
        if (seen_contains(seen, f)) {
            P.lslot[q] = LS_SEEN;
            return;
        }
        const uint32_t nadd = P.score[q * (uint64_t)SW4 + 1].z >> 16;
        P.lslot[q] = owner_bid(OT, mask, round + 1u, f, owner_order(g0 + pl, r, (nadd + (P.pnm[pl] & 1u) + 1u) >> 1), loc);
    });
}

// ... once every bid of the round is in (the received ones too), a round below the split size (a split
// round's commit decides its own candidates itself): the verdict in lslot (LS_WIN / LS_SEEN) and each
// winner into the seen set, *inserted counting them (the bids counted the winners on their parents).
template <int MX>
__global__ __launch_bounds__(256) void k_local_flags(KParams P, Seen seen, const ESlot *OT, uint32_t round,
                                                     uint32_t W, uint32_t self, uint64_t g0,
                                                     unsigned long long *inserted) {
    const uint32_t tag = round + 1u;
    uint32_t mine = 0;
    each_successor<MX>(P, [&](uint64_t pl, uint32_t r, uint64_t q) {  // (sharded rounds: the sparse layout)
        const uint32_t g = P.lslot[q];
        if (g == LS_ELECT || g == LS_SEEN) return;  // another shard's, or seen: nothing to decide
        const bool w = owner_same(OT[g].k, owner_key(tag, owner_order(g0 + pl, r, 0u)));
        P.lslot[q] = w ? LS_WIN : LS_SEEN;
        if (w) {
            seen_insert(seen, P.fp[q]);
            mine++;
        }
    });
    block_count_add(mine, inserted);
}

static inline unsigned grid_for(uint64_t n) {
    const uint64_t cap = 256ull * RMC_GRID_PER_CU;  // one-wave blocks per CU (default 32) on 256 CUs
    return (unsigned)(n < cap ? (n ? n : 1) : cap);
}

template <int N, int V, int MR, bool BFV = false>
struct Launch {
    static constexpr int MX = Spec<N, V, MR>::MAXS + (BFV ? Spec<N, V, MR>::MCAP : 0);
    static size_t bm_bytes(const KParams &P) { return (size_t)P.t.bmw * 4; }
    static void single(const KParams &P, hipStream_t s) {
        hipLaunchKernelGGL((k_expand<N, V, MR, M_SINGLE, BFV>), dim3(1), dim3(64), bm_bytes(P), s, P);
    }
    static void fused(const KParams &P, hipStream_t s) {
        if (!P.route) {  // a block per XF_PARENTS parents, fingerprints and election in the same launch
            const uint64_t nbat = (P.p_end - P.p_begin + XF_PARENTS - 1) / XF_PARENTS;
            hipLaunchKernelGGL((k_expand_items<N, V, MR, BFV, true, XF_PARENTS>), dim3((unsigned)(nbat < 8192 ? (nbat ? nbat : 1) : 8192)),
                               dim3(XB_THREADS), 0, s, P);
            return;
        }
        // a sharded round below the split size: a wave per parent, fingerprints routed to their owners
        hipLaunchKernelGGL((k_expand<N, V, MR, M_FUSED, BFV>), dim3(grid_for(P.p_end - P.p_begin)), dim3(64),
                           bm_bytes(P), s, P);
    }
    static void split(const KParams &P, hipStream_t s) {
        const uint64_t nbat = (P.p_end - P.p_begin + XB_PARENTS - 1) / XB_PARENTS;
        hipLaunchKernelGGL((k_expand_items<N, V, MR, BFV, false, XB_PARENTS>), dim3((unsigned)(nbat < 2048 ? (nbat ? nbat : 1) : 2048)),
                           dim3(items_threads<N, V, MR, false>()), 0, s, P);
    }
    static void hash_probe(const KParams &P, uint64_t np, hipStream_t s) {
        const uint64_t blocks = (np + 255) / 256;  // four one-group waves per block
        hipLaunchKernelGGL((k_hash_probe<N, V, MR, MX>), dim3(blocks ? (unsigned)(blocks < 16384ull ? blocks : 16384ull) : 1u),
                           dim3(256), 0, s, P);
    }
    static void insert(const KParams &P, uint64_t np, hipStream_t s) {
        const uint64_t blocks = (np + 255) / 256;
        hipLaunchKernelGGL((k_insert_winners<MX>), dim3(blocks ? (unsigned)(blocks < 16384ull ? blocks : 16384ull) : 1u),
                           dim3(256), 0, s, P);
    }
    static void wincount(const KParams &P, uint64_t np, hipStream_t s) {
        const uint64_t tiles = (np + WTILE - 1) / WTILE;
        hipLaunchKernelGGL((k_wincount<N, V, MR>), dim3(tiles ? (unsigned)tiles : 1u), dim3(1024), 0, s, P);
    }
    static void commit(const KParams &P, hipStream_t s) {
        if constexpr (MX <= XB_THREADS) {
            if (!P.route && !P.split && !P.plist) {  // a block per 16 parents, records in LDS
                const uint64_t nbat = (P.p_end - P.p_begin + XC_PARENTS - 1) / XC_PARENTS;
                hipLaunchKernelGGL((k_commit_items<N, V, MR, MX, true, XC_PARENTS>),
                                   dim3((unsigned)(nbat < 8192 ? (nbat ? nbat : 1) : 8192)), dim3(XB_THREADS), 0, s, P);
                return;
            }
        }
        hipLaunchKernelGGL((k_commit<N, V, MR, BFV>), dim3(grid_for(P.p_end - P.p_begin)), dim3(64), 0, s, P);
    }
    static void commit_split(const KParams &P, uint64_t np, hipStream_t s) {
        const uint64_t blocks = (np + 255) / 256;  // a wave per 64 parents with winners (at most np of them)
        if constexpr (MX <= XB_THREADS) {
            {  // a block per 64 parents with winners, records in LDS
                const uint64_t nbat = (np + 63) / 64;
                hipLaunchKernelGGL((k_commit_items<N, V, MR, MX, false, 64>), dim3((unsigned)(nbat < 2048 ? (nbat ? nbat : 1) : 2048)),
                                   dim3(XB_THREADS), 0, s, P);
                hipLaunchKernelGGL((k_commit_finish<MX, Spec<N, V, MR>::RECW_MAX>), dim3(1), dim3(64), 0, s, P);
                return;
            }
        }
        hipLaunchKernelGGL((k_commit_split<N, V, MR, MX>), dim3(blocks ? (unsigned)(blocks < 16384ull ? blocks : 16384ull) : 1u),
                           dim3(256), 0, s, P);
        hipLaunchKernelGGL((k_commit_finish<MX, Spec<N, V, MR>::RECW_MAX>), dim3(1), dim3(64), 0, s, P);
    }
    static void local_elect(const KParams &P, uint64_t np, Seen seen, ESlot *OT,
                            uint64_t mask, uint32_t round, uint32_t W, uint32_t self, uint64_t g0, hipStream_t s) {
        const uint64_t blocks = (np + 255) / 256;  // a wave per 64 parents (each_successor)
        hipLaunchKernelGGL((k_local_elect<MX, Spec<N, V, MR>::SW4>), dim3(blocks ? (unsigned)(blocks < 16384ull ? blocks : 16384ull) : 1u),
                           dim3(256), 0, s, P, seen, OT, mask, round, W, self, g0);
    }
    static void local_flags(const KParams &P, uint64_t np, Seen seen, const ESlot *OT, uint32_t round,
                            uint32_t W, uint32_t self, uint64_t g0, unsigned long long *inserted, hipStream_t s) {
        const uint64_t blocks = (np + 255) / 256;
        hipLaunchKernelGGL((k_local_flags<MX>),
                           dim3(blocks ? (unsigned)(blocks < 16384ull ? blocks : 16384ull) : 1u), dim3(256), 0, s, P,
                           seen, OT, round, W, self, g0, inserted);
    }
    static void fps(const KParams &P, uint64_t n, hipStream_t s) {
        hipLaunchKernelGGL((k_fp_states<N, V, MR>), dim3(grid_for(n)), dim3(64), 0, s, P, n);
    }
    static void invs(const KParams &P, uint64_t n, int32_t *out, hipStream_t s) {
        hipLaunchKernelGGL((k_inv_states<N, V, MR>), dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, P, n, out);
    }
    static void enc(const uint32_t *c, uint32_t *o) { encode_core<N, V>(c, o); }
    static void dec(const uint32_t *w, uint32_t *c) { decode_core<N, V>(w, c); }
};

template <int N, int V, int MR, bool BFV>
static void fill(KernelSet *ks) {
    using S = Spec<N, V, MR>;
    ks->N = N; ks->V = V; ks->MR = MR; ks->MCAP = S::MCAP; ks->CCW = S::CCW; ks->RECW_MAX = S::RECW_MAX;
    ks->maxsucc = S::MAXS + (BFV ? S::MCAP : 0);
    ks->single = &Launch<N, V, MR, BFV>::single;
    ks->fused = &Launch<N, V, MR, BFV>::fused;
    ks->split = &Launch<N, V, MR, BFV>::split;
    ks->hash_probe = &Launch<N, V, MR, BFV>::hash_probe;
    ks->ctxw = ctx_words<N, V>();
    ks->insert = &Launch<N, V, MR, BFV>::insert;
    ks->wincount = &Launch<N, V, MR, BFV>::wincount;
    ks->commit = &Launch<N, V, MR, BFV>::commit;
    ks->commit_split = &Launch<N, V, MR, BFV>::commit_split;
    ks->local_elect = &Launch<N, V, MR, BFV>::local_elect;
    ks->local_flags = &Launch<N, V, MR, BFV>::local_flags;
    ks->fp_states = &Launch<N, V, MR>::fps;
    ks->inv_states = &Launch<N, V, MR>::invs;
    ks->encode = &Launch<N, V, MR>::enc;
    ks->decode = &Launch<N, V, MR>::dec;
}

bool get_kernels(int N, int V, int msg_cap, bool become_follower, KernelSet *ks) {
    const int MR = msg_cap <= 64 ? 1 : 2;
#define RMC_CASE(n, v, mr)                                        \
    if (N == n && V == v && MR == mr) {                           \
        if (become_follower) fill<n, v, mr, true>(ks);            \
        else fill<n, v, mr, false>(ks);                           \
        return true;                                              \
    }
    RMC_CASE(2, 1, 1) RMC_CASE(2, 2, 1)
    RMC_CASE(3, 1, 1) RMC_CASE(3, 2, 1) RMC_CASE(3, 3, 1)
    RMC_CASE(3, 1, 2) RMC_CASE(3, 2, 2)
    RMC_CASE(4, 1, 2) RMC_CASE(4, 2, 2)
    RMC_CASE(5, 1, 2) RMC_CASE(5, 2, 2)
#undef RMC_CASE
    return false;
}

__global__ __launch_bounds__(256) void k_rehash(const ulonglong2 *__restrict__ Told, uint64_t old_cap, Seen dst) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < old_cap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const ulonglong2 e = Told[i];
        if (e.x) seen_insert(dst, e);
    }
}

__global__ __launch_bounds__(256) void k_insert(const ulonglong2 *__restrict__ fp, uint64_t n, Seen seen) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        seen_insert(seen, fp[i]);
}

__global__ __launch_bounds__(256) void k_rebase(const uint64_t *__restrict__ in, uint64_t n, uint64_t sub,
                                                uint64_t *__restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = in[i] - sub;
}

static inline unsigned grid256(uint64_t n) {
    const uint64_t b = (n + 255) / 256, cap = 256ull * 16ull;
    return (unsigned)(b < cap ? (b ? b : 1) : cap);
}

__global__ __launch_bounds__(256) void k_eslot_clear(ESlot *t, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        t[i] = ESlot{0ull, 0ull, ~0ull, 0ull};
}
void launch_eslot_clear(ESlot *t, uint64_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_eslot_clear, dim3(grid256(n)), dim3(256), 0, s, t, n);
}

void launch_rehash(const ulonglong2 *Told, uint64_t old_cap, Seen dst, hipStream_t s) {
    hipLaunchKernelGGL(k_rehash, dim3(grid256(old_cap)), dim3(256), 0, s, Told, old_cap, dst);
}
// the device loop's control blocks (both of the pair) and the fused expansion's self-loop counters
// (each level's finish_level re-arms them for the next)
__global__ __launch_bounds__(64) void k_set_ctl(LevelCtl *dst, int n, LevelCtl v, unsigned long long *sum) {
    if (threadIdx.x < (unsigned)n) dst[threadIdx.x] = v;
    if (threadIdx.x == 0 && sum) {
#pragma unroll
        for (int k = 0; k < SELF_STRIPES; k++) sum[SUM_SELF_STRIPE + SELF_STRIDE * k] = 0ull;  // (fused self-loops)
    }
}
void launch_set_ctl(LevelCtl *dst, int n, const LevelCtl &v, unsigned long long *gen, hipStream_t s) {
    hipLaunchKernelGGL(k_set_ctl, dim3(1), dim3(64), 0, s, dst, n, v, gen);
}

__global__ __launch_bounds__(64) void k_init_level(uint32_t *ring, const uint32_t *rec, uint32_t words,
                                                   uint64_t *off, const ulonglong2 *fp, Seen seen) {
    for (uint32_t i = threadIdx.x; i < words; i += 64) ring[i] = rec[i];
    if (threadIdx.x == 0) {
        off[0] = 0;
        seen_insert(seen, fp[0]);
    }
}
void launch_init_level(uint32_t *ring, const uint32_t *rec, uint32_t words, uint64_t *off,
                       const ulonglong2 *fp, Seen seen, hipStream_t s) {
    hipLaunchKernelGGL(k_init_level, dim3(1), dim3(64), 0, s, ring, rec, words, off, fp, seen);
}

void launch_insert_fps(const ulonglong2 *fp, uint64_t n, Seen seen, hipStream_t s) {
    hipLaunchKernelGGL(k_insert, dim3(grid256(n)), dim3(256), 0, s, fp, n, seen);
}
void launch_nzlist(const KParams &P, uint64_t np, hipStream_t s) {
    const uint64_t tiles = (np + WTILE - 1) / WTILE;
    hipLaunchKernelGGL(k_nzlist, dim3(tiles ? (unsigned)tiles : 1u), dim3(1024), 0, s, P);
}
void launch_rebase(const uint64_t *in, uint64_t n, uint64_t sub, uint64_t *out, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_rebase, dim3(grid256(n)), dim3(256), 0, s, in, n, sub, out);
}

// ---- sharded round (W > 1) -------------------------------------------------------------------
// Source: successors of the round's parents (sparse slots q = pl * maxsucc + r, r < cnt[pl]) per
// owner, into ocnt[W] (zeroed by the caller).
__global__ __launch_bounds__(256) void k_route_count(const ulonglong2 *__restrict__ fp, const uint32_t *__restrict__ cnt,
                                                     uint64_t np, uint32_t maxsucc, uint32_t W, uint32_t *__restrict__ ocnt) {
    __shared__ uint32_t h[64];
    if (threadIdx.x < 64) h[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t pl = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; pl < np; pl += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t t = cnt[pl];
        for (uint32_t r = 0; r < t; r++) atomicAdd(&h[fp_owner(fp[pl * maxsucc + r], W)], 1u);
    }
    __syncthreads();
    if (threadIdx.x < W && h[threadIdx.x]) atomicAdd(&ocnt[threadIdx.x], h[threadIdx.x]);
}

// Source: every successor another shard owns to that owner's segment of the send buffer
// (cursor[o] = the segment's next free item, preset to its start): {fingerprint, global key =
// (parent's global index in the level << 10) | rank among its successors (< 1024, checked at
// create)} -- the key orders the level's successors as TLC generates them -- and perm[item] = its
// slot q, for the owner's verdict to come back to.  Successors the source owns itself stay where
// they are: k_local_elect / k_local_flags decide them.
__global__ __launch_bounds__(256) void k_route_place(const ulonglong2 *__restrict__ fp, const uint32_t *__restrict__ cnt,
                                                     uint64_t np, uint32_t maxsucc, uint32_t W, uint32_t *__restrict__ cursor,
                                                     uint64_t g0, XItem *__restrict__ items, uint32_t *__restrict__ perm,
                                                     uint32_t self) {
    __shared__ uint32_t h[64], base[64];
    for (uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x; t0 < np; t0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t pl = t0 + threadIdx.x;
        if (threadIdx.x < 64) h[threadIdx.x] = 0;
        __syncthreads();
        const uint32_t t = pl < np ? cnt[pl] : 0u;
        for (uint32_t r = 0; r < t; r++) {
            const uint32_t o = fp_owner(fp[pl * maxsucc + r], W);
            if (o != self) atomicAdd(&h[o], 1u);
        }
        __syncthreads();
        if (threadIdx.x < W) {
            const uint32_t c = h[threadIdx.x];
            base[threadIdx.x] = c ? atomicAdd(&cursor[threadIdx.x], c) : 0u;
            h[threadIdx.x] = 0;
        }
        __syncthreads();
        for (uint32_t r = 0; r < t; r++) {
            const uint64_t q = pl * maxsucc + r;
            const ulonglong2 f = fp[q];
            const uint32_t o = fp_owner(f, W);
            if (o == self) continue;
            const uint32_t pos = base[o] + atomicAdd(&h[o], 1u);
            items[pos] = XItem{f.x, f.y, owner_order(g0 + pl, r, 0u)};
            perm[pos] = (uint32_t)q;
        }
        __syncthreads();
    }
}

// Owner: the received successors of the round -- bids (owner_bid) by k_owner_elect, and by the
// owner's own successors in k_local_elect.
__global__ __launch_bounds__(256) void k_owner_elect(const XItem *__restrict__ it, uint64_t R, Seen seen,
                                                     ESlot *OT, uint64_t mask, uint32_t round,
                                                     uint32_t *__restrict__ rslot, OwnerLocal loc) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < R; i += (uint64_t)gridDim.x * blockDim.x) {
        const XItem e = it[i];
        const ulonglong2 f = make_ulonglong2(e.x, e.y);
        rslot[i] = seen_contains(seen, f) ? LS_SEEN : owner_bid(OT, mask, round + 1u, f, e.key, loc);
    }
}

// Owner: verdicts (1 = the fingerprint's first successor in TLC order among all shards, not seen
// before); each winner goes into the seen set, *inserted counts them.
__global__ __launch_bounds__(256) void k_owner_flags(const XItem *__restrict__ it, uint64_t R,
                                                     const uint32_t *__restrict__ rslot,
                                                     const ESlot *__restrict__ OT, uint32_t round, Seen seen,
                                                     uint32_t *__restrict__ flag, unsigned long long *inserted) {
    const uint32_t tag = round + 1u;
    uint32_t mine = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < R; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t g = rslot[i];
        const XItem e = it[i];
        const bool w = g != LS_SEEN && owner_same(OT[g].k, owner_key(tag, e.key));
        flag[i] = w ? 1u : 0u;
        if (w) {
            seen_insert(seen, make_ulonglong2(e.x, e.y));
            mine++;
        }
    }
    block_count_add(mine, inserted);
}

// Source: the owners' verdicts back on the successor slots (lslot = LS_WIN / LS_SEEN), and each
// winner counted on its parent as the fused election would (wacc = winners | extra words << 12).
__global__ __launch_bounds__(256) void k_scatter_win(const uint32_t *__restrict__ perm, const uint32_t *__restrict__ flag,
                                                     uint64_t G, const uint4 *__restrict__ score, uint32_t sw4,
                                                     const uint32_t *__restrict__ pnm, uint32_t maxsucc,
                                                     uint32_t *__restrict__ lslot, uint32_t *__restrict__ wacc) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < G; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t q = perm[i];
        const bool w = flag[i] != 0;
        lslot[q] = w ? LS_WIN : LS_SEEN;
        if (w) {
            const uint32_t pl = q / maxsucc;
            const uint32_t nadd = score[(uint64_t)q * sw4 + 1].z >> 16;
            const uint32_t e = (nadd + (pnm[pl] & 1u) + 1u) >> 1;
            atomicAdd(&wacc[pl], 1u + (e << 12));
        }
    }
}

// Owner: record sizes of received winners (sidecar .w), for the offset scan
__global__ __launch_bounds__(256) void k_side_sizes(const uint4 *__restrict__ side, uint64_t n, uint32_t *__restrict__ sz) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        sz[i] = side[i].w;
}

// Owner: received winners appended to the next level -- level-relative record offsets
// (rel0 + scanned sizes) and trace entries (parent's global id, slot key)
__global__ __launch_bounds__(256) void k_accept_side(const uint4 *__restrict__ side, const uint32_t *__restrict__ off,
                                                     uint64_t n, uint64_t rel0, uint64_t *__restrict__ noff,
                                                     uint64_t *__restrict__ par, uint16_t *__restrict__ pslot) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 e = side[i];
        noff[i] = rel0 + off[i];
        par[i] = (uint64_t)e.x | ((uint64_t)e.y << 32);
        pslot[i] = (uint16_t)e.z;
    }
}

__global__ void k_owner_of(const ulonglong2 *__restrict__ fp, uint32_t W, uint32_t *out) {
    if (threadIdx.x == 0) out[0] = fp_owner(fp[0], W);
}

void launch_route_count(const ulonglong2 *fp, const uint32_t *cnt, uint64_t np, uint32_t maxsucc, uint32_t W,
                        uint32_t *ocnt, hipStream_t s) {
    if (np) hipLaunchKernelGGL(k_route_count, dim3(grid256(np)), dim3(256), 0, s, fp, cnt, np, maxsucc, W, ocnt);
}
void launch_route_place(const ulonglong2 *fp, const uint32_t *cnt, uint64_t np, uint32_t maxsucc, uint32_t W,
                        uint32_t *cursor, uint64_t g0, XItem *items, uint32_t *perm, uint32_t self, hipStream_t s) {
    if (np)
        hipLaunchKernelGGL(k_route_place, dim3(grid256(np)), dim3(256), 0, s, fp, cnt, np, maxsucc, W, cursor, g0, items,
                           perm, self);
}
void launch_owner_elect(const XItem *it, uint64_t R, Seen seen, ESlot *OT, uint64_t mask,
                        uint32_t round, uint32_t *rslot, uint32_t *wacc, uint64_t g0, uint64_t np, hipStream_t s) {
    if (R)
        hipLaunchKernelGGL(k_owner_elect, dim3(grid256(R)), dim3(256), 0, s, it, R, seen, OT, mask, round, rslot,
                           OwnerLocal{wacc, g0, np});
}
void launch_owner_flags(const XItem *it, uint64_t R, const uint32_t *rslot, const ESlot *OT, uint32_t round,
                        Seen seen, uint32_t *flag, unsigned long long *inserted, hipStream_t s) {
    if (R)
        hipLaunchKernelGGL(k_owner_flags, dim3(grid256(R)), dim3(256), 0, s, it, R, rslot, OT, round, seen, flag,
                           inserted);
}
void launch_scatter_win(const uint32_t *perm, const uint32_t *flag, uint64_t G, const uint4 *score, uint32_t sw4,
                        const uint32_t *pnm, uint32_t maxsucc, uint32_t *lslot, uint32_t *wacc, hipStream_t s) {
    if (G)
        hipLaunchKernelGGL(k_scatter_win, dim3(grid256(G)), dim3(256), 0, s, perm, flag, G, score, sw4, pnm, maxsucc,
                           lslot, wacc);
}
void launch_side_sizes(const uint4 *side, uint64_t n, uint32_t *sz, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_side_sizes, dim3(grid256(n)), dim3(256), 0, s, side, n, sz);
}
void launch_accept_side(const uint4 *side, const uint32_t *off, uint64_t n, uint64_t rel0, uint64_t *noff,
                        uint64_t *par, uint16_t *pslot, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_accept_side, dim3(grid256(n)), dim3(256), 0, s, side, off, n, rel0, noff, par, pslot);
}
__global__ __launch_bounds__(256) void k_seen_query(const ulonglong2 *__restrict__ fp, uint64_t n, Seen seen, uint32_t W,
                                                    uint32_t self, uint8_t *__restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (W <= 1 || fp_owner(fp[i], W) == self) out[i] = seen_contains(seen, fp[i]) ? 1u : 0u;
}
void launch_seen_query(const ulonglong2 *fp, uint64_t n, Seen seen, uint32_t W, uint32_t self, uint8_t *out,
                       hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_seen_query, dim3(grid256(n)), dim3(256), 0, s, fp, n, seen, W, self, out);
}
void launch_owner_of(const ulonglong2 *fp, uint32_t W, uint32_t *out, hipStream_t s) {
    hipLaunchKernelGGL(k_owner_of, dim3(1), dim3(64), 0, s, fp, W, out);
}

}  // namespace rmc
