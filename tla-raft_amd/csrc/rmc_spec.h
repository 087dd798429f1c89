// rmc_spec.h -- Raft.tla compiled ahead of time onto a fixed-width packed state.
//
// Shared by the device kernels (rmc_kernels.hip) and the host engine.  Every
// definition cites the spec text it encodes: /root/reference/Raft.tla (tla:N),
// Raft.cfg (cfg:N).  Nothing here is generic TLA+: the 12 variables (tla:26,29,34)
// and 4 message record shapes (tla:117-125,149,254-263,283-290,310-317) are
// hard-wired.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RMC_HD __host__ __device__ __forceinline__
#else
#define RMC_HD inline
#endif

namespace rmc {

// ---- enumerations ---------------------------------------------------------------
enum Role : uint32_t { FOL = 0, CAN = 1, LEA = 2 };            // Follower, Candidate, Leader (tla:14)
enum MType : uint32_t { VREQ = 0, VRESP = 1, AREQ = 2, ARESP = 3 }; // tla:8
// Next's disjuncts in textual order (tla:418-430): the enumeration order TLC uses.  BF =
// BecomeFollower, in Next only in the tla:420 variant (between UpdateTerm and ResponseVote); its
// id follows the never-enabled FollowerAppendEntry's (11) so the ids of Raft.tla's actions stay put.
enum Act : uint32_t { BC = 0, UT, RV, BL, CR, LAE, FAE, FRE, HAR, LCC, RS, NACT, FAPP = NACT, BF };
constexpr uint32_t VF_NONE = 15;   // votedFor = None (tla:94)
constexpr int MAXN = 5;
constexpr int MAXV = 3;

// ---- packed core layout (32-bit words; 4-bit nibbles) -----------------------------
//   W_VF   votedFor[i]       nibble i (VF_NONE = None)           tla:26
//   W_CT   currentTerm[i]    nibble i                            tla:26
//   W_ROLE role[i]           nibble i                            tla:29
//   W_CI   commitIndex[i]    nibble i                            tla:29
//   W_LL   Len(logs[i])      nibble i                            tla:26
//   W_LOG+i  logs[i][x], x = 2..V+1: byte x-2 = term | val<<4     (logs[i][1] = [0,None] implicit, tla:97)
//   W_MI+i matchIndex[i][j]  nibble j                            tla:29
//   W_NI+i nextIndex[i][j]   nibble j                            tla:29
//   W_PEND pendingResponse[i][j] bit i*N+j                       tla:34
//   W_MISC electionCount [3:0], restartCount [7:4], valSent[v] bit 8+v (1 = FALSE, 0 = None),
//          |msgs| [23:16]                                       tla:34
// A state record in HBM is CW core words followed by MCAP u16 message ids, sorted
// ascending; ids are assigned in TLC's value order, so the sorted id list is the
// order in which TLC enumerates \E m \in msgs.
template <int N, int V>
struct Layout {
    static constexpr int W_VF = 0, W_CT = 1, W_ROLE = 2, W_CI = 3, W_LL = 4;
    static constexpr int W_LOG = 5, W_MI = 5 + N, W_NI = 5 + 2 * N, W_PEND = 5 + 3 * N, W_MISC = 6 + 3 * N;
    static constexpr int NW = 7 + 3 * N;                 // core words
    static constexpr int CW = (NW + 3) / 4 * 4;          // core words padded to 16 B
};

RMC_HD uint32_t nib(uint32_t w, int i) { return (w >> (4 * i)) & 15u; }
RMC_HD uint32_t setnib(uint32_t w, int i, uint32_t v) { return (w & ~(15u << (4 * i))) | ((v & 15u) << (4 * i)); }

// ---- storage codec: the nibble core above, bit-packed for HBM ------------------------------
// The kernels compute on the nibble layout (constant-position fields in registers); frontier
// records and the successor staging store the same fields with the widths the spec's domains
// need (tla:8-16, cfg:3-4: terms <= MaxElection <= 7, indices <= |Vals| + 2, restarts <= 15,
// |msgs| <= 255).  Raft.cfg's core (3 servers, 2 values) is exactly 128 bits -- 16 B instead
// of the nibble layout's 64 B.  A record in HBM is CCW packed core words followed by |msgs|
// u16 message ids (TLC order), padded to a whole word: CCW + ceil(|msgs| / 2) words.
constexpr int bits_for(int maxval) { return maxval <= 0 ? 0 : 1 + bits_for(maxval >> 1); }

// bits of the packed core of (N, V) -- Codec<N, V>::BITS, for the host at run time
constexpr int codec_bits(int N, int V) {
    return N * (bits_for(N) + 3 + 2 + 2 * bits_for(V + 1)) + N * V * (3 + bits_for(V - 1)) +
           N * N * (bits_for(V + 1) + bits_for(V + 2)) + N * N + 3 + 4 + V + 8;
}

template <int N, int V>
struct Codec {
    static constexpr int B_VF = bits_for(N);                  // 0 = None, k + 1 = server k
    static constexpr int B_CT = 3;                            // currentTerm 0..MaxElection (<= 7)
    static constexpr int B_RO = 2;                            // Follower / Candidate / Leader
    static constexpr int B_IX = bits_for(V + 1);              // commitIndex, Len(logs), matchIndex: 1..V+1
    static constexpr int B_NI = bits_for(V + 2);              // nextIndex 2..V+2
    static constexpr int B_VAL = bits_for(V - 1);             // a log entry's value 0..V-1
    static constexpr int B_ENT = 3 + B_VAL;                   // log entry: term | val
    static constexpr int BITS = N * (B_VF + B_CT + B_RO + 2 * B_IX) + N * V * B_ENT + N * N * (B_IX + B_NI) +
                                N * N + 3 + 4 + V + 8;
    static constexpr int CCW = (BITS + 31) / 32;              // packed core words
    static_assert(BITS == codec_bits(N, V), "codec_bits must follow the field widths above");
};

RMC_HD void bits_put(uint32_t *w, int pos, uint32_t v, int b) {
    if (b == 0) return;
    const int i = pos >> 5, o = pos & 31;
    w[i] |= v << o;
    if (o + b > 32) w[i + 1] |= v >> (32 - o);
}
RMC_HD uint32_t bits_get(const uint32_t *w, int pos, int b) {
    if (b == 0) return 0u;
    const int i = pos >> 5, o = pos & 31;
    uint32_t v = w[i] >> o;
    if (o + b > 32) v |= w[i + 1] << (32 - o);
    return b >= 32 ? v : (v & ((1u << b) - 1u));
}

// nibble core c[Layout::NW] -> packed words o[Codec::CCW] (every position is a compile-time
// constant once the loops unroll)
template <int N, int V>
RMC_HD void encode_core(const uint32_t *c, uint32_t *o) {
    using L = Layout<N, V>;
    using C = Codec<N, V>;
#pragma unroll
    for (int k = 0; k < C::CCW; k++) o[k] = 0u;
    int pos = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
        const uint32_t vf = nib(c[L::W_VF], i);
        bits_put(o, pos, vf == VF_NONE ? 0u : vf + 1u, C::B_VF); pos += C::B_VF;
        bits_put(o, pos, nib(c[L::W_CT], i), C::B_CT); pos += C::B_CT;
        bits_put(o, pos, nib(c[L::W_ROLE], i), C::B_RO); pos += C::B_RO;
        bits_put(o, pos, nib(c[L::W_CI], i), C::B_IX); pos += C::B_IX;
        bits_put(o, pos, nib(c[L::W_LL], i), C::B_IX); pos += C::B_IX;
#pragma unroll
        for (int x = 0; x < V; x++) {
            const uint32_t b = (c[L::W_LOG + i] >> (8 * x)) & 0xFFu;
            bits_put(o, pos, (b & 7u) | ((b >> 4) << 3), C::B_ENT); pos += C::B_ENT;
        }
    }
#pragma unroll
    for (int i = 0; i < N; i++)
#pragma unroll
        for (int j = 0; j < N; j++) {
            bits_put(o, pos, nib(c[L::W_MI + i], j), C::B_IX); pos += C::B_IX;
            bits_put(o, pos, nib(c[L::W_NI + i], j), C::B_NI); pos += C::B_NI;
        }
    bits_put(o, pos, c[L::W_PEND] & ((1u << (N * N)) - 1u), N * N); pos += N * N;
    const uint32_t misc = c[L::W_MISC];
    bits_put(o, pos, misc & 7u, 3); pos += 3;
    bits_put(o, pos, (misc >> 4) & 15u, 4); pos += 4;
    bits_put(o, pos, (misc >> 8) & ((1u << V) - 1u), V); pos += V;
    bits_put(o, pos, (misc >> 16) & 0xFFu, 8);
}

template <int N, int V>
RMC_HD void decode_core(const uint32_t *w, uint32_t *c) {
    using L = Layout<N, V>;
    using C = Codec<N, V>;
#pragma unroll
    for (int k = 0; k < L::NW; k++) c[k] = 0u;
    int pos = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
        const uint32_t vf = bits_get(w, pos, C::B_VF); pos += C::B_VF;
        c[L::W_VF] |= (vf == 0u ? VF_NONE : vf - 1u) << (4 * i);
        c[L::W_CT] |= bits_get(w, pos, C::B_CT) << (4 * i); pos += C::B_CT;
        c[L::W_ROLE] |= bits_get(w, pos, C::B_RO) << (4 * i); pos += C::B_RO;
        c[L::W_CI] |= bits_get(w, pos, C::B_IX) << (4 * i); pos += C::B_IX;
        c[L::W_LL] |= bits_get(w, pos, C::B_IX) << (4 * i); pos += C::B_IX;
#pragma unroll
        for (int x = 0; x < V; x++) {
            const uint32_t e = bits_get(w, pos, C::B_ENT); pos += C::B_ENT;
            c[L::W_LOG + i] |= ((e & 7u) | ((e >> 3) << 4)) << (8 * x);
        }
    }
#pragma unroll
    for (int i = 0; i < N; i++)
#pragma unroll
        for (int j = 0; j < N; j++) {
            c[L::W_MI + i] |= bits_get(w, pos, C::B_IX) << (4 * j); pos += C::B_IX;
            c[L::W_NI + i] |= bits_get(w, pos, C::B_NI) << (4 * j); pos += C::B_NI;
        }
    c[L::W_PEND] = bits_get(w, pos, N * N); pos += N * N;
    uint32_t misc = bits_get(w, pos, 3); pos += 3;
    misc |= bits_get(w, pos, 4) << 4; pos += 4;
    misc |= bits_get(w, pos, V) << 8; pos += V;
    misc |= bits_get(w, pos, 8) << 16;
    c[L::W_MISC] = misc;
}

// |msgs| of a packed core (its last 8 bits)
template <int N, int V>
RMC_HD uint32_t core_nm(const uint32_t *w) { return bits_get(w, Codec<N, V>::BITS - 8, 8); }

// ring-buffer position: x < 2 * cap
RMC_HD uint64_t ring_wrap(uint64_t x, uint64_t cap) { return x >= cap ? x - cap : x; }

// ---- message info word ------------------------------------------------------------
// [1:0] type  [4:2] src  [7:5] dst  [11:8] term  [15:12] x1  [19:16] x2  [23:20] x3
// [24] entry present  [28:25] entry term  [31:29] entry val
//   VoteReq    x1 = lastLogIndex, x2 = lastLogTerm                (tla:117-125)
//   VoteResp   -                                                  (tla:149)
//   AppendReq  x1 = prevLogIndex, x2 = prevLogTerm, x3 = leaderCommit, entries = <<entry>> or <<>> (tla:254-263)
//   AppendResp x1 = prevLogIndex, x2 = succ                       (tla:283-290, 310-317)
RMC_HD uint32_t minfo(uint32_t type, uint32_t src, uint32_t dst, uint32_t term, uint32_t x1, uint32_t x2,
                      uint32_t x3, uint32_t ent, uint32_t et, uint32_t ev) {
    return type | (src << 2) | (dst << 5) | (term << 8) | (x1 << 12) | (x2 << 16) | (x3 << 20) | (ent << 24) |
           (et << 25) | (ev << 29);
}
RMC_HD uint32_t mi_type(uint32_t m) { return m & 3u; }
RMC_HD uint32_t mi_src(uint32_t m) { return (m >> 2) & 7u; }
RMC_HD uint32_t mi_dst(uint32_t m) { return (m >> 5) & 7u; }
RMC_HD uint32_t mi_term(uint32_t m) { return (m >> 8) & 15u; }
RMC_HD uint32_t mi_x1(uint32_t m) { return (m >> 12) & 15u; }
RMC_HD uint32_t mi_x2(uint32_t m) { return (m >> 16) & 15u; }
RMC_HD uint32_t mi_x3(uint32_t m) { return (m >> 20) & 15u; }
RMC_HD uint32_t mi_ent(uint32_t m) { return (m >> 24) & 1u; }
RMC_HD uint32_t mi_et(uint32_t m) { return (m >> 25) & 15u; }
RMC_HD uint32_t mi_ev(uint32_t m) { return (m >> 29) & 7u; }

// ---- natural (mixed-radix) index of a message ------------------------------------------
// The static universe of records the actions can build.  nat -> id (TLC order) is a
// table built on the host (Universe below).
struct Dims {
    int n, V, E;
    uint32_t nVQ, nVP, nAQ, nAP;  // sizes per type
    uint32_t bVP, bAQ, bAP;       // bases
    uint32_t total;
};

RMC_HD Dims make_dims(int n, int V, int E) {
    Dims d;
    d.n = n; d.V = V; d.E = E;
    uint32_t P = (uint32_t)(n * n), e = (uint32_t)E, v1 = (uint32_t)V + 1;
    d.nVQ = P * e * v1 * (e + 1);
    d.nVP = P * e;
    d.nAQ = P * e * v1 * (e + 1) * (1 + e * (uint32_t)V) * v1;
    d.nAP = P * e * v1 * 2;
    d.bVP = d.nVQ;
    d.bAQ = d.bVP + d.nVP;
    d.bAP = d.bAQ + d.nAQ;
    d.total = d.bAP + d.nAP;
    return d;
}

// term >= 1 for every message (terms of sent messages are currentTerm values after
// at least one election, tla:111,121).
RMC_HD uint32_t nat_vreq(const Dims &d, uint32_t src, uint32_t dst, uint32_t term, uint32_t lli, uint32_t llt) {
    return ((((src * d.n + dst) * d.E + (term - 1)) * (d.V + 1) + (lli - 1)) * (d.E + 1)) + llt;
}
RMC_HD uint32_t nat_vresp(const Dims &d, uint32_t src, uint32_t dst, uint32_t term) {
    return d.bVP + (src * d.n + dst) * d.E + (term - 1);
}
RMC_HD uint32_t nat_areq(const Dims &d, uint32_t src, uint32_t dst, uint32_t term, uint32_t pli, uint32_t plt,
                         uint32_t ent, uint32_t et, uint32_t ev, uint32_t lc) {
    uint32_t e = ent ? 1u + (et - 1) * d.V + ev : 0u;
    return d.bAQ +
           ((((((src * d.n + dst) * d.E + (term - 1)) * (d.V + 1) + (pli - 1)) * (d.E + 1) + plt) *
                 (1 + d.E * d.V) +
             e) *
                (d.V + 1) +
            (lc - 1));
}
RMC_HD uint32_t nat_aresp(const Dims &d, uint32_t src, uint32_t dst, uint32_t term, uint32_t pli, uint32_t succ) {
    return d.bAP + ((((src * d.n + dst) * d.E + (term - 1)) * (d.V + 1) + (pli - 1)) * 2 + succ);
}

// ---- hashing --------------------------------------------------------------------------
// Symmetry+VIEW fingerprint (tla:21,38).  Per server k, its exact own-state U[k] (votedFor as
// None/self/other, term, role, commitIndex, log, matchIndex[k][k], nextIndex[k][k]) and, per peer l,
// its pair state X_f[k][l] (matchIndex[k][l], nextIndex[k][l], votedFor[k] = l, and the sum of the
// per-message hashes of msgs with src = k, dst = l) -- server-relative, no server ids.  Each is
// mixed once into a content matrix
//   C_f[k][k] = mix64(U[k] ^ CK_U_f),   C_f[k][l] = mix64(X_f[k][l] ^ CK_X_f)        (f = 0, 1)
// and a permutation pi, which puts server k at position pi(k), is priced by position constants:
//   H_f(pi) = sum_{k,l} C_f[k][l] * K_f[pi(k)][pi(l)]       (mod 2^64, K_f odd, host seeds)
// so a state costs its N^2 content mixes once (a successor: its acting server's row) and each
// permutation only N^2 multiply-adds.  The fingerprint is the minimum of (H_1, H_0) over the
// permutations consistent with the servers' signatures sig[k] = sum_l C_1[k][l] (sorted; ties
// enumerated): states of one orbit have permuted signatures, so they take the minimum over the
// same multiset of H values -- a class invariant; distinct contents sum to distinct values except
// with probability ~2^-64 per half.
RMC_HD uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
RMC_HD uint64_t splitmix(uint64_t &x) {
    x += 0x9e3779b97f4a7c15ULL;
    return mix64(x);
}

constexpr uint64_t SEED_PAIR = 0x9a1b2c3d4e5f6071ULL;  // position constants (host)
constexpr uint64_t SEED_MSG = 0x0123456789abcdefULL;
constexpr uint64_t PAIR_K0 = 0x9e3779b97f4a7c15ULL, PAIR_K1 = 0xc2b2ae3d27d4eb4fULL;
constexpr uint64_t CK_U0 = 0x2545f4914f6cdd1dULL, CK_U1 = 0x8cb92ba72f3d8dd7ULL;
constexpr uint64_t CK_X0 = 0x9fb21c651e98df25ULL, CK_X1 = 0xd6e8feb86659fd93ULL;
RMC_HD uint64_t cmix_own(uint64_t u, int f) { return mix64(u ^ (f ? CK_U1 : CK_U0)); }
RMC_HD uint64_t cmix_pair(uint64_t x, int f) { return mix64(x ^ (f ? CK_X1 : CK_X0)); }
// position constants: K_f[a][b] = seeds[f * MAXN * MAXN + a * MAXN + b] (odd)
constexpr int SEEDS_PER_F = MAXN * MAXN;

// per-message hash pair of everything but src/dst (those are positions in the pair sums),
// from the message's info word: the host's table (Universe::gmsg) and the expansion kernel's
// added messages use this one definition
struct MsgHash { uint64_t x, y; };
// One mix64 per family: body * K + seed is a bijection of the 32-bit body and mix64 a bijection, so
// each family is a well-mixed injective image of the body (an outer mix64 over a seeded inner one
// added nothing but 2 of the 4 multiply-heavy mixes the expansion pays per added message).
RMC_HD MsgHash msg_hash(uint32_t info) {
    const uint64_t body = (uint64_t)info & ~0xFCull;
    return {mix64(body * 0x9e3779b97f4a7c15ULL + SEED_MSG),
            mix64(body * 0xc2b2ae3d27d4eb4fULL + (SEED_MSG + 0x632be59bd9b4e019ULL))};
}

// slot key (16 bit): server<<11 | position<<7 | witness -- increasing in TLC order; the position
// of an action is its place in Next (BF right after UT)
RMC_HD uint32_t act_pos(uint32_t a) { return a <= UT ? a : (a == BF ? 2u : a + 1u); }
RMC_HD uint32_t pos_act(uint32_t p) { return p <= 1u ? p : (p == 2u ? (uint32_t)BF : p - 1u); }
RMC_HD uint32_t slot_key(uint32_t s, uint32_t a, uint32_t w) { return (s << 11) | (act_pos(a) << 7) | w; }
RMC_HD uint32_t key_server(uint32_t k) { return k >> 11; }
RMC_HD uint32_t key_action(uint32_t k) { return pos_act((k >> 7) & 15u); }
RMC_HD uint32_t key_witness(uint32_t k) { return k & 127u; }
constexpr uint32_t KEY_NONE = 0xFFFFu;

}  // namespace rmc
