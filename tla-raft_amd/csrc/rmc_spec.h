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
// Next's disjuncts in textual order (tla:418-430): the enumeration order TLC uses.
enum Act : uint32_t { BC = 0, UT, RV, BL, CR, LAE, FAE, FRE, HAR, LCC, RS, NACT };
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
// Symmetry+VIEW fingerprint (tla:21,38): fp(s) = min over permutations pi of the
// 128-bit structured hash H(pi(view(s))), with
//   H_f(w) = sum_k Z_f(k, U_w[k]) + sum_{k != l} Z_f(k, l, P_w[k][l])     (mod 2^64, f = 0,1)
// where U_w[k] is the exact packed own-state of server k (votedFor as None/self/
// other, term, role, commitIndex, log, matchIndex[k][k], nextIndex[k][k]) and
// P_w[k][l] combines matchIndex[k][l], nextIndex[k][l], votedFor[k] = l and the sum
// of per-message hashes of msgs with src = k, dst = l.  Every term is a strong mix
// of (position, content), so H is a Zobrist-style hash of the whole view; all
// states in one orbit produce the same multiset {H(pi(s))} and hence the same min.
RMC_HD uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
RMC_HD uint64_t splitmix(uint64_t &x) {
    x += 0x9e3779b97f4a7c15ULL;
    return mix64(x);
}

constexpr uint64_t SEED_SERVER = 0x5ee1d5e5a7c0ffeeULL;
constexpr uint64_t SEED_PAIR = 0x9a1b2c3d4e5f6071ULL;
constexpr uint64_t SEED_MSG = 0x0123456789abcdefULL;
constexpr uint64_t PAIR_K0 = 0x9e3779b97f4a7c15ULL, PAIR_K1 = 0xc2b2ae3d27d4eb4fULL;

// per-message hash pair of everything but src/dst (those are positions in the pair sums),
// from the message's info word: the host's table (Universe::gmsg) and the expansion kernel's
// added messages use this one definition
struct MsgHash { uint64_t x, y; };
RMC_HD MsgHash msg_hash(uint32_t info) {
    const uint64_t body = (uint64_t)info & ~0xFCull;
    return {mix64(SEED_MSG ^ mix64(body * 0x9e3779b97f4a7c15ULL + 1)),
            mix64((SEED_MSG + 0x632be59bd9b4e019ULL) ^ mix64(body * 0xc2b2ae3d27d4eb4fULL + 7))};
}

// slot key (16 bit): server<<11 | action<<7 | witness -- increasing in TLC order
RMC_HD uint32_t slot_key(uint32_t s, uint32_t a, uint32_t w) { return (s << 11) | (a << 7) | w; }
RMC_HD uint32_t key_server(uint32_t k) { return k >> 11; }
RMC_HD uint32_t key_action(uint32_t k) { return (k >> 7) & 15u; }
RMC_HD uint32_t key_witness(uint32_t k) { return k & 127u; }
constexpr uint32_t KEY_NONE = 0xFFFFu;

}  // namespace rmc
