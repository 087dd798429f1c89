// rmc_plan.h -- host bookkeeping of the sharded BFS round (pure C++, no HIP): who sends what to
// whom, at which offsets, and which shard must grow a receive buffer first.
//
// The sharded level exchanges three all-to-all-v payloads
// per round: successors to their fingerprint's owner, the owner's verdicts back, and the winners'
// records to the shards owning their next-level indices.  Every shard's counts are gathered on
// every rank as one W x K matrix (one row per shard: its counts to each destination, then its
// receive capacities and its failure code), so every rank derives the same offsets, the same
// decision to grow a receive buffer before the payload moves, and the same failure -- no rank can
// be left waiting in a send or receive its peer never posts.  tests/plan_test.cpp checks these
// functions at W = 1..8 against a direct simulation of the exchange.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace rmc {

// cnt[s * W + d] = items shard s sends to shard d (a row-major W x W block of the gathered matrix)
struct XPlan {
    std::vector<uint64_t> send_cnt, send_off;  // per destination d (send_off: prefix over d)
    std::vector<uint64_t> recv_cnt, recv_off;  // per source s (recv_off: prefix over s, W + 1 entries)
    uint64_t send_total = 0, recv_total = 0;
};

// shard r's plan from the gathered counts; `stride` = the row width of the gathered matrix
inline XPlan make_plan(const uint64_t *cnt, int W, int stride, int r) {
    XPlan p;
    p.send_cnt.assign(W, 0);
    p.send_off.assign(W + 1, 0);
    p.recv_cnt.assign(W, 0);
    p.recv_off.assign(W + 1, 0);
    for (int d = 0; d < W; d++) {
        p.send_cnt[d] = cnt[(size_t)r * stride + d];
        p.send_off[d + 1] = p.send_off[d] + p.send_cnt[d];
    }
    for (int s = 0; s < W; s++) {
        p.recv_cnt[s] = cnt[(size_t)s * stride + r];
        p.recv_off[s + 1] = p.recv_off[s] + p.recv_cnt[s];
    }
    p.send_total = p.send_off[W];
    p.recv_total = p.recv_off[W];
    return p;
}

// the reverse exchange (verdicts back to the sources): what r received comes back from r
inline XPlan reverse_plan(const XPlan &p) {
    XPlan q;
    q.send_cnt = p.recv_cnt;
    q.send_off = p.recv_off;
    q.recv_cnt = p.send_cnt;
    q.recv_off = p.send_off;
    q.send_total = p.recv_total;
    q.recv_total = p.send_total;
    return q;
}

// One point-to-point transfer of an exchange, in items: the RCCL branch posts, for its peer, a
// send of (src_off, n) and a receive of (dst_off, n); the virtual branch copies src_off of shard
// `from` to dst_off of shard `to`.
struct Xfer {
    int from, to;
    uint64_t src_off, dst_off, n;
};

// every transfer of an exchange among W shards with these plans (plans[r] = shard r's), in the
// order the virtual branch copies them (source-major)
inline std::vector<Xfer> transfers(const std::vector<XPlan> &plans) {
    const int W = (int)plans.size();
    std::vector<Xfer> x;
    for (int s = 0; s < W; s++)
        for (int d = 0; d < W; d++) {
            const uint64_t n = plans[s].send_cnt[d];
            if (n) x.push_back({s, d, plans[s].send_off[d], plans[d].recv_off[s], n});
        }
    return x;
}

// Block-cyclic next level: global index g of a level lives on shard
// (g / B) % W at local index (g / (B W)) B + g % B.  A source holding the winners with global
// next-level indices [x0, x0 + w) sends each contiguous piece to its owner, in order.
struct Piece {
    int d;               // destination shard
    uint64_t i0, i1;     // winner range of the source (0-based within its w winners)
};

inline std::vector<Piece> route_pieces(uint64_t x0, uint64_t w, uint64_t B, int W) {
    std::vector<Piece> pcs;
    for (uint64_t x = x0; x < x0 + w;) {
        const uint64_t b = x / B, y = std::min(x0 + w, (b + 1) * B);
        pcs.push_back({(int)(b % (uint64_t)W), x - x0, y - x0});
        x = y;
    }
    return pcs;
}

// Items per destination and the send layout of a source's pieces: if no destination owns two of
// them, the pieces already lie grouped (send_off[d] = the piece's start); otherwise the source
// regroups them by destination, in order, and send_off is the grouped copy's layout.
struct PieceLayout {
    std::vector<uint64_t> cnt, off;
    bool regroup = false;
};

inline PieceLayout piece_layout(const std::vector<Piece> &pcs, int W) {
    PieceLayout L;
    L.cnt.assign(W, 0);
    L.off.assign(W, 0);
    std::vector<int> seen(W, 0);
    for (const Piece &p : pcs) {
        L.regroup |= seen[p.d]++ > 0;
        L.cnt[p.d] += p.i1 - p.i0;
    }
    if (!L.regroup) {
        for (const Piece &p : pcs) L.off[p.d] = p.i0;
    } else {
        uint64_t at = 0;
        for (int d = 0; d < W; d++) { L.off[d] = at; at += L.cnt[d]; }
    }
    return L;
}

// Shards whose receive buffer must grow before the payload moves: need[r] + 1 > cap[r].  Every rank
// computes the same list from the gathered matrix, so all of them take the extra agreement step.
inline std::vector<int> must_grow(const std::vector<uint64_t> &need, const std::vector<uint64_t> &cap) {
    std::vector<int> g;
    for (size_t r = 0; r < need.size(); r++)
        if (need[r] + 1 > cap[r]) g.push_back((int)r);
    return g;
}

}  // namespace rmc
