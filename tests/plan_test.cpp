// Host test of the sharded round's bookkeeping (tla-raft_amd/csrc/rmc_plan.h) at W = 1..8.
//
// The engine's RCCL branch posts, per peer, one send (send_off, send_cnt) and one receive
// (recv_off, recv_cnt) from its own plan; the virtual branch copies every transfer of all W plans.
// Both must move exactly the same bytes.  This program simulates the three payloads of a round on
// host arrays -- successors to their owners, verdicts back, winners to the owners of their
// block-cyclic next-level indices -- and checks, against direct definitions:
//   * the RCCL view of every rank equals the virtual transfer list (same offsets, same counts);
//   * every owner receives exactly the items sent to it, grouped by source in source order;
//   * the reverse plan brings every verdict back to the slot it answers;
//   * every winner lands on the shard (g / B) % W at the position the block-cyclic layout gives
//     it, in global order, whether the source sends its pieces in place or regrouped;
//   * must_grow names exactly the shards whose receive need reaches their capacity.
// Exit status 0 and "plan ok" on success.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "rmc_plan.h"

using namespace rmc;

static int fails = 0;
#define CHECK(c)                                                                     \
    do {                                                                             \
        if (!(c)) {                                                                  \
            if (fails++ < 20) std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
        }                                                                            \
    } while (0)

// one all-to-all-v with the virtual branch's copies; returns the receive buffers
static std::vector<std::vector<uint64_t>> run_virtual(const std::vector<XPlan> &P,
                                                      const std::vector<std::vector<uint64_t>> &send) {
    const int W = (int)P.size();
    std::vector<std::vector<uint64_t>> recv(W);
    for (int r = 0; r < W; r++) recv[r].assign(P[r].recv_total, ~0ull);
    for (const Xfer &x : transfers(P))
        for (uint64_t k = 0; k < x.n; k++) recv[x.to][x.dst_off + k] = send[x.from][x.src_off + k];
    return recv;
}

// the same exchange as the RCCL ranks post it: each rank's sends and receives from its own plan,
// matched by (sender, receiver) as the communicator matches them
static std::vector<std::vector<uint64_t>> run_rccl(const std::vector<XPlan> &P,
                                                   const std::vector<std::vector<uint64_t>> &send) {
    const int W = (int)P.size();
    std::vector<std::vector<uint64_t>> recv(W);
    for (int r = 0; r < W; r++) recv[r].assign(P[r].recv_total, ~0ull);
    for (int r = 0; r < W; r++)          // receiver
        for (int p = 0; p < W; p++) {    // its peer (the sender)
            const uint64_t nr = P[r].recv_cnt[p], ns = P[p].send_cnt[r];
            CHECK(nr == ns);             // a receive posted for every send, of the same size
            for (uint64_t k = 0; k < std::min(nr, ns); k++)
                recv[r][P[r].recv_off[p] + k] = send[p][P[p].send_off[r] + k];
        }
    return recv;
}

int main() {
    std::mt19937_64 rng(20261017);
    for (int W = 1; W <= 8; W++) {
        for (int trial = 0; trial < 60; trial++) {
            // ---- successors to their owners: a W x (W + 2) gathered matrix (counts, cap, fail) ----
            const int K = W + 2;
            std::vector<uint64_t> M((size_t)W * K, 0);
            std::vector<std::vector<uint64_t>> owner_of(W);  // per source, the owner of each item in send order
            for (int s = 0; s < W; s++) {
                for (int d = 0; d < W; d++) M[(size_t)s * K + d] = (trial % 7 == 0 && d == s) ? 0 : rng() % 40;
                M[(size_t)s * K + W] = rng() % 120;  // receive capacity
            }
            std::vector<XPlan> P(W);
            for (int r = 0; r < W; r++) P[r] = make_plan(M.data(), W, K, r);
            // send buffers: item = (source << 32) | index, grouped by owner in owner order
            std::vector<std::vector<uint64_t>> send(W);
            for (int s = 0; s < W; s++) {
                uint64_t idx = 0;
                for (int d = 0; d < W; d++) {
                    CHECK(P[s].send_off[d] == idx);
                    for (uint64_t k = 0; k < M[(size_t)s * K + d]; k++) send[s].push_back(((uint64_t)s << 32) | idx++);
                }
                CHECK(P[s].send_total == send[s].size());
            }
            const auto rv = run_virtual(P, send);
            const auto rr = run_rccl(P, send);
            CHECK(rv == rr);
            for (int o = 0; o < W; o++) {
                // grouped by source in source order, each group in the source's send order
                std::vector<uint64_t> exp;
                for (int s = 0; s < W; s++)
                    for (uint64_t k = 0; k < M[(size_t)s * K + o]; k++) exp.push_back(send[s][P[s].send_off[o] + k]);
                CHECK(rv[o] == exp);
            }
            // verdicts back: the owner answers item x with f(x); each source slot gets its own answer
            std::vector<XPlan> Q(W);
            for (int r = 0; r < W; r++) Q[r] = reverse_plan(P[r]);
            std::vector<std::vector<uint64_t>> ans(W);
            for (int o = 0; o < W; o++)
                for (uint64_t x : rv[o]) ans[o].push_back(x * 2654435761ull + 7);
            const auto back = run_virtual(Q, ans);
            CHECK(back == run_rccl(Q, ans));
            for (int s = 0; s < W; s++) {
                CHECK(back[s].size() == send[s].size());
                for (size_t i = 0; i < send[s].size() && i < back[s].size(); i++)
                    CHECK(back[s][i] == send[s][i] * 2654435761ull + 7);
            }
            // receive growth: exactly the shards whose need + 1 exceeds their capacity
            std::vector<uint64_t> need(W, 0), cap(W, 0);
            for (int o = 0; o < W; o++) {
                for (int t = 0; t < W; t++) need[o] += M[(size_t)t * K + o];
                cap[o] = M[(size_t)o * K + W];
                CHECK(need[o] == P[o].recv_total);
            }
            const std::vector<int> g = must_grow(need, cap);
            size_t gi = 0;
            for (int o = 0; o < W; o++) {
                const bool grows = need[o] + 1 > cap[o];
                if (grows) { CHECK(gi < g.size() && g[gi] == o); gi++; }
            }
            CHECK(gi == g.size());

            // ---- winners to the owners of their block-cyclic next-level indices ----
            const uint64_t Bk = 1 + rng() % 9;          // block size (chunk_parents)
            const uint64_t base = rng() % 50;            // winners of earlier rounds in the level
            std::vector<uint64_t> Aw(W + 1, base);       // global index range of each source's winners
            for (int s = 0; s < W; s++) Aw[s + 1] = Aw[s] + (trial % 5 == 0 ? rng() % (3 * Bk * W + 1) : rng() % (Bk + 3));
            const int K2 = 2 * W + 3;
            std::vector<uint64_t> M2((size_t)W * K2, 0);
            std::vector<std::vector<uint64_t>> wsend(W), wwords(W);
            std::vector<PieceLayout> lay(W);
            std::vector<std::vector<uint64_t>> woff(W);
            for (int s = 0; s < W; s++) {
                const uint64_t x0 = Aw[s], w = Aw[s + 1] - Aw[s];
                const std::vector<Piece> pcs = route_pieces(x0, w, Bk, W);
                // pieces tile [0, w) in order, each inside one block
                uint64_t at = 0;
                for (const Piece &pe : pcs) {
                    CHECK(pe.i0 == at && pe.i1 > pe.i0);
                    CHECK((x0 + pe.i0) / Bk == (x0 + pe.i1 - 1) / Bk);
                    CHECK(pe.d == (int)(((x0 + pe.i0) / Bk) % (uint64_t)W));
                    at = pe.i1;
                }
                CHECK(at == w);
                lay[s] = piece_layout(pcs, W);
                // the outbox: winner i = global index x0 + i, record of (i % 3 + 1) words
                std::vector<uint64_t> rec_w(w), rec_off(w + 1, 0);
                for (uint64_t i = 0; i < w; i++) { rec_w[i] = i % 3 + 1; rec_off[i + 1] = rec_off[i] + rec_w[i]; }
                std::vector<uint64_t> side(w), words;
                for (uint64_t i = 0; i < w; i++) {
                    side[i] = x0 + i;
                    for (uint64_t k = 0; k < rec_w[i]; k++) words.push_back(((x0 + i) << 8) | k);
                }
                std::vector<uint64_t> wcnt(W, 0), wl(W, 0);
                for (const Piece &pe : pcs) wcnt[pe.d] += rec_off[pe.i1] - rec_off[pe.i0];
                if (!lay[s].regroup) {
                    for (const Piece &pe : pcs) wl[pe.d] = rec_off[pe.i0];
                    wsend[s] = side;
                    wwords[s] = words;
                } else {  // grouped copy by destination, pieces in order
                    uint64_t wat = 0;
                    for (int d = 0; d < W; d++) { wl[d] = wat; wat += wcnt[d]; }
                    for (int d = 0; d < W; d++)
                        for (const Piece &pe : pcs) {
                            if (pe.d != d) continue;
                            for (uint64_t i = pe.i0; i < pe.i1; i++) wsend[s].push_back(side[i]);
                            for (uint64_t k = rec_off[pe.i0]; k < rec_off[pe.i1]; k++) wwords[s].push_back(words[k]);
                        }
                    CHECK(wsend[s].size() == w && wwords[s].size() == words.size());
                }
                woff[s] = wl;
                for (int d = 0; d < W; d++) {
                    M2[(size_t)s * K2 + d] = lay[s].cnt[d];
                    M2[(size_t)s * K2 + W + d] = wcnt[d];
                }
            }
            std::vector<XPlan> PS(W), PW(W);
            for (int r = 0; r < W; r++) {
                PS[r] = make_plan(M2.data(), W, K2, r);
                PW[r] = make_plan(M2.data() + W, W, K2, r);
                for (int d = 0; d < W; d++) { PS[r].send_off[d] = lay[r].off[d]; PW[r].send_off[d] = woff[r][d]; }
            }
            const auto got = run_virtual(PS, wsend);
            const auto gotw = run_virtual(PW, wwords);
            CHECK(got == run_rccl(PS, wsend));
            CHECK(gotw == run_rccl(PW, wwords));
            for (int o = 0; o < W; o++) {
                // exactly this round's global indices owned by o, in increasing order (= its local order)
                std::vector<uint64_t> exp, expw;
                for (uint64_t x = Aw[0]; x < Aw[W]; x++)
                    if ((int)((x / Bk) % (uint64_t)W) == o) {
                        exp.push_back(x);
                        for (uint64_t k = 0; k < (x - Aw[std::upper_bound(Aw.begin(), Aw.end(), x) - Aw.begin() - 1]) % 3 + 1; k++)
                            expw.push_back((x << 8) | k);
                    }
                CHECK(got[o] == exp);
                CHECK(gotw[o] == expw);
                // and those local indices are consecutive in the block-cyclic layout
                for (size_t i = 1; i < exp.size(); i++) {
                    const uint64_t a = (exp[i - 1] / (Bk * W)) * Bk + exp[i - 1] % Bk;
                    const uint64_t b = (exp[i] / (Bk * W)) * Bk + exp[i] % Bk;
                    CHECK(b == a + 1);
                }
            }
        }
    }
    if (fails) {
        std::printf("%d failures\n", fails);
        return 1;
    }
    std::printf("plan ok\n");
    return 0;
}
