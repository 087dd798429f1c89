// rmc_engine.hip -- host orchestration of the level-synchronous GPU BFS behind the C-ABI.
//
// Replaces TLC's ModelChecker / Worker loop (run by myrun.sh:3) for Raft.tla:
//   * level L's states live in HBM as variable-length packed records (rmc_spec.h Codec: packed
//     core + sorted message ids) in a ring of 32-bit words, in TLC -workers 1 FIFO order, with a
//     level-relative word offset per state; level L+1 is written right behind level L, and the
//     space of the chunks of level L already expanded is reused once the ring is at its budget;
//   * a level is expanded in chunks of parents by three fused launches (expand + fingerprint +
//     seen-set probe + election + staging, winner count, commit);
//   * new states are appended to the next level in the order TLC would have enqueued them, so
//     discovery order (and therefore which concrete state represents a VIEW class, SURVEY
//     App. D.2) matches TLC with one worker;
//   * the seen set holds 128-bit fingerprints while small, then 64-bit words in a table sized
//     once from the memory budget (the probe run from the home slot carries the rest);
//   * every state's parent reference + slot key (the trace, TLC's states/ metadir) goes to host
//     memory chunk by chunk;
//   * the first error in TLC order (invariant / eval error / Assert / deadlock) stops the search
//     with TLC's counters at that point and a replayable trace.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include <fcntl.h>
#include <unistd.h>

#include "rmc.h"
#include "rmc_kernels.h"
#include "rmc_spec.h"

#ifdef RMC_WITH_RCCL
#include <rccl/rccl.h>
#endif

using namespace rmc;

namespace {

#define HIPCHK(x)                                                                                 \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) throw Fail(RMC_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct Fail {
    int code;
    std::string msg;
    Fail(int c, std::string m) : code(c), msg(std::move(m)) {}
};

// ---------------------------------------------------------------------------------------
// Message universe: every record the 11 actions can build, ordered as TLC orders
// values (record: field count, then sorted (name, value) pairs).
// ---------------------------------------------------------------------------------------
struct Universe {
    Dims d;
    std::vector<uint32_t> info;     // by id
    std::vector<uint16_t> nat2id;   // by natural index (0xFFFF = unused)
    std::vector<ulonglong2> gmsg;   // by id

    void build(int n, int V, int E) {
        d = make_dims(n, V, E);
        struct Item {
            std::array<int, 10> key;
            uint32_t nat, info;
        };
        std::vector<Item> items;
        items.reserve(d.total);
        for (int src = 0; src < n; src++)
            for (int dst = 0; dst < n; dst++)
                for (int term = 1; term <= E; term++) {
                    // VoteResp: 4 fields dst, src, term, type
                    items.push_back({{0, dst, src, term, 0, 0, 0, 0, 0, 0},
                                     nat_vresp(d, src, dst, term),
                                     minfo(VRESP, src, dst, term, 0, 0, 0, 0, 0, 0)});
                    for (int i = 1; i <= V + 1; i++) {
                        for (int lt = 0; lt <= E; lt++)  // VoteReq: dst, lastLogIndex, lastLogTerm, src, term, type
                            items.push_back({{1, dst, 0, i, lt, src, term, 0, 0, 0},
                                             nat_vreq(d, src, dst, term, i, lt),
                                             minfo(VREQ, src, dst, term, i, lt, 0, 0, 0, 0)});
                        for (int succ = 0; succ <= 1; succ++)  // AppendResp: dst, prevLogIndex, src, succ, term, type
                            items.push_back({{1, dst, 1, i, src, succ, term, 0, 0, 0},
                                             nat_aresp(d, src, dst, term, i, succ),
                                             minfo(ARESP, src, dst, term, i, succ, 0, 0, 0, 0)});
                        for (int plt = 0; plt <= E; plt++)
                            for (int lc = 1; lc <= V + 1; lc++) {
                                // AppendReq: dst, entries, leaderCommit, prevLogIndex, prevLogTerm, src, term, type
                                items.push_back({{2, dst, 0, 0, 0, lc, i, plt, src, term},
                                                 nat_areq(d, src, dst, term, i, plt, 0, 0, 0, lc),
                                                 minfo(AREQ, src, dst, term, i, plt, lc, 0, 0, 0)});
                                for (int et = 1; et <= E; et++)
                                    for (int ev = 0; ev < V; ev++)
                                        items.push_back({{2, dst, 1, et, ev, lc, i, plt, src, term},
                                                         nat_areq(d, src, dst, term, i, plt, 1, et, ev, lc),
                                                         minfo(AREQ, src, dst, term, i, plt, lc, 1, et, ev)});
                            }
                    }
                }
        if (items.size() != d.total) throw Fail(RMC_E_ARG, "message universe size mismatch");
        if (items.size() >= 0xFFFF) throw Fail(RMC_E_CAPACITY, "message universe exceeds 16-bit ids");
        std::sort(items.begin(), items.end(), [](const Item &a, const Item &b) { return a.key < b.key; });
        info.resize(items.size());
        gmsg.resize(items.size());
        nat2id.assign(d.total ? d.total : 1, 0xFFFF);
        for (size_t id = 0; id < items.size(); id++) {
            info[id] = items[id].info;
            nat2id[items[id].nat] = (uint16_t)id;
            const MsgHash h = msg_hash(items[id].info);  // rmc_spec.h: the kernels' definition too
            gmsg[id].x = h.x;
            gmsg[id].y = h.y;
        }
        if (info.empty()) { info.push_back(0); gmsg.push_back(make_ulonglong2(0, 0)); }
    }
};

template <class T>
T *dmalloc(size_t n) {
    void *p = nullptr;
    if (n == 0) n = 1;
    hipError_t e = hipMalloc(&p, n * sizeof(T));
    if (e != hipSuccess) {
        (void)hipGetLastError();
        throw Fail(RMC_E_MEMORY, "hipMalloc(" + std::to_string(n * sizeof(T)) + " B): " + hipGetErrorString(e));
    }
    return (T *)p;
}
template <class T>
T *dmalloc_try(size_t n) {  // nullptr instead of an exception
    void *p = nullptr;
    if (hipMalloc(&p, (n ? n : 1) * sizeof(T)) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return (T *)p;
}
template <class T>
void dfree(T *&p) {
    if (p) (void)hipFree((void *)p);
    p = nullptr;
}

uint64_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

uint64_t free_device_bytes() {
    size_t f = 0, t = 0;
    if (hipMemGetInfo(&f, &t) != hipSuccess) return 0;
    return f;
}

// Host array in pinned blocks (falls back to pageable blocks): the trace of every state the run
// found, written by asynchronous device-to-host copies chunk by chunk, never reallocated.
template <class T>
struct HostArr {
    static constexpr uint64_t B = 1ull << 22;
    struct Blk {
        T *p = nullptr;
        bool pinned = false;
    };
    std::vector<Blk> blk;
    uint64_t n = 0;
    HostArr() = default;
    HostArr(const HostArr &) = delete;
    HostArr &operator=(const HostArr &) = delete;
    HostArr(HostArr &&o) noexcept : blk(std::move(o.blk)), n(o.n) { o.blk.clear(); o.n = 0; }
    HostArr &operator=(HostArr &&o) noexcept {
        if (this != &o) { release(); blk = std::move(o.blk); n = o.n; o.blk.clear(); o.n = 0; }
        return *this;
    }
    ~HostArr() { release(); }
    void release() {
        for (Blk &b : blk) {
            if (b.pinned) (void)hipHostFree(b.p);
            else delete[] b.p;
        }
        blk.clear();
        n = 0;
    }
    void reserve_to(uint64_t m) {
        while ((uint64_t)blk.size() * B < m) {
            Blk b;
            if (hipHostMalloc((void **)&b.p, B * sizeof(T), hipHostMallocDefault) == hipSuccess) {
                b.pinned = true;
            } else {
                (void)hipGetLastError();
                b.p = new T[B];
            }
            blk.push_back(b);
        }
    }
    T get(uint64_t i) const { return blk[i / B].p[i % B]; }
    void set(uint64_t i, T v) {
        reserve_to(i + 1);
        blk[i / B].p[i % B] = v;
        n = std::max(n, i + 1);
    }
    // elements [at, at + cnt) from device memory, enqueued on `s` (the caller syncs before reading)
    void from_device(const T *dev, uint64_t at, uint64_t cnt, hipStream_t s) {
        reserve_to(at + cnt);
        for (uint64_t i = 0; i < cnt;) {
            const uint64_t g = at + i, k = std::min(cnt - i, B - g % B);
            HIPCHK(hipMemcpyAsync(blk[g / B].p + g % B, dev + i, k * sizeof(T), hipMemcpyDeviceToHost, s));
            i += k;
        }
        n = std::max(n, at + cnt);
    }
    void to_device(T *dev, uint64_t at, uint64_t cnt) const {
        for (uint64_t i = 0; i < cnt;) {
            const uint64_t g = at + i, k = std::min(cnt - i, B - g % B);
            HIPCHK(hipMemcpy(dev + i, blk[g / B].p + g % B, k * sizeof(T), hipMemcpyHostToDevice));
            i += k;
        }
    }
    template <class F>
    void for_range(uint64_t at, uint64_t cnt, F &&f) const {  // f(pointer, count) over contiguous pieces
        for (uint64_t i = 0; i < cnt;) {
            const uint64_t g = at + i, k = std::min(cnt - i, B - g % B);
            f(blk[g / B].p + g % B, k);
            i += k;
        }
    }
    void copy_from(const HostArr &o, uint64_t at, uint64_t cnt) {
        reserve_to(at + cnt);
        for (uint64_t i = 0; i < cnt; i++) blk[(at + i) / B].p[(at + i) % B] = o.get(at + i);
        n = std::max(n, at + cnt);
    }
};

enum Phase { PH_COUNT = 0, PH_HASH = 1, PH_DEDUP = 2, PH_MAT = 3, PH_XCHG = 4, PH_OTHER = 5 };

struct TraceStep {
    std::vector<int32_t> unpacked;
    int32_t action, server, witness;
};

}  // namespace


// Per-shard device state.  One shard per GPU (RCCL rank) -- or several "virtual"
// shards in one process on one device, which runs the identical partition/exchange
// logic with device copies instead of RCCL (the multi-GPU parity tests use it).
struct Shard {
    int id = 0;  // global shard index = owner id
    // frontier ring: record word k of level-local state p at R[wrap(cur_wbase + cur_off[p] + k)];
    // the next level's records follow at nbase() (level-relative offsets in nxt_off)
    uint32_t *R = nullptr;
    uint64_t rcap = 0;
    bool ring_fixed = false;            // sized from the budget: no further growth, consumed space reused
    uint64_t cur_wbase = 0, cur_words = 0, nxt_words = 0, peak_words = 0;
    uint64_t *cur_off = nullptr, *nxt_off = nullptr;
    uint64_t cur_off_cap = 0, nxt_off_cap = 0;
    uint64_t cur_n = 0, nxt_n = 0;
    uint64_t nbase() const { return ring_wrap(cur_wbase + cur_words, rcap); }
    // seen-set shard
    ulonglong2 *T = nullptr;
    unsigned long long *Tc = nullptr;
    uint64_t T_cap = 0, T_count = 0;
    Seen seen() const { return Seen{Tc ? nullptr : T, Tc, Tc ? 0 : T_cap - 1, T_cap}; }
    // trace: parent reference (shard << 48 | local gid) + slot key per local gid; the device
    // buffers hold gids from tflushed on, the host arrays everything before
    uint64_t *par = nullptr;
    uint16_t *pslot = nullptr;
    uint64_t trace_cap = 0, tflushed = 0;
    uint64_t tdev = 0;  // gid of device trace index 0 (set to tflushed when a kernel sequence starts)
    HostArr<uint64_t> hpar;
    HostArr<uint16_t> hslot;
    std::vector<uint64_t> level_start;  // local gid of the first state of each level
    // chunk buffers (source side)
    uint32_t *cnt = nullptr, *off = nullptr, *lslot = nullptr, *wflag = nullptr, *wpos = nullptr;
    ulonglong2 *fp = nullptr;
    unsigned long long *L = nullptr;
    ulonglong2 *LXY = nullptr;  // fused path: fingerprint of each election slot (tagged)
    uint32_t epoch = 0;
    uint32_t lxy_epoch0 = 0;    // epoch of the last LXY clear (16-bit tags repeat after 65535 epochs)
    // fused single-shard level: sparse successor staging (slot q = chunk parent * maxsucc + rank)
    uint4 *score = nullptr;
    uint32_t *wcnt = nullptr, *wacc = nullptr, *pnm = nullptr, *wposw = nullptr, *ctick = nullptr;
    uint32_t *bw = nullptr, *bg = nullptr, *boff = nullptr, *bww = nullptr, *boffw = nullptr, *tickets = nullptr;
    // device-driven level loop: control block, per-level records, and their pinned host copies
    LevelCtl *ctl = nullptr, *hctl = nullptr, *hsnap = nullptr;
    LevelRec *lrec = nullptr, *hlrec = nullptr;
    void *tmp = nullptr;
    size_t tmp_bytes = 0;
    // exchange buffers (W > 1)
    uint32_t *okey = nullptr, *okey2 = nullptr, *iota = nullptr, *perm = nullptr, *sflag = nullptr, *spos = nullptr;
    ulonglong2 *sfp = nullptr;
    unsigned long long *ocnt = nullptr;
    ulonglong2 *rfp = nullptr;
    uint32_t *rlslot = nullptr, *rflag = nullptr, *rpos = nullptr, *rcount = nullptr;
    uint64_t rcap_x = 0;
    uint32_t *sx = nullptr, *rx = nullptr;
    uint64_t sx_cap = 0, rx_cap = 0;
    uint64_t *pick_idx = nullptr;
    // errors, summary
    unsigned long long *err = nullptr, *sum = nullptr, *hsum = nullptr;
    uint32_t *flags = nullptr;
    // per-chunk host bookkeeping (sharded path)
    uint64_t p0 = 0, np = 0, G = 0;
};

struct rmc_ctx {
    rmc_config cfg{};
    KernelSet ks{};
    Universe U;
    std::string err;
    hipStream_t stream = nullptr;
    int N = 0, V = 0, RECW = 0;  // RECW = the longest record (fixed-stride buffers)
    uint32_t inv_order = 0;      // invariants in cfg order (check_invs)
    int W = 1, rank = 0;  // shards in the run, this process's first shard
    bool virt = false;    // all W shards live in this process
#ifdef RMC_WITH_RCCL
    ncclComm_t comm = nullptr;
#endif

    // device tables
    uint32_t *d_info = nullptr;
    uint16_t *d_nat2id = nullptr;
    ulonglong2 *d_gmsg = nullptr;
    uint8_t *d_perms = nullptr;
    uint64_t *d_seeds = nullptr;
    int np = 0;
    uint64_t scheme_hash = 0;  // identifies the fingerprint scheme (seeds, message hashes): checkpoints

    std::vector<Shard> sh;
    uint64_t chunk_parents = 0, Gcap = 0, Lcap_max = 0;
    // W > 1: levels below shard_min states are expanded whole on every shard with the fused
    // single-GPU level (replicated: no exchange); the run shards from the first level that reaches it
    uint64_t shard_min = 0;
    bool replicated = false;

    std::vector<hipEvent_t> evpool;
    std::vector<hipEvent_t> gev;  // device-loop group snapshots
    bool timing_on = true;        // rmc_set_timing
    struct EvRec { int ph; int a, b; };
    std::vector<EvRec> evrecs;
    int evused = 0;

    // scratch for single-state hooks
    uint32_t *d_one = nullptr, *d_out = nullptr, *d_keys = nullptr, *d_cnt1 = nullptr;
    ulonglong2 *d_fp1 = nullptr;
    int32_t *d_inv = nullptr;
    unsigned long long *d_err1 = nullptr;
    uint32_t *d_flags1 = nullptr;
    unsigned long long *d_red = nullptr, *h_red = nullptr;  // collective scratch

    // progress
    bool inited = false, finished = false;
    int status = RMC_OK;
    int depth = 0;
    uint64_t total_generated = 0, total_distinct = 0, queue_at_end = 0;
    int violated = -1;
    uint64_t err_ref = 0;  // state whose trace is reported: shard << 48 | local gid
    uint32_t err_last_slot = KEY_NONE;  // sharded: slot of the violating successor (not stored anywhere)
    std::vector<TraceStep> trace;
    double seconds = 0;

    KParams base(const Shard &s) const {
        KParams P{};
        P.d = U.d;
        P.E = cfg.max_election;
        P.R = cfg.max_restart;
        P.seeded = cfg.spec_variant == RMC_SPEC_SEEDED;
        P.check_deadlock = cfg.check_deadlock;
        P.inv_mask = cfg.invariants;
        P.inv_order = inv_order;
        P.t.info = d_info;
        P.t.nat2id = d_nat2id;
        P.t.gmsg = d_gmsg;
        P.t.perms = d_perms;
        P.t.seeds = d_seeds;
        P.t.np = np;
        P.seen = s.seen();
        P.rcap = ~0ull;  // fixed-stride buffers unless a ring is set
        P.err = s.err;
        P.flags = s.flags;
        P.par = s.par;
        P.pslot = s.pslot;
        P.trace_base = s.tdev;
        return P;
    }

    // the current level in the shard's ring as the parents of a launch
    void ring_params(const Shard &s, KParams &P) const {
        P.front = s.R;
        P.foff = s.cur_off;
        P.fbase = s.cur_wbase;
        P.rcap = s.rcap;
        P.next = s.R;
        P.noff = s.nxt_off;
        P.nbase = s.nbase();
    }

    // fused single-shard level: the chunk buffers every kernel of the level shares
    KParams chunk_params(const Shard &s) const {
        KParams Q = base(s);
        ring_params(s, Q);
        Q.cnt = s.cnt; Q.fp = s.fp; Q.wpos = s.wpos; Q.wcnt = s.wcnt; Q.wacc = s.wacc; Q.pnm = s.pnm;
        Q.wposw = s.wposw; Q.bw = s.bw; Q.bg = s.bg; Q.boff = s.boff; Q.bww = s.bww; Q.boffw = s.boffw;
        Q.tickets = s.tickets; Q.ctick = s.ctick; Q.sum = s.sum;
        Q.score = s.score; Q.lslot = s.lslot; Q.L = s.L; Q.LXY = s.LXY;
        return Q;
    }

    // ---- packing (unpacked int32 interchange <-> record) ------------------------------
    // A fixed-stride record: packed core (ks.CCW words) + ids; RECW words.
    void pack(const int32_t *u, uint32_t *rec) const {
        const int n = N, Vv = V;
        std::vector<uint32_t> w(Layout<MAXN, MAXV>::NW + 8, 0);
        int k = 0;
        auto L_VF = 0, L_CT = 1, L_ROLE = 2, L_CI = 3, L_LL = 4, L_LOG = 5, L_MI = 5 + n, L_NI = 5 + 2 * n,
             L_PEND = 5 + 3 * n, L_MISC = 6 + 3 * n;
        auto check = [](int v, int lo, int hi, const char *what) {
            if (v < lo || v > hi) throw Fail(RMC_E_ARG, std::string("state field out of range: ") + what);
        };
        for (int i = 0; i < n; i++) {
            check(u[k + i], -1, n - 1, "votedFor");
            w[L_VF] = setnib(w[L_VF], i, u[k + i] < 0 ? VF_NONE : (uint32_t)u[k + i]);
        }
        k += n;
        for (int i = 0; i < n; i++) { check(u[k + i], 0, 7, "currentTerm"); w[L_CT] = setnib(w[L_CT], i, u[k + i]); }
        k += n;
        for (int i = 0; i < n; i++) { check(u[k + i], 0, 2, "role"); w[L_ROLE] = setnib(w[L_ROLE], i, u[k + i]); }
        k += n;
        for (int i = 0; i < n; i++) { check(u[k + i], 1, Vv + 1, "commitIndex"); w[L_CI] = setnib(w[L_CI], i, u[k + i]); }
        k += n;
        std::vector<int> ll(n);
        for (int i = 0; i < n; i++) {
            check(u[k + i], 1, Vv + 1, "Len(logs)");
            ll[i] = u[k + i];
            w[L_LL] = setnib(w[L_LL], i, u[k + i]);
        }
        k += n;
        for (int i = 0; i < n; i++)
            for (int x = 1; x <= Vv + 1; x++) {
                const int t = u[k], v = u[k + 1];
                k += 2;
                if (x >= 2 && x <= ll[i]) {
                    check(t, 0, 7, "log term");
                    check(v, 0, Vv - 1, "log value");
                    w[L_LOG + i] |= (uint32_t)((t & 15) | ((v & 15) << 4)) << (8 * (x - 2));
                }
            }
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) { check(u[k], 0, Vv + 1, "matchIndex"); w[L_MI + i] = setnib(w[L_MI + i], j, u[k++]); }
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) { check(u[k], 0, Vv + 2, "nextIndex"); w[L_NI + i] = setnib(w[L_NI + i], j, u[k++]); }
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) w[L_PEND] |= (u[k++] ? 1u : 0u) << (i * n + j);
        check(u[k], 0, 7, "electionCount");
        check(u[k + 1], 0, 15, "restartCount");
        uint32_t misc = (uint32_t)(u[k] & 15) | ((uint32_t)(u[k + 1] & 15) << 4);
        k += 2;
        for (int v = 0; v < Vv; v++) misc |= (u[k++] != -1 ? 1u : 0u) << (8 + v);
        const int nm = u[k++];
        if (nm < 0 || nm > ks.MCAP) throw Fail(RMC_E_CAPACITY, "state has more messages than msg_cap");
        std::vector<uint16_t> ids;
        for (int q = 0; q < nm; q++, k += 8) {
            const int *m = u + k;
            uint32_t nat;
            switch (m[0]) {
            case VREQ: nat = nat_vreq(U.d, m[1], m[2], m[3], m[4], m[5]); break;
            case VRESP: nat = nat_vresp(U.d, m[1], m[2], m[3]); break;
            case AREQ:
                nat = m[7] < 0 ? nat_areq(U.d, m[1], m[2], m[3], m[4], m[5], 0, 0, 0, m[6])
                               : nat_areq(U.d, m[1], m[2], m[3], m[4], m[5], 1, m[7] / 8, m[7] % 8, m[6]);
                break;
            case ARESP: nat = nat_aresp(U.d, m[1], m[2], m[3], m[4], m[5]); break;
            default: throw Fail(RMC_E_ARG, "bad message type");
            }
            if (nat >= U.d.total || U.nat2id[nat] == 0xFFFF) throw Fail(RMC_E_ARG, "message outside the universe");
            ids.push_back(U.nat2id[nat]);
        }
        std::sort(ids.begin(), ids.end());
        ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
        misc |= (uint32_t)ids.size() << 16;
        w[L_MISC] = misc;
        std::memset(rec, 0, (size_t)RECW * 4);
        ks.encode(w.data(), rec);
        uint16_t *rid = reinterpret_cast<uint16_t *>(rec + ks.CCW);
        for (size_t q = 0; q < ids.size(); q++) rid[q] = ids[q];
    }

    std::vector<int32_t> unpack(const uint32_t *rec) const {
        const int n = N, Vv = V;
        const int L_VF = 0, L_CT = 1, L_ROLE = 2, L_CI = 3, L_LL = 4, L_LOG = 5, L_MI = 5 + n, L_NI = 5 + 2 * n,
                  L_PEND = 5 + 3 * n, L_MISC = 6 + 3 * n;
        std::vector<uint32_t> c(Layout<MAXN, MAXV>::NW + 8, 0);
        ks.decode(rec, c.data());
        const uint32_t misc = c[L_MISC];
        const int nm = (misc >> 16) & 0xFF;
        std::vector<int32_t> o;
        o.reserve(RMC_UNPACKED_INTS(n, Vv, nm));
        for (int i = 0; i < n; i++) { uint32_t v = nib(c[L_VF], i); o.push_back(v == VF_NONE ? -1 : (int)v); }
        for (int i = 0; i < n; i++) o.push_back(nib(c[L_CT], i));
        for (int i = 0; i < n; i++) o.push_back(nib(c[L_ROLE], i));
        for (int i = 0; i < n; i++) o.push_back(nib(c[L_CI], i));
        for (int i = 0; i < n; i++) o.push_back(nib(c[L_LL], i));
        for (int i = 0; i < n; i++)
            for (int x = 1; x <= Vv + 1; x++) {
                if (x == 1) { o.push_back(0); o.push_back(-1); continue; }
                if (x > (int)nib(c[L_LL], i)) { o.push_back(0); o.push_back(0); continue; }
                const uint32_t b = (c[L_LOG + i] >> (8 * (x - 2))) & 0xFF;
                o.push_back(b & 15);
                o.push_back(b >> 4);
            }
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) o.push_back(nib(c[L_MI + i], j));
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) o.push_back(nib(c[L_NI + i], j));
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) o.push_back((c[L_PEND] >> (i * n + j)) & 1);
        o.push_back(misc & 15);
        o.push_back((misc >> 4) & 15);
        for (int v = 0; v < Vv; v++) o.push_back(((misc >> (8 + v)) & 1) ? 0 : -1);
        o.push_back(nm);
        const uint16_t *rid = reinterpret_cast<const uint16_t *>(rec + ks.CCW);
        for (int q = 0; q < nm; q++) {
            const uint32_t m = U.info[rid[q]];
            const int t = mi_type(m);
            o.push_back(t);
            o.push_back(mi_src(m));
            o.push_back(mi_dst(m));
            o.push_back(mi_term(m));
            switch (t) {
            case VREQ: o.push_back(mi_x1(m)); o.push_back(mi_x2(m)); o.push_back(0); o.push_back(0); break;
            case VRESP: o.push_back(0); o.push_back(0); o.push_back(0); o.push_back(0); break;
            case ARESP: o.push_back(mi_x1(m)); o.push_back(mi_x2(m)); o.push_back(0); o.push_back(0); break;
            default:
                o.push_back(mi_x1(m));
                o.push_back(mi_x2(m));
                o.push_back(mi_x3(m));
                o.push_back(mi_ent(m) ? (int)(mi_et(m) * 8 + mi_ev(m)) : -1);
            }
        }
        return o;
    }

    std::vector<uint32_t> init_record() const {
        std::vector<int32_t> u;
        const int n = N;
        for (int i = 0; i < n; i++) u.push_back(-1);  // votedFor = None (tla:94)
        for (int i = 0; i < n; i++) u.push_back(0);   // currentTerm = 0 (tla:95)
        for (int i = 0; i < n; i++) u.push_back(FOL); // role = Follower (tla:96)
        for (int i = 0; i < n; i++) u.push_back(1);   // commitIndex = 1 (tla:100)
        for (int i = 0; i < n; i++) u.push_back(1);   // logs = <<[term |-> 0, val |-> None]>> (tla:97)
        for (int i = 0; i < n; i++)
            for (int x = 1; x <= V + 1; x++) { u.push_back(0); u.push_back(x == 1 ? -1 : 0); }
        for (int i = 0; i < n * n; i++) u.push_back(1);  // matchIndex (tla:98)
        for (int i = 0; i < n * n; i++) u.push_back(2);  // nextIndex (tla:99)
        for (int i = 0; i < n * n; i++) u.push_back(0);  // pendingResponse (tla:104)
        u.push_back(0);                                  // electionCount (tla:101)
        u.push_back(0);                                  // restartCount (tla:102)
        for (int v = 0; v < V; v++) u.push_back(-1);     // valSent = None (tla:105)
        u.push_back(0);                                  // msgs = {} (tla:103)
        std::vector<uint32_t> rec(RECW, 0);
        pack(u.data(), rec.data());
        return rec;
    }

    uint32_t record_words(const uint32_t *rec) const {
        std::vector<uint32_t> c(Layout<MAXN, MAXV>::NW + 8, 0);
        ks.decode(rec, c.data());
        return (uint32_t)ks.CCW + ((((c[6 + 3 * N] >> 16) & 0xFFu) + 1u) >> 1);
    }

    // ---- allocation -----------------------------------------------------------------
    void setup() {
        if (cfg.n_servers < 1 || cfg.n_servers > MAXN) throw Fail(RMC_E_ARG, "n_servers must be 1..5");
        if (cfg.n_vals < 0 || cfg.n_vals > MAXV) throw Fail(RMC_E_ARG, "n_vals must be 0..3");
        if (cfg.max_election < 0 || cfg.max_election > 7) throw Fail(RMC_E_ARG, "max_election must be 0..7");
        if (cfg.max_restart < 0 || cfg.max_restart > 15) throw Fail(RMC_E_ARG, "max_restart must be 0..15");
        if (cfg.invariants & ~0x7Fu) throw Fail(RMC_E_ARG, "unknown invariant bits");
        // invariant order: the cfg's, else bit order; every listed invariant must be selected
        inv_order = 0;
        if (cfg.invariant_order) {
            uint32_t seen = 0;
            int k = 0;
            for (uint32_t o = cfg.invariant_order; o; o >>= 4, k++) {
                const uint32_t id = (o & 15u) - 1u;
                if ((o & 15u) == 0 || id >= 7 || !(cfg.invariants & (1u << id)) || (seen & (1u << id)) || k >= 7)
                    throw Fail(RMC_E_ARG, "invariant_order does not list the selected invariants");
                seen |= 1u << id;
            }
            if (seen != cfg.invariants) throw Fail(RMC_E_ARG, "invariant_order does not list every selected invariant");
            inv_order = cfg.invariant_order;
        } else {
            int k = 0;
            for (int b = 0; b < 7; b++)
                if (cfg.invariants & (1u << b)) inv_order |= (uint32_t)(b + 1) << (4 * k++);
        }
        const int ws = cfg.world_size > 1 ? cfg.world_size : 1;
        if (cfg.virtual_shards > 1 && ws > 1) throw Fail(RMC_E_ARG, "virtual_shards and world_size > 1 are exclusive");
        if (cfg.virtual_shards > 64 || ws > 64) throw Fail(RMC_E_ARG, "at most 64 shards");
        virt = cfg.virtual_shards > 1;
        W = virt ? cfg.virtual_shards : ws;
        rank = virt ? 0 : (ws > 1 ? cfg.rank : 0);
        if (rank < 0 || rank >= W) throw Fail(RMC_E_ARG, "rank out of range");
        N = cfg.n_servers;
        V = cfg.n_vals;
        int cap = cfg.msg_cap ? cfg.msg_cap : (N <= 3 ? 64 : 128);
        if (!get_kernels(N, V, cap, &ks))
            throw Fail(RMC_E_ARG, "no compiled kernels for n_servers=" + std::to_string(N) + " n_vals=" +
                                      std::to_string(V) + " msg_cap=" + std::to_string(cap));
        RECW = ks.RECW_MAX;
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
            throw Fail(RMC_E_DEVICE, "no HIP device: the model checker runs only on the GPU");
        if (cfg.device >= 0) HIPCHK(hipSetDevice(cfg.device));
        hipDeviceProp_t prop;
        int dev = 0;
        HIPCHK(hipGetDevice(&dev));
        HIPCHK(hipGetDeviceProperties(&prop, dev));
        if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
            throw Fail(RMC_E_DEVICE, std::string("device is ") + prop.gcnArchName + ", kernels are built for gfx950");
        HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        if (W > 1 && !virt) {
#ifdef RMC_WITH_RCCL
            if (!cfg.comm_unique_id) throw Fail(RMC_E_ARG, "world_size > 1 needs comm_unique_id (rmc_comm_unique_id)");
            ncclUniqueId id;
            std::memcpy(&id, cfg.comm_unique_id, sizeof id);
            if (ncclCommInitRank(&comm, W, id, rank) != ncclSuccess) throw Fail(RMC_E_COMM, "ncclCommInitRank failed");
#else
            throw Fail(RMC_E_COMM, "built without RCCL");
#endif
        }

        U.build(N, V, cfg.max_election);
        d_info = dmalloc<uint32_t>(U.info.size());
        d_nat2id = dmalloc<uint16_t>(U.nat2id.size());
        d_gmsg = dmalloc<ulonglong2>(U.gmsg.size());
        HIPCHK(hipMemcpy(d_info, U.info.data(), U.info.size() * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(d_nat2id, U.nat2id.data(), U.nat2id.size() * 2, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(d_gmsg, U.gmsg.data(), U.gmsg.size() * 16, hipMemcpyHostToDevice));

        // Permutations(Servers) (tla:21), or the identity without SYMMETRY
        std::vector<uint8_t> perms;
        std::vector<int> a(N);
        for (int i = 0; i < N; i++) a[i] = i;
        do {
            for (int i = 0; i < MAXN; i++) perms.push_back(i < N ? (uint8_t)a[i] : 0);
        } while (!cfg.no_symmetry && std::next_permutation(a.begin(), a.end()));
        np = (int)(perms.size() / MAXN);
        d_perms = dmalloc<uint8_t>(perms.size());
        HIPCHK(hipMemcpy(d_perms, perms.data(), perms.size(), hipMemcpyHostToDevice));
        std::vector<uint64_t> seeds(2 * (MAXN + MAXN * MAXN));
        uint64_t x = SEED_SERVER;
        for (int i = 0; i < MAXN; i++) { seeds[i] = splitmix(x); seeds[MAXN + MAXN * MAXN + i] = splitmix(x); }
        x = SEED_PAIR;
        for (int i = 0; i < MAXN * MAXN; i++) {
            seeds[MAXN + i] = splitmix(x);
            seeds[2 * MAXN + MAXN * MAXN + i] = splitmix(x);
        }
        d_seeds = dmalloc<uint64_t>(seeds.size());
        HIPCHK(hipMemcpy(d_seeds, seeds.data(), seeds.size() * 8, hipMemcpyHostToDevice));
        // fingerprint scheme identity (checkpoints): seeds, message hashes, record codec, slot hash
        scheme_hash = 0x5eed5c4e3e000004ull;  // 4: signature-coset minimum for n >= 4
        auto mixin = [&](uint64_t v) { scheme_hash = mix64(scheme_hash ^ (v + 0x9e3779b97f4a7c15ull)); };
        for (uint64_t s : seeds) mixin(s);
        for (const ulonglong2 &g : U.gmsg) { mixin(g.x); mixin(g.y); }
        mixin((uint64_t)ks.CCW);
        mixin((uint64_t)Codec<3, 2>::BITS);

        // successor slots per chunk: dense for the sharded path, sparse (parents x maxsucc) for
        // the fused single-GPU path, whose staging holds SW4 * 16 + 36 bytes per slot
        Gcap = cfg.chunk_successors ? cfg.chunk_successors : (W > 1 ? (virt ? (1ull << 23) : (1ull << 26)) : (1ull << 26));
        Gcap = std::max<uint64_t>(Gcap, (uint64_t)ks.maxsucc * 64);
        if (Gcap >= (1ull << 30)) throw Fail(RMC_E_ARG, "chunk_successors must be < 2^30");
        chunk_parents = Gcap / ks.maxsucc;
        shard_min = W > 1 ? (cfg.shard_min_states ? cfg.shard_min_states : (1ull << 20)) : 0;
        const bool fused_ok = W == 1 || shard_min > 1;  // shard 0 runs the fused single-GPU level
        if (fused_ok) chunk_parents = std::min<uint64_t>(chunk_parents, (uint64_t)WTILE * 1024);  // winner-count tiles
        Lcap_max = next_pow2(2 * Gcap);

        sh.resize(virt ? W : 1);
        for (size_t i = 0; i < sh.size(); i++) alloc_shard(sh[i], virt ? (int)i : rank, fused_ok && i == 0);

        d_one = dmalloc<uint32_t>(RECW);
        d_out = dmalloc<uint32_t>((size_t)ks.maxsucc * RECW);
        d_keys = dmalloc<uint32_t>(ks.maxsucc);
        d_cnt1 = dmalloc<uint32_t>(4);
        d_fp1 = dmalloc<ulonglong2>(ks.maxsucc + 1);
        d_inv = dmalloc<int32_t>(7);
        d_err1 = dmalloc<unsigned long long>(ERR_NSLOTS);
        d_flags1 = dmalloc<uint32_t>(4);
        d_red = dmalloc<unsigned long long>(4 * 64 + 8);
        HIPCHK(hipHostMalloc((void **)&h_red, (4 * 64 + 8) * 8, hipHostMallocDefault));
        HIPCHK(hipStreamSynchronize(stream));
    }

    void alloc_shard(Shard &s, int id, bool fused) {
        s.id = id;
        s.cnt = dmalloc<uint32_t>(chunk_parents + 1);
        s.off = dmalloc<uint32_t>(chunk_parents + 1);
        s.fp = dmalloc<ulonglong2>(Gcap);
        s.lslot = dmalloc<uint32_t>(Gcap);
        s.wflag = dmalloc<uint32_t>(Gcap + 1);
        s.wpos = dmalloc<uint32_t>(Gcap + 1);
        HIPCHK(hipMemsetAsync(s.cnt, 0, (chunk_parents + 1) * 4, stream));
        HIPCHK(hipMemsetAsync(s.wflag, 0, (Gcap + 1) * 4, stream));
        s.L = dmalloc<unsigned long long>(Lcap_max);
        // an all-ones election word is older than every epoch's (elect_key) and, for the sharded
        // path's (epoch << 32) | j words, of no epoch
        HIPCHK(hipMemsetAsync(s.L, 0xFF, Lcap_max * 8, stream));
        if (fused) {
            s.LXY = dmalloc<ulonglong2>(Lcap_max);
            HIPCHK(hipMemsetAsync(s.LXY, 0, Lcap_max * 16, stream));
            int sw4 = ks.N >= 4 ? 3 : 2;
            s.score = dmalloc<uint4>(Gcap * (uint64_t)sw4);
            s.wcnt = dmalloc<uint32_t>(chunk_parents + 1);
            s.wacc = dmalloc<uint32_t>(chunk_parents + 1);
            s.pnm = dmalloc<uint32_t>(chunk_parents + 1);
            s.wposw = dmalloc<uint32_t>(chunk_parents + 1);
            s.ctick = dmalloc<uint32_t>(33 * 32);
            HIPCHK(hipMemsetAsync(s.ctick, 0, 33 * 32 * 4, stream));
            HIPCHK(hipMemsetAsync(s.wacc, 0, (chunk_parents + 1) * 4, stream));
            s.bw = dmalloc<uint32_t>(1024);
            s.bg = dmalloc<uint32_t>(1024);
            s.boff = dmalloc<uint32_t>(1024);
            s.bww = dmalloc<uint32_t>(1024);
            s.boffw = dmalloc<uint32_t>(1024);
            s.tickets = dmalloc<uint32_t>(4);
            HIPCHK(hipMemsetAsync(s.tickets, 0, 16, stream));
            s.ctl = dmalloc<LevelCtl>(1);
            s.lrec = dmalloc<LevelRec>(LREC_CAP);
            HIPCHK(hipHostMalloc((void **)&s.hctl, sizeof(LevelCtl), hipHostMallocDefault));
            HIPCHK(hipHostMalloc((void **)&s.hsnap, 3 * sizeof(LevelCtl), hipHostMallocDefault));
            HIPCHK(hipHostMalloc((void **)&s.hlrec, sizeof(LevelRec) * LREC_CAP, hipHostMallocDefault));
        }
        size_t t1 = 0, t2 = 0;
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, t1, s.cnt, s.off, (int)Gcap + 1, stream));
        if (W > 1) {
            s.okey = dmalloc<uint32_t>(Gcap);
            s.okey2 = dmalloc<uint32_t>(Gcap);
            s.iota = dmalloc<uint32_t>(Gcap);
            s.perm = dmalloc<uint32_t>(Gcap);
            s.sflag = dmalloc<uint32_t>(Gcap + 1);
            s.spos = dmalloc<uint32_t>(Gcap + 1);
            s.sfp = dmalloc<ulonglong2>(Gcap);
            s.ocnt = dmalloc<unsigned long long>(64);
            s.pick_idx = dmalloc<uint64_t>(2 * 65);
            int bits = 0;
            while ((1 << bits) < W) bits++;
            HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, t2, s.okey, s.okey2, s.iota, s.perm, (int)Gcap, 0,
                                                      std::max(bits, 1), stream));
        }
        s.tmp_bytes = std::max(t1, t2);
        s.tmp = dmalloc<uint8_t>(s.tmp_bytes);
        s.T_cap = 1ull << (cfg.seen_log2 ? cfg.seen_log2 : 22);
        s.T = dmalloc<ulonglong2>(s.T_cap);
        HIPCHK(hipMemsetAsync(s.T, 0, s.T_cap * 16, stream));
        s.err = dmalloc<unsigned long long>(ERR_NSLOTS);
        s.flags = dmalloc<uint32_t>(4);
        HIPCHK(hipMemsetAsync(s.err, 0xFF, ERR_NSLOTS * 8, stream));
        HIPCHK(hipMemsetAsync(s.flags, 0, 16, stream));
        s.sum = dmalloc<unsigned long long>(160);
        HIPCHK(hipHostMalloc((void **)&s.hsum, 160 * 8, hipHostMallocDefault));
        s.rcap = 1ull << 14;
        s.R = dmalloc<uint32_t>(s.rcap);
        s.cur_off_cap = s.nxt_off_cap = 1 << 16;
        s.cur_off = dmalloc<uint64_t>(s.cur_off_cap);
        s.nxt_off = dmalloc<uint64_t>(s.nxt_off_cap);
        s.trace_cap = 1 << 20;
        s.par = dmalloc<uint64_t>(s.trace_cap);
        s.pslot = dmalloc<uint16_t>(s.trace_cap);
    }

    void free_shard(Shard &s) {
        dfree(s.R); dfree(s.cur_off); dfree(s.nxt_off); dfree(s.T); dfree(s.Tc); dfree(s.par); dfree(s.pslot);
        dfree(s.cnt); dfree(s.off);
        dfree(s.lslot); dfree(s.wflag); dfree(s.wpos); dfree(s.fp); dfree(s.L); dfree(s.LXY); dfree(s.tmp); dfree(s.okey);
        dfree(s.okey2); dfree(s.iota); dfree(s.perm); dfree(s.sflag); dfree(s.spos); dfree(s.sfp); dfree(s.ocnt);
        dfree(s.rfp); dfree(s.rlslot); dfree(s.rflag); dfree(s.rpos); dfree(s.rcount); dfree(s.sx); dfree(s.rx);
        dfree(s.pick_idx); dfree(s.err); dfree(s.sum); dfree(s.flags);
        dfree(s.score); dfree(s.wcnt); dfree(s.wacc); dfree(s.pnm); dfree(s.wposw); dfree(s.ctick);
        dfree(s.bw); dfree(s.bg); dfree(s.boff); dfree(s.bww); dfree(s.boffw); dfree(s.tickets);
        dfree(s.ctl); dfree(s.lrec);
        if (s.hsum) (void)hipHostFree(s.hsum);
        if (s.hctl) (void)hipHostFree(s.hctl);
        if (s.hsnap) (void)hipHostFree(s.hsnap);
        if (s.hlrec) (void)hipHostFree(s.hlrec);
        s.hsum = nullptr; s.hctl = nullptr; s.hsnap = nullptr; s.hlrec = nullptr;
        s.hpar.release();
        s.hslot.release();
    }

    void release() {
        if (stream) (void)hipStreamSynchronize(stream);
        for (Shard &s : sh) free_shard(s);
        sh.clear();
        dfree(d_info); dfree(d_nat2id); dfree(d_gmsg); dfree(d_perms); dfree(d_seeds);
        dfree(d_one); dfree(d_out); dfree(d_keys); dfree(d_cnt1); dfree(d_fp1); dfree(d_inv); dfree(d_err1);
        dfree(d_flags1); dfree(d_red);
        if (h_red) (void)hipHostFree(h_red);
        h_red = nullptr;
        for (hipEvent_t e : evpool) (void)hipEventDestroy(e);
        evpool.clear();
        for (hipEvent_t e : gev) (void)hipEventDestroy(e);
        gev.clear();
#ifdef RMC_WITH_RCCL
        if (comm) (void)ncclCommDestroy(comm);
        comm = nullptr;
#endif
        if (stream) (void)hipStreamDestroy(stream);
        stream = nullptr;
    }

    // ---- frontier storage --------------------------------------------------------------------
    // offsets array with `used` entries kept
    void ensure_off(uint64_t *&p, uint64_t &cap, uint64_t used, uint64_t need) {
        if (need <= cap) return;
        const uint64_t nc = std::max<uint64_t>(need + need / 2, cap * 2);
        uint64_t *nb = dmalloc<uint64_t>(nc);
        if (used) HIPCHK(hipMemcpyAsync(nb, p, used * 8, hipMemcpyDeviceToDevice, stream));
        HIPCHK(hipStreamSynchronize(stream));
        dfree(p);
        p = nb;
        cap = nc;
    }

    // copy `words` ring words starting at ring position `from` (wrapping) to dst (linear)
    void ring_copy_out(const Shard &s, uint64_t from, uint64_t words, uint32_t *dst) {
        const uint64_t n1 = std::min(words, s.rcap - from);
        if (n1) HIPCHK(hipMemcpyAsync(dst, s.R + from, n1 * 4, hipMemcpyDeviceToDevice, stream));
        if (words > n1) HIPCHK(hipMemcpyAsync(dst + n1, s.R, (words - n1) * 4, hipMemcpyDeviceToDevice, stream));
    }

    // replace the ring by one of `nc` words holding the live region (the current level and the
    // next level so far) from position 0
    bool ring_realloc(Shard &s, uint64_t nc) {
        uint32_t *nr = dmalloc_try<uint32_t>(nc);
        if (!nr) return false;
        ring_copy_out(s, s.cur_wbase, s.cur_words + s.nxt_words, nr);
        HIPCHK(hipStreamSynchronize(stream));
        dfree(s.R);
        s.R = nr;
        s.rcap = nc;
        s.cur_wbase = 0;
        return true;
    }

    // Room for `extra` more words of the next level.  `consumed` = words at the start of the
    // current level that are no longer needed (its chunks already expanded): a ring at its budget
    // reuses them.
    void ensure_ring(Shard &s, uint64_t extra, uint64_t consumed) {
        const uint64_t live = s.cur_words + s.nxt_words;
        if (live + extra <= s.rcap) return;
        if (!s.ring_fixed) {
            const uint64_t nc = std::max<uint64_t>(s.rcap * 2, (live + extra) + (live + extra) / 2);
            if (ring_realloc(s, nc)) return;
        }
        if (live - consumed + extra <= s.rcap) return;
        throw Fail(RMC_E_MEMORY, "frontier ring full: " + std::to_string((live - consumed + extra) * 4) +
                                     " B of live frontier records needed, ring is " + std::to_string(s.rcap * 4) +
                                     " B (rmc_config.frontier_mem_bytes, or more GPUs)");
    }

    // device trace buffer for `need` entries from tflushed on (everything earlier is on the host)
    void grow_trace(Shard &s, uint64_t need) {
        if (need <= s.trace_cap) return;
        HIPCHK(hipStreamSynchronize(stream));  // pending flushes read the old buffers
        const uint64_t nc = std::max<uint64_t>(need + need / 2, s.trace_cap * 2);
        dfree(s.par);
        dfree(s.pslot);
        s.par = dmalloc<uint64_t>(nc);
        s.pslot = dmalloc<uint16_t>(nc);
        s.trace_cap = nc;
    }

    // trace entries of gids [tflushed, upto) to the host (asynchronous, stream-ordered)
    void flush_trace(Shard &s, uint64_t upto) {
        if (upto <= s.tflushed) return;
        const uint64_t n = upto - s.tflushed, at = s.tflushed - s.tdev;
        s.hpar.from_device(s.par + at, s.tflushed, n, stream);
        s.hslot.from_device(s.pslot + at, s.tflushed, n, stream);
        s.tflushed = upto;
    }
    // the device trace buffer starts over at the first gid not yet on the host
    void trace_restart(Shard &s) { s.tdev = s.tflushed; }

    // Seen set: keep the load <= 1/2 in the full (16-B) table, grown x4 by rehash, up to
    // 2^compact_log2 slots; then migrate once to the compact table sized from the budget, whose
    // load may reach 0.9.
    void grow_seen(Shard &s, uint64_t need) {
        if (s.Tc) {
            if ((double)need > 0.9 * (double)s.T_cap)
                throw Fail(RMC_E_MEMORY, "seen set full: " + std::to_string(need) + " fingerprints in " +
                                             std::to_string(s.T_cap) + " 8-B slots (rmc_config.seen_mem_bytes, or more GPUs)");
            return;
        }
        if (need * 2 <= s.T_cap) return;
        uint64_t nc = s.T_cap;
        while (need * 2 > nc) nc *= 4;
        if (nc > (1ull << full_max_log2())) {
            migrate_compact(s, s.T_count);
            grow_seen(s, need);
            return;
        }
        ulonglong2 *nT = dmalloc<ulonglong2>(nc);
        HIPCHK(hipMemsetAsync(nT, 0, nc * 16, stream));
        launch_rehash(s.T, s.T_cap, Seen{nT, nullptr, nc - 1, nc}, stream);
        HIPCHK(hipStreamSynchronize(stream));
        dfree(s.T);
        s.T = nT;
        s.T_cap = nc;
    }

    uint32_t full_max_log2() const { return cfg.compact_log2 ? cfg.compact_log2 : 27; }

    // Switch to the compact seen set now if the full one would have to grow past its limit to take
    // `need` (a bound): callers then size their chunk on the compact table's room.
    void maybe_migrate(Shard &s, uint64_t need) {
        if (s.Tc || need * 2 <= s.T_cap) return;
        uint64_t nc = s.T_cap;
        while (need * 2 > nc) nc *= 4;
        if (nc > (1ull << full_max_log2())) migrate_compact(s, s.T_count);
    }

    void migrate_compact(Shard &s, uint64_t need) {
        const uint64_t local = sh.size();
        HIPCHK(hipStreamSynchronize(stream));
        const uint64_t budget = cfg.seen_mem_bytes ? cfg.seen_mem_bytes : free_device_bytes() / 2 / local;
        const uint64_t slots = budget / 8 / 64 * 64;
        if ((double)need > 0.85 * (double)slots)
            throw Fail(RMC_E_MEMORY, "seen set: " + std::to_string(need) + " fingerprints do not fit the budget of " +
                                         std::to_string(budget) + " B");
        unsigned long long *Tc = dmalloc<unsigned long long>(slots);
        HIPCHK(hipMemsetAsync(Tc, 0, slots * 8, stream));
        launch_rehash(s.T, s.T_cap, Seen{nullptr, Tc, 0, slots}, stream);
        HIPCHK(hipStreamSynchronize(stream));
        dfree(s.T);
        s.Tc = Tc;
        s.T_cap = slots;
        // the run is large: the frontier ring goes to its budget and stops growing
        fix_ring(s, local);
    }

    // The frontier ring at its budget: rmc_config.frontier_mem_bytes (which may be smaller than the
    // ring so far, down to the live frontier), else 70 % of the free device memory.
    void fix_ring(Shard &s, uint64_t local) {
        const uint64_t live = s.cur_words + s.nxt_words;
        uint64_t words;
        if (cfg.frontier_mem_bytes) {
            words = std::max<uint64_t>(cfg.frontier_mem_bytes / 4, live + 1);
        } else {
            HIPCHK(hipStreamSynchronize(stream));
            words = std::max<uint64_t>((uint64_t)((double)free_device_bytes() * 0.7) / local / 4, s.rcap);
        }
        if (words != s.rcap && !ring_realloc(s, words))
            throw Fail(RMC_E_MEMORY, "frontier ring of " + std::to_string(words * 4) + " B");
        s.ring_fixed = true;
    }

    // would a chunk bounded by `gub` successors fit without growing a fixed ring or a compact seen set?
    bool seen_room(const Shard &s, uint64_t need) const { return !s.Tc || (double)need <= 0.9 * (double)s.T_cap; }
    bool ring_room(const Shard &s, uint64_t extra, uint64_t consumed) const {
        return !s.ring_fixed || s.cur_words + s.nxt_words - consumed + extra <= s.rcap;
    }

    template <class T>
    void grow_plain(T *&p, uint64_t &cap, uint64_t need) {
        if (need <= cap) return;
        uint64_t nc = std::max<uint64_t>(need + need / 2, 1024);
        dfree(p);
        p = dmalloc<T>(nc);
        cap = nc;
    }

    void grow_recv(Shard &s, uint64_t need) {
        if (need + 1 <= s.rcap_x) return;
        uint64_t nc = std::max<uint64_t>(need + need / 2 + 1, 1024);
        dfree(s.rfp); dfree(s.rlslot); dfree(s.rflag); dfree(s.rpos);
        s.rfp = dmalloc<ulonglong2>(nc);
        s.rlslot = dmalloc<uint32_t>(nc);
        s.rflag = dmalloc<uint32_t>(nc);
        s.rpos = dmalloc<uint32_t>(nc);
        HIPCHK(hipMemsetAsync(s.rflag, 0, nc * 4, stream));
        s.rcap_x = nc;
        if (!s.rcount) s.rcount = dmalloc<uint32_t>(4);
    }

    // Phase timing by event pairs on the engine's stream, read back at the next sync
    // point (no extra synchronisation inside a level).
    int ev() {
        if (evused == (int)evpool.size()) {
            hipEvent_t e;
            HIPCHK(hipEventCreate(&e));
            evpool.push_back(e);
        }
        return evused++;
    }
    template <class F>
    void timed(int ph, F &&f) {
        if (!timing_on || (cfg.timing_phases && !(cfg.timing_phases & (1u << ph)))) { f(); return; }
        const int a = ev();
        HIPCHK(hipEventRecord(evpool[a], stream));
        f();
        const int b = ev();
        HIPCHK(hipEventRecord(evpool[b], stream));
        evrecs.push_back({ph, a, b});
    }
    void collect_times(rmc_level_stats *st) {  // call after a stream sync
        for (const EvRec &r : evrecs) {
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, evpool[r.a], evpool[r.b]));
            if (st) {
                st->kernel_ms[r.ph] += ms;
                st->kernel_launches[r.ph] += 1;
            }
        }
        evrecs.clear();
        evused = 0;
    }

    template <class T>
    T d2h(const T *p) {
        T v;
        HIPCHK(hipMemcpyAsync(&v, p, sizeof(T), hipMemcpyDeviceToHost, stream));
        HIPCHK(hipStreamSynchronize(stream));
        return v;
    }

    // ---- collectives over shards --------------------------------------------------------
    // Every host value handed to these is this process's contribution (virtual mode: the
    // sum/max over all local shards already IS the global value).
    void allreduce(uint64_t *v, int n, bool is_max) {
        if (W == 1 || virt) return;
#ifdef RMC_WITH_RCCL
        for (int i = 0; i < n; i++) h_red[i] = v[i];
        HIPCHK(hipMemcpyAsync(d_red, h_red, n * 8, hipMemcpyHostToDevice, stream));
        if (ncclAllReduce(d_red, d_red, n, ncclUint64, is_max ? ncclMax : ncclSum, comm, stream) != ncclSuccess)
            throw Fail(RMC_E_COMM, "ncclAllReduce failed");
        HIPCHK(hipMemcpyAsync(h_red, d_red, n * 8, hipMemcpyDeviceToHost, stream));
        HIPCHK(hipStreamSynchronize(stream));
        for (int i = 0; i < n; i++) v[i] = h_red[i];
#endif
    }

    // counts: c_out[local d][s] = c_in[local s][d]
    void exchange_counts(const std::vector<std::vector<uint64_t>> &in, std::vector<std::vector<uint64_t>> &out) {
        out.assign(sh.size(), std::vector<uint64_t>(W, 0));
        if (virt || W == 1) {
            for (int s = 0; s < W && s < (int)in.size(); s++)
                for (int d = 0; d < (int)sh.size(); d++) out[d][s] = in[s][d];
            return;
        }
#ifdef RMC_WITH_RCCL
        for (int d = 0; d < W; d++) h_red[d] = in[0][d];
        HIPCHK(hipMemcpyAsync(d_red, h_red, W * 8, hipMemcpyHostToDevice, stream));
        if (ncclAllToAll(d_red, d_red + 64, 1, ncclUint64, comm, stream) != ncclSuccess)
            throw Fail(RMC_E_COMM, "ncclAllToAll failed");
        HIPCHK(hipMemcpyAsync(h_red, d_red + 64, W * 8, hipMemcpyDeviceToHost, stream));
        HIPCHK(hipStreamSynchronize(stream));
        for (int s = 0; s < W; s++) out[0][s] = h_red[s];
#endif
    }

    // alltoallv of fixed-size items: send[local s] segment d (cnt scnt[s][d] at soff[s][d]) ->
    // recv[local d] segment s (at roff[d][s]).
    void exchange_items(const std::vector<const void *> &send, const std::vector<std::vector<uint64_t>> &scnt,
                        const std::vector<std::vector<uint64_t>> &soff, const std::vector<void *> &recv,
                        const std::vector<std::vector<uint64_t>> &roff, size_t elem) {
        if (virt || W == 1) {
            for (int s = 0; s < W; s++)
                for (int d = 0; d < W; d++) {
                    const uint64_t n = scnt[s][d];
                    if (!n) continue;
                    HIPCHK(hipMemcpyAsync((char *)recv[d] + roff[d][s] * elem, (const char *)send[s] + soff[s][d] * elem,
                                          n * elem, hipMemcpyDeviceToDevice, stream));
                }
            return;
        }
#ifdef RMC_WITH_RCCL
        // recv counts are the transposed send counts, known to the caller through roff
        if (ncclGroupStart() != ncclSuccess) throw Fail(RMC_E_COMM, "ncclGroupStart failed");
        for (int peer = 0; peer < W; peer++) {
            const uint64_t ns = scnt[0][peer];
            const uint64_t nr = roff[0][peer + 1] - roff[0][peer];
            if (ns && ncclSend((const char *)send[0] + soff[0][peer] * elem, ns * elem, ncclUint8, peer, comm, stream) != ncclSuccess)
                throw Fail(RMC_E_COMM, "ncclSend failed");
            if (nr && ncclRecv((char *)recv[0] + roff[0][peer] * elem, nr * elem, ncclUint8, peer, comm, stream) != ncclSuccess)
                throw Fail(RMC_E_COMM, "ncclRecv failed");
        }
        if (ncclGroupEnd() != ncclSuccess) throw Fail(RMC_E_COMM, "ncclGroupEnd failed");
#endif
    }

    // successors of one record already in d_one: keys + records in d_out
    uint32_t expand_one(std::vector<uint32_t> *keys, std::vector<uint32_t> *recs, std::vector<ulonglong2> *fps,
                        bool *assert_fail) {
        HIPCHK(hipMemsetAsync(d_err1, 0xFF, ERR_NSLOTS * 8, stream));
        HIPCHK(hipMemsetAsync(d_flags1, 0, 16, stream));
        KParams P = base(sh[0]);
        P.err = d_err1;
        P.flags = d_flags1;
        P.front = d_one;
        P.p_begin = 0;
        P.p_end = 1;
        P.next = d_out;
        P.fp = d_fp1;
        P.out_keys = d_keys;
        P.out_count = d_cnt1;
        HIPCHK(hipMemsetAsync(d_cnt1, 0, 16, stream));
        ks.single(P, stream);
        HIPCHK(hipGetLastError());
        const uint32_t cnt = d2h(d_cnt1);
        unsigned long long e[ERR_NSLOTS];
        uint32_t fl[4];
        HIPCHK(hipMemcpy(e, d_err1, sizeof e, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(fl, d_flags1, sizeof fl, hipMemcpyDeviceToHost));
        if (fl[0]) throw Fail(RMC_E_CAPACITY, "a successor exceeds msg_cap messages");
        *assert_fail = e[ERR_ASSERT] != ~0ull;
        if (keys) {
            keys->resize(cnt);
            if (cnt) HIPCHK(hipMemcpy(keys->data(), d_keys, cnt * 4, hipMemcpyDeviceToHost));
        }
        if (recs) {
            recs->resize((size_t)cnt * RECW);
            if (cnt) HIPCHK(hipMemcpy(recs->data(), d_out, (size_t)cnt * RECW * 4, hipMemcpyDeviceToHost));
        }
        if (fps) {
            fps->resize(cnt);
            if (cnt) HIPCHK(hipMemcpy(fps->data(), d_fp1, cnt * 16, hipMemcpyDeviceToHost));
        }
        return cnt;
    }

    // level-local parent p of shard s (current level) -> d_one (RECW words, fixed stride)
    void record_to_one(Shard &s, uint64_t p) {
        const uint64_t o = d2h(s.cur_off + p);
        ring_copy_out(s, ring_wrap(s.cur_wbase + o, s.rcap), std::min<uint64_t>(RECW, s.rcap), d_one);
        HIPCHK(hipStreamSynchronize(stream));
    }

    // ---- BFS --------------------------------------------------------------------------
    int init(rmc_level_stats *st) {
        if (inited) throw Fail(RMC_E_STATE, "rmc_init called twice");
        auto t0 = std::chrono::steady_clock::now();
        std::vector<uint32_t> rec = init_record();
        const uint32_t rw = record_words(rec.data());
        HIPCHK(hipMemcpy(d_one, rec.data(), RECW * 4, hipMemcpyHostToDevice));
        KParams P = base(sh[0]);
        P.front = d_one;
        P.fp = d_fp1;
        ks.fp_states(P, 1, stream);
        ks.inv_states(P, 1, d_inv, stream);
        uint32_t owner = 0;
        replicated = W > 1 && shard_min > 1;
        if (W > 1 && !replicated) {
            launch_owner_of(d_fp1, (uint32_t)W, d_cnt1, stream);
            owner = d2h(d_cnt1);
        }
        int32_t iv[7];
        HIPCHK(hipMemcpyAsync(iv, d_inv, sizeof iv, hipMemcpyDeviceToHost, stream));
        HIPCHK(hipStreamSynchronize(stream));
        const uint64_t zero = 0;
        for (Shard &s : sh) {
            s.level_start = {0};
            s.cur_n = 0;
            s.cur_wbase = s.cur_words = s.nxt_words = 0;
            if (replicated ? &s != &sh[0] : (uint32_t)s.id != owner) continue;
            HIPCHK(hipMemcpyAsync(s.R, d_one, rw * 4, hipMemcpyDeviceToDevice, stream));
            HIPCHK(hipMemcpyAsync(s.cur_off, &zero, 8, hipMemcpyHostToDevice, stream));
            launch_insert_fps(d_fp1, 1, s.seen(), stream);
            s.hpar.set(0, ~0ull);
            s.hslot.set(0, 0);
            s.tflushed = 1;
            s.cur_n = 1;
            s.cur_words = rw;
            s.T_count = 1;
        }
        HIPCHK(hipStreamSynchronize(stream));
        total_generated = 1;  // TLC counts the initial state as generated
        total_distinct = 1;
        depth = 1;
        inited = true;
        status = RMC_OK;
        for (uint32_t o = inv_order; o; o >>= 4) {
            const int b = (int)(o & 15u) - 1;
            if (iv[b] != 1) {
                status = iv[b] == 0 ? RMC_VIOLATION : RMC_EVAL_ERROR;
                violated = b;
                err_ref = ((uint64_t)owner << 48);
                err_last_slot = KEY_NONE;
                queue_at_end = 0;
                finished = true;
                build_trace();
                break;
            }
        }
        seconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (st) {
            std::memset(st, 0, sizeof *st);
            st->level = 1;
            st->status = status;
            st->total_generated = total_generated;
            st->total_distinct = total_distinct;
            st->queue = finished ? 0 : 1;
            st->new_states = 1;
            st->expanded = 0;
            st->seconds = seconds;
            st->new_bytes = rw * 4ull;
        }
        return status;
    }

    int step(rmc_level_stats *st) {
        if (!inited) throw Fail(RMC_E_STATE, "rmc_step before rmc_init");
        if (finished) return status == RMC_OK ? RMC_DONE : status;
        rmc_level_stats local;
        if (!st) st = &local;
        std::memset(st, 0, sizeof *st);
        if (replicated && sh[0].cur_n >= shard_min) enter_sharded();
        return (W == 1 || replicated) ? step_single(st) : step_sharded(st);
    }

    // shard t takes over parents [o, o + n) of shard src's current level: records (their words)
    // into t's ring from position 0, offsets rebased to the first of them
    void take_parents(Shard &src, Shard &t, uint64_t o, uint64_t n) {
        const uint64_t F = src.cur_n;
        const uint64_t w_lo = o < F ? d2h(src.cur_off + o) : src.cur_words;
        const uint64_t w_hi = o + n < F ? d2h(src.cur_off + o + n) : src.cur_words;
        if (&src == &t) {
            ensure_off(t.nxt_off, t.nxt_off_cap, 0, std::max<uint64_t>(n, 1));
            launch_rebase(t.cur_off + o, n, w_lo, t.nxt_off, stream);
            std::swap(t.cur_off, t.nxt_off);
            std::swap(t.cur_off_cap, t.nxt_off_cap);
            t.cur_wbase = ring_wrap(t.cur_wbase + w_lo, t.rcap);
        } else {
            t.cur_words = t.nxt_words = 0;
            t.cur_wbase = 0;
            ensure_ring(t, w_hi - w_lo, 0);
            ring_copy_out(src, ring_wrap(src.cur_wbase + w_lo, src.rcap), w_hi - w_lo, t.R);
            ensure_off(t.cur_off, t.cur_off_cap, 0, std::max<uint64_t>(n, 1));
            launch_rebase(src.cur_off + o, n, w_lo, t.cur_off, stream);
        }
        t.cur_words = w_hi - w_lo;
        t.cur_n = n;
        HIPCHK(hipStreamSynchronize(stream));
    }

    // Replicated -> sharded, at the start of the first level with >= shard_min states.  Every
    // shard holds that level whole (and every state seen so far in its seen set); shard i keeps
    // parents [F*i/W, F*(i+1)/W) as its frontier, so parent references of the next level,
    // (i << 48 | gid), name shard i's copy of them.  Earlier replicated levels are referenced as
    // shard 0's (tag 0), whose copy stays intact: each shard writes new states only past its range.
    void enter_sharded() {
        Shard &s0 = sh[0];
        const size_t L = s0.level_start.size();
        const uint64_t F = s0.cur_n, base = s0.level_start[L - 1];
        auto off = [&](int i) { return F * (uint64_t)i / (uint64_t)W; };
        HIPCHK(hipStreamSynchronize(stream));
        if (virt) {
            for (int i = 1; i < W; i++) {
                Shard &t = sh[i];
                const uint64_t o = off(i), n = off(i + 1) - o;
                if (s0.Tc) {
                    if (!t.Tc || t.T_cap != s0.T_cap) {
                        dfree(t.T);
                        dfree(t.Tc);
                        t.Tc = dmalloc<unsigned long long>(s0.T_cap);
                        t.T_cap = s0.T_cap;
                    }
                    HIPCHK(hipMemcpyAsync(t.Tc, s0.Tc, s0.T_cap * 8, hipMemcpyDeviceToDevice, stream));
                } else {
                    if (t.T_cap != s0.T_cap || !t.T) {
                        dfree(t.T);
                        t.T = dmalloc<ulonglong2>(s0.T_cap);
                        t.T_cap = s0.T_cap;
                    }
                    HIPCHK(hipMemcpyAsync(t.T, s0.T, s0.T_cap * 16, hipMemcpyDeviceToDevice, stream));
                }
                t.T_count = s0.T_count;
                t.level_start = s0.level_start;
                t.level_start.back() = base + o;
                take_parents(s0, t, o, n);
                t.hpar.copy_from(s0.hpar, base + o, n);
                t.hslot.copy_from(s0.hslot, base + o, n);
                t.tflushed = base + o + n;
                t.epoch = std::max(t.epoch, s0.epoch);
            }
            take_parents(s0, s0, 0, off(1));
            s0.tflushed = base + off(1);
        } else {
            const uint64_t o = off(rank), n = off(rank + 1) - o;
            take_parents(s0, s0, o, n);
            s0.level_start.back() = base + o;
            s0.tflushed = base + o + n;
        }
        HIPCHK(hipStreamSynchronize(stream));
        replicated = false;
    }

    // First error in TLC order among the error slots: smaller (parent, slot) first; on a
    // tie the Assert wins (its sub-action's batch is discarded).
    static int first_error(const unsigned long long *e, unsigned long long *best) {
        int kind = -1;
        *best = ~0ull;
        const int order[4] = {ERR_ASSERT, ERR_DEADLOCK, ERR_INV, ERR_EVAL};
        for (int q = 0; q < 4; q++) {
            const int kk = order[q];
            if (e[kk] == ~0ull) continue;
            if (kind < 0 || (e[kk] >> 8) < (*best >> 8)) { kind = kk; *best = e[kk]; }
        }
        return kind;
    }

    // The fused path's election slots carry 16-bit epoch tags (elect_tag): before the next
    // `ahead` epochs could reuse a tag still in LXY, clear it (all tags are nonzero).
    void renew_election_tags(Shard &s, uint32_t ahead) {
        if (!s.LXY || s.epoch + ahead - s.lxy_epoch0 < 0xFFFFu) return;
        HIPCHK(hipMemsetAsync(s.LXY, 0, Lcap_max * 16, stream));
        s.lxy_epoch0 = s.epoch;
    }

    void end_level(Shard &s, uint64_t gid_nxt, int L) {
        std::swap(s.cur_off, s.nxt_off);
        std::swap(s.cur_off_cap, s.nxt_off_cap);
        s.cur_wbase = s.nbase();
        s.cur_words = s.nxt_words;
        s.nxt_words = 0;
        s.cur_n = s.nxt_n;
        s.nxt_n = 0;
        if (s.cur_n) s.level_start.push_back(gid_nxt);
        (void)L;
    }

    int step_single(rmc_level_stats *st) {
        auto t0 = std::chrono::steady_clock::now();
        Shard &s = sh[0];
        const int L = (int)s.level_start.size();  // expanding level L (1-based)
        st->level = L;
        st->expanded = s.cur_n;
        const uint64_t gid_cur = s.level_start[L - 1];
        const uint64_t gid_nxt = gid_cur + s.cur_n;
        uint64_t level_gen = 0;
        s.nxt_n = 0;
        s.nxt_words = 0;
        const uint64_t MSW = (uint64_t)ks.maxsucc * (uint64_t)ks.RECW_MAX;
        for (uint64_t p0 = 0; p0 < s.cur_n; p0 += chunk_parents) {
            const uint64_t p1 = std::min(s.cur_n, p0 + chunk_parents), np_ = p1 - p0;
            // Small chunks size the next level, trace and seen set on the successor upper bound
            // without a host round trip; large ones read the winner count back before commit.
            const uint64_t Gub = np_ * (uint64_t)ks.maxsucc;
            maybe_migrate(s, s.T_count + Gub);
            const uint64_t consumed = (s.ring_fixed && p0) ? d2h(s.cur_off + p0) : 0;
            // bounds that a fixed ring or a compact seen set cannot take go the exact way
            const bool small = Gub <= (1ull << 20) && seen_room(s, s.T_count + Gub) && ring_room(s, np_ * MSW, consumed);
            if (small) {
                ensure_ring(s, np_ * MSW, consumed);
                ensure_off(s.nxt_off, s.nxt_off_cap, s.nxt_n, s.nxt_n + Gub);
                grow_trace(s, Gub);
                grow_seen(s, s.T_count + Gub);
            }
            const uint64_t Lcap = std::min(next_pow2(2 * Gub), Lcap_max);
            renew_election_tags(s, 1);
            ++s.epoch;
            trace_restart(s);
            auto params = [&] {
                KParams Q = chunk_params(s);
                Q.p_begin = p0; Q.p_end = p1; Q.next_base = s.nxt_n; Q.next_wbase = s.nxt_words;
                Q.gid_next_base = gid_nxt; Q.gid_parent_base = gid_cur;
                Q.Lmask = Lcap - 1;
                Q.epoch = s.epoch;
                return Q;
            };
            // expand + fingerprint + seen-set probe + staging, one evaluation per parent
            timed(PH_HASH, [&] { ks.fused(params(), stream); });
            timed(PH_DEDUP, [&] { ks.wincount(params(), np_, stream); });
            if (!small) {
                HIPCHK(hipMemcpyAsync(s.hsum, s.sum, 8 * 8, hipMemcpyDeviceToHost, stream));
                HIPCHK(hipStreamSynchronize(stream));
                collect_times(st);
                const uint64_t Wub = s.hsum[1], Wwords = s.hsum[SUM_WORDS];
                ensure_ring(s, Wwords, consumed);
                ensure_off(s.nxt_off, s.nxt_off_cap, s.nxt_n, s.nxt_n + Wub);
                grow_trace(s, Wub);
                grow_seen(s, s.T_count + Wub);
            }
            timed(PH_MAT, [&] { ks.commit(params(), stream); });  // + chunk summary
            HIPCHK(hipMemcpyAsync(s.hsum, s.sum, 8 * 8, hipMemcpyDeviceToHost, stream));
            HIPCHK(hipStreamSynchronize(stream));
            HIPCHK(hipGetLastError());
            collect_times(st);
            const uint64_t G = s.hsum[0], Wn = s.hsum[1], Ww = s.hsum[SUM_WORDS];
            if (s.hsum[2 + ERR_NSLOTS]) throw Fail(RMC_E_CAPACITY, "a state exceeds msg_cap = " + std::to_string(ks.MCAP) + " messages");
            flush_trace(s, gid_nxt + s.nxt_n + Wn);
            level_gen += G;
            s.T_count += Wn;
            unsigned long long best;
            const int kind = first_error(s.hsum + 2, &best);
            if (kind >= 0) {
                stop_on_error(kind, best, p0, s.nxt_n, gid_cur, gid_nxt, level_gen - G, st);
                st->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                seconds += st->seconds;
                return status;
            }
            s.nxt_n += Wn;
            s.nxt_words += Ww;
            s.peak_words = std::max(s.peak_words, s.cur_words - consumed + s.nxt_words);
        }
        total_generated += level_gen;
        total_distinct += s.nxt_n;
        st->generated = level_gen;
        st->new_states = s.nxt_n;
        st->new_bytes = s.nxt_words * 4;
        end_level(s, gid_nxt, L);
        if (s.cur_n) {
            depth = L + 1;
        } else {
            finished = true;
            status = RMC_DONE;
            queue_at_end = 0;
        }
        HIPCHK(hipStreamSynchronize(stream));  // the trace copies of the level
        st->total_generated = total_generated;
        st->total_distinct = total_distinct;
        st->queue = s.cur_n;
        st->status = finished ? RMC_DONE : RMC_OK;
        st->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        seconds += st->seconds;
        return st->status;
    }

    // ---- device-driven levels (single GPU) ---------------------------------------------
    // Up to `maxl` levels are enqueued with no host round trip: each level's commit writes the
    // next level's parent count, id bases, ring positions, epoch and table size into the control
    // block that the following kernels read, and stops the loop on an empty level, an error, or a
    // level whose successor bound might not fit the buffers (the host then grows them and
    // carries on).
    int batch_levels() const { return cfg.device_levels ? (int)cfg.device_levels : LREC_CAP; }
    uint64_t dev_parents() const { return std::min<uint64_t>(chunk_parents, 1ull << 15); }
    bool batch_ok() const {
        const Shard &s = sh[0];
        const uint64_t first = s.cur_n * (uint64_t)ks.maxsucc;
        return (W == 1 || (replicated && s.cur_n < shard_min)) && inited && !finished && cfg.device_levels != 1 &&
               s.cur_n > 0 && s.cur_n <= dev_parents() && ring_room(s, first * (uint64_t)ks.RECW_MAX, 0) &&
               seen_room(s, s.T_count + 2 * first);
    }

    // Returns the number of level stats written to out[0..maxl] (the error level included).
    int step_batch(rmc_level_stats *out, int maxl) {
        auto t0 = std::chrono::steady_clock::now();
        Shard &s = sh[0];
        const uint64_t DP = dev_parents(), MS = (uint64_t)ks.maxsucc;
        const int K = std::max(1, std::min(maxl, LREC_CAP));
        // capacities with headroom for several levels; the first level always fits
        uint64_t target = std::min(std::max<uint64_t>(s.cur_n * MS * 32, 1ull << 16), DP * MS);
        maybe_migrate(s, s.T_count + 2 * target);
        if (!ring_room(s, s.cur_n * MS * (uint64_t)ks.RECW_MAX, 0) || !seen_room(s, s.T_count + 2 * s.cur_n * MS))
            return 0;  // the first level no longer fits (the seen set just became compact): host-driven level
        if (s.ring_fixed) target = std::min<uint64_t>(target, (s.rcap - s.cur_words) / (uint64_t)ks.RECW_MAX);
        if (s.Tc) target = std::min<uint64_t>(target, ((uint64_t)(0.9 * (double)s.T_cap) - s.T_count) / 2);
        target = std::max<uint64_t>(target, s.cur_n * MS);  // batch_ok: the first level fits
        s.nxt_words = 0;
        ensure_ring(s, target * (uint64_t)ks.RECW_MAX, 0);
        ensure_off(s.cur_off, s.cur_off_cap, s.cur_n, target);
        ensure_off(s.nxt_off, s.nxt_off_cap, 0, target);
        const int L0 = (int)s.level_start.size();
        const uint64_t gid0 = s.level_start[L0 - 1];
        grow_trace(s, 4 * target);
        grow_seen(s, s.T_count + 2 * target);
        trace_restart(s);
        LevelCtl &h = *s.hctl;
        std::memset(&h, 0, sizeof h);
        h.cur_n = s.cur_n;
        h.gid_cur = gid0;
        h.T_count = s.T_count;
        h.Lmask = std::min(next_pow2(2 * s.cur_n * MS), Lcap_max) - 1;
        h.cur_wbase = s.cur_wbase;
        h.cur_words = s.cur_words;
        h.off_cap = std::min(s.cur_off_cap, s.nxt_off_cap);
        h.rcap = s.rcap;
        h.trace_base = s.tdev;
        h.trace_cap = s.trace_cap;
        h.T_cap = s.Tc ? (uint64_t)((double)s.T_cap * 1.8) : s.T_cap;  // compact: load <= 0.9
        h.chunk_parents = replicated ? std::min<uint64_t>(DP, shard_min - 1) : DP;  // stop before sharding starts
        h.Lcap_max = Lcap_max;
        h.level = (uint32_t)L0;
        renew_election_tags(s, K + 1);
        h.epoch = ++s.epoch;
        h.stop = CTL_RUN;
        h.batch = (uint32_t)K;
        HIPCHK(hipMemcpyAsync(s.ctl, &h, sizeof h, hipMemcpyHostToDevice, stream));
        uint64_t *offs[2] = {s.cur_off, s.nxt_off};
        std::vector<size_t> mark(K);
        // Levels go in groups; after each group a snapshot of the control block is copied back
        // with an event.  Group g + 2 is enqueued only once group g's snapshot says the loop is
        // still running, so the device always has a group queued and at most two groups of
        // no-op launches follow the last level.
        const int GL = 4, ngroups = (K + GL - 1) / GL;
        while ((int)gev.size() < 3) {
            hipEvent_t e;
            HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            gev.push_back(e);
        }
        auto enqueue_group = [&](int g) {
            for (int i = g * GL; i < std::min(K, (g + 1) * GL); i++) {
                mark[i] = evrecs.size();
                KParams Q = chunk_params(s);
                Q.foff = offs[i & 1];
                Q.noff = offs[(i + 1) & 1];
                Q.ctl = s.ctl;
                Q.lrec = s.lrec;
                Q.p_begin = 0;
                Q.p_end = DP;  // grids are sized on the bound; the kernels read the level from ctl
                timed(PH_HASH, [&] { ks.fused(Q, stream); });
                timed(PH_DEDUP, [&] { ks.wincount(Q, DP, stream); });
                timed(PH_MAT, [&] { ks.commit(Q, stream); });
            }
            HIPCHK(hipMemcpyAsync(&s.hsnap[g % 3], s.ctl, sizeof(LevelCtl), hipMemcpyDeviceToHost, stream));
            HIPCHK(hipEventRecord(gev[g % 3], stream));
        };
        int enq = 0;
        for (; enq < std::min(2, ngroups); enq++) enqueue_group(enq);
        for (; enq < ngroups; enq++) {
            HIPCHK(hipEventSynchronize(gev[(enq - 2) % 3]));
            if (s.hsnap[(enq - 2) % 3].stop != CTL_RUN) break;
            enqueue_group(enq);
        }
        for (int i = enq * GL; i < K; i++) mark[i] = evrecs.size();
        HIPCHK(hipMemcpyAsync(s.hctl, s.ctl, sizeof(LevelCtl), hipMemcpyDeviceToHost, stream));
        HIPCHK(hipMemcpyAsync(s.hsum, s.sum, 8 * 8, hipMemcpyDeviceToHost, stream));
        HIPCHK(hipStreamSynchronize(stream));
        HIPCHK(hipGetLastError());
        const LevelCtl c = *s.hctl;
        const int D = (int)c.done_levels;
        if (D > 0 && D <= K) {
            HIPCHK(hipMemcpyAsync(s.hlrec, s.lrec, sizeof(LevelRec) * D, hipMemcpyDeviceToHost, stream));
            HIPCHK(hipStreamSynchronize(stream));
        }
        if (D > K || c.stop == CTL_RUN) throw Fail(RMC_E_STATE, "device level loop did not stop");
        const int nst = D + (c.stop == CTL_ERROR ? 1 : 0);
        for (int i = 0; i < nst; i++) std::memset(&out[i], 0, sizeof out[i]);
        // phase times of the levels that ran (later levels' kernels returned at once)
        for (size_t j = 0; j < evrecs.size(); j++) {
            const int lv = (int)(std::upper_bound(mark.begin(), mark.end(), j) - mark.begin()) - 1;
            if (lv < 0 || lv >= nst) continue;
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, evpool[evrecs[j].a], evpool[evrecs[j].b]));
            out[lv].kernel_ms[evrecs[j].ph] += ms;
            out[lv].kernel_launches[evrecs[j].ph] += 1;
        }
        evrecs.clear();
        evused = 0;
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        for (int i = 0; i < D; i++) {
            const LevelRec &r = s.hlrec[i];
            rmc_level_stats *st = &out[i];
            const int L = L0 + i;
            const uint64_t gid_nxt = s.level_start[L - 1] + r.expanded;
            total_generated += r.generated;
            total_distinct += r.new_states;
            s.T_count += r.new_states;
            if (r.new_states) {
                s.level_start.push_back(gid_nxt);
                depth = L + 1;
            } else {
                finished = true;
                status = RMC_DONE;
                queue_at_end = 0;
            }
            st->level = L;
            st->expanded = r.expanded;
            st->generated = r.generated;
            st->new_states = r.new_states;
            st->new_bytes = r.words * 4;
            st->total_generated = total_generated;
            st->total_distinct = total_distinct;
            st->queue = r.new_states;
            st->status = finished ? RMC_DONE : RMC_OK;
            st->seconds = el / nst;
        }
        if (D & 1) {
            std::swap(s.cur_off, s.nxt_off);
            std::swap(s.cur_off_cap, s.nxt_off_cap);
        }
        s.cur_n = c.cur_n;
        s.cur_wbase = c.cur_wbase;
        s.cur_words = c.cur_words;
        s.nxt_n = 0;
        s.nxt_words = 0;
        s.epoch = c.epoch;
        s.peak_words = std::max(s.peak_words, s.cur_words);
        if (s.T_count != c.T_count) throw Fail(RMC_E_STATE, "device level loop: seen-set count mismatch");
        flush_trace(s, c.gid_cur + c.cur_n);
        seconds += el;
        if (c.stop == CTL_ERROR) {
            // the level the loop stopped in is intact: report its error as the host path does
            rmc_level_stats *st = &out[D];
            st->seconds = el / nst;
            if (s.hsum[2 + ERR_NSLOTS]) throw Fail(RMC_E_CAPACITY, "a state exceeds msg_cap = " + std::to_string(ks.MCAP) + " messages");
            const int L = (int)s.level_start.size();
            st->level = L;
            st->expanded = s.cur_n;
            const uint64_t gid_cur = s.level_start[L - 1];
            flush_trace(s, gid_cur + s.cur_n + s.hsum[1]);  // the error level's winners
            s.T_count += s.hsum[1];
            unsigned long long best;
            const int kind = first_error(s.hsum + 2, &best);
            if (kind < 0) throw Fail(RMC_E_STATE, "device level loop stopped without an error");
            stop_on_error(kind, best, 0, 0, gid_cur, gid_cur + s.cur_n, 0, st);
        }
        HIPCHK(hipStreamSynchronize(stream));
        return nst;
    }

    // TLC's counters at the moment the first error (in -workers 1 order) is reported.
    void stop_on_error(int kind, unsigned long long ek, uint64_t p0, uint64_t nxt_before, uint64_t gid_cur,
                       uint64_t gid_nxt, uint64_t gen_before_chunk, rmc_level_stats *st) {
        Shard &s = sh[0];
        HIPCHK(hipStreamSynchronize(stream));
        const uint64_t p = ek >> 24;                       // level-local parent
        const uint32_t slot = (uint32_t)((ek >> 8) & 0xFFFF);
        const int which = (int)(ek & 0xFF);
        const uint64_t pl = p - p0;
        // successors of the chunk's parents before p, and winners before p
        uint64_t off_p = 0;
        if (pl) {
            std::vector<uint32_t> cn(pl);
            HIPCHK(hipMemcpy(cn.data(), s.cnt, pl * 4, hipMemcpyDeviceToHost));
            for (uint32_t x : cn) off_p += x;
        }
        const uint64_t wbase = (uint64_t)d2h(s.boff + pl / WTILE) + d2h(s.wpos + pl);
        // winners among p's first `upto` successor slots (election table of this chunk)
        auto winners_in = [&](uint32_t upto) -> uint64_t {
            if (!upto) return 0;
            std::vector<uint32_t> ls(upto);
            HIPCHK(hipMemcpy(ls.data(), s.lslot + pl * ks.maxsucc, upto * 4, hipMemcpyDeviceToHost));
            uint64_t w = 0;
            for (uint32_t r = 0; r < upto; r++)
                if (ls[r] < LS_ELECT && ((uint32_t)d2h(s.L + ls[r]) >> 2) == (uint32_t)(pl * ks.maxsucc + r)) w++;
            return w;
        };
        // successors of p, in order, to find the sub-action batch boundaries
        record_to_one(s, p);
        std::vector<uint32_t> keys;
        bool af = false;
        expand_one(&keys, nullptr, nullptr, &af);
        const uint32_t grp = slot >> 7;  // (server, action)
        uint32_t cut = 0, batch_end = 0;
        for (uint32_t k : keys) {
            if ((k >> 7) < grp) cut++;
            if ((k >> 7) <= grp) batch_end++;
        }
        uint64_t gen = gen_before_chunk + off_p;
        uint64_t winners_before;
        if (kind == ERR_INV || kind == ERR_EVAL) {
            gen += batch_end;  // TLC adds the whole sub-action's batch before fingerprinting it
            uint32_t rank_ = 0;
            for (uint32_t k : keys) rank_ += k < slot;
            winners_before = wbase + winners_in(rank_);
            err_ref = gid_nxt + nxt_before + winners_before;
            total_distinct += nxt_before + winners_before + 1;
            queue_at_end = (s.cur_n - p - 1) + nxt_before + winners_before;
            status = kind == ERR_INV ? RMC_VIOLATION : RMC_EVAL_ERROR;
            violated = which;
            depth = (int)s.level_start.size() + 1;
        } else {
            if (kind == ERR_ASSERT) gen += cut;  // the failing sub-action's batch is never counted
            winners_before = wbase + (kind == ERR_ASSERT ? winners_in(cut) : 0);
            err_ref = gid_cur + p;
            total_distinct += nxt_before + winners_before;
            queue_at_end = (s.cur_n - p - 1) + nxt_before + winners_before;
            status = kind == ERR_ASSERT ? RMC_ASSERT : RMC_DEADLOCK;
            if (winners_before + nxt_before > 0) depth = (int)s.level_start.size() + 1;
        }
        err_last_slot = KEY_NONE;
        total_generated += gen;
        st->generated = gen;
        st->new_states = nxt_before + winners_before + ((kind == ERR_INV || kind == ERR_EVAL) ? 1 : 0);
        st->total_generated = total_generated;
        st->total_distinct = total_distinct;
        st->queue = queue_at_end;
        st->status = status;
        finished = true;
        build_trace();
    }

    // ---- sharded level (W > 1): fingerprint-owner partition, exchange, owner election --
    // Order: chunk c of every shard's frontier, then source shard, then TLC order within
    // the source's chunk.  Identical to TLC -workers 1 order when W == 1.
    int step_sharded(rmc_level_stats *st) {
        auto t0 = std::chrono::steady_clock::now();
        const int L = (int)sh[0].level_start.size();
        st->level = L;
        uint64_t agg[2] = {0, 0};
        for (Shard &s : sh) agg[0] = std::max<uint64_t>(agg[0], (s.cur_n + chunk_parents - 1) / chunk_parents);
        for (Shard &s : sh) { st->expanded += s.cur_n; s.nxt_n = 0; s.nxt_words = 0; }
        allreduce(agg, 1, true);
        const uint64_t nchunks = agg[0];
        const size_t NL = sh.size();
        uint64_t level_gen = 0, level_new = 0;
        std::vector<std::vector<uint64_t>> scnt(W, std::vector<uint64_t>(W, 0)), soff(W, std::vector<uint64_t>(W + 1, 0)),
            rcnt, roff(W, std::vector<uint64_t>(W + 1, 0)), swin(W, std::vector<uint64_t>(W, 0)),
            swoff(W, std::vector<uint64_t>(W + 1, 0)), rwin, rwoff(W, std::vector<uint64_t>(W + 1, 0));
        std::vector<const void *> sendp(W);
        std::vector<void *> recvp(W);
        const uint64_t XW = (uint64_t)RECW + 4;
        for (uint64_t c = 0; c < nchunks; c++) {
            // (A) expand, fingerprint, partition by owner -- every local shard as a source
            for (size_t li = 0; li < NL; li++) {
                Shard &s = sh[li];
                const uint64_t gid_cur = s.level_start[L - 1];
                s.p0 = c * chunk_parents;
                s.np = s.cur_n > s.p0 ? std::min<uint64_t>(chunk_parents, s.cur_n - s.p0) : 0;
                s.G = 0;
                std::fill(scnt[li].begin(), scnt[li].end(), 0);
                if (!s.np) continue;
                KParams Q = base(s);
                ring_params(s, Q);
                Q.p_begin = s.p0; Q.p_end = s.p0 + s.np; Q.cnt = s.cnt; Q.off = s.off; Q.fp = s.fp;
                Q.gid_parent_base = gid_cur;
                timed(PH_COUNT, [&] {
                    ks.count(Q, stream);
                    HIPCHK(hipcub::DeviceScan::ExclusiveSum(s.tmp, s.tmp_bytes, s.cnt, s.off, (int)s.np + 1, stream));
                });
                s.G = d2h(s.off + s.np);
                collect_times(st);
                if (!s.G) continue;
                int bits = 0;
                while ((1 << bits) < W) bits++;
                timed(PH_HASH, [&] { ks.hash(Q, stream); });
                timed(PH_XCHG, [&] {
                    HIPCHK(hipMemsetAsync(s.ocnt, 0, 64 * 8, stream));
                    launch_owner_keys(s.fp, s.G, (uint32_t)W, s.okey, s.iota, s.ocnt, stream);
                    HIPCHK(hipcub::DeviceRadixSort::SortPairs(s.tmp, s.tmp_bytes, s.okey, s.okey2, s.iota, s.perm,
                                                              (int)s.G, 0, bits, stream));
                    launch_gather_fp(s.fp, s.perm, s.G, s.sfp, stream);
                });
                HIPCHK(hipMemcpyAsync(s.hsum, s.ocnt, W * 8, hipMemcpyDeviceToHost, stream));
                HIPCHK(hipStreamSynchronize(stream));
                collect_times(st);
                for (int d = 0; d < W; d++) scnt[li][d] = s.hsum[d];
                level_gen += s.G;
            }
            for (size_t li = 0; li < NL; li++) {
                soff[li][0] = 0;
                for (int d = 0; d < W; d++) soff[li][d + 1] = soff[li][d] + scnt[li][d];
            }
            exchange_counts(scnt, rcnt);
            for (size_t li = 0; li < NL; li++) {
                roff[li][0] = 0;
                for (int q = 0; q < W; q++) roff[li][q + 1] = roff[li][q] + rcnt[li][q];
                grow_recv(sh[li], roff[li][W]);
                sendp[li] = sh[li].sfp;
                recvp[li] = sh[li].rfp;
            }
            timed(PH_XCHG, [&] { exchange_items(sendp, scnt, soff, recvp, roff, 16); });
            // (B) owners: seen-set probe + election of the first (source, j) per fingerprint
            for (size_t li = 0; li < NL; li++) {
                Shard &o = sh[li];
                const uint64_t R = roff[li][W];
                if (!R) continue;
                uint32_t Rv = (uint32_t)R;
                HIPCHK(hipMemcpyAsync(o.rcount, &Rv, 4, hipMemcpyHostToDevice, stream));
                uint64_t Lcap = std::min(next_pow2(2 * R), Lcap_max);
                if (R * 2 > Lcap_max) throw Fail(RMC_E_CAPACITY, "owner receive batch exceeds the election table");
                ++o.epoch;
                timed(PH_DEDUP, [&] {
                    launch_dedup(o.rfp, o.rcount, R, o.seen(), o.L, Lcap - 1, o.epoch, o.rlslot, stream);
                    launch_recv_flags(o.rlslot, o.L, R, o.rflag, stream);
                });
                HIPCHK(hipStreamSynchronize(stream));
            }
            // flags back to the sources (reverse exchange)
            for (size_t li = 0; li < NL; li++) { sendp[li] = sh[li].rflag; recvp[li] = sh[li].sflag; }
            {
                std::vector<std::vector<uint64_t>> rev(W, std::vector<uint64_t>(W, 0));
                for (size_t li = 0; li < NL; li++)
                    for (int q = 0; q < W; q++) rev[li][q] = rcnt[li][q];
                timed(PH_XCHG, [&] { exchange_items(sendp, rev, roff, recvp, soff, 4); });
            }
            // (C) sources: winner positions in owner-grouped order, materialize into exchange records
            for (size_t li = 0; li < NL; li++) {
                Shard &s = sh[li];
                std::fill(swin[li].begin(), swin[li].end(), 0);
                if (!s.G) { std::fill(swoff[li].begin(), swoff[li].end(), 0); continue; }
                HIPCHK(hipcub::DeviceScan::ExclusiveSum(s.tmp, s.tmp_bytes, s.sflag, s.spos, (int)s.G + 1, stream));
                std::vector<uint64_t> idx(W + 1);
                for (int d = 0; d <= W; d++) idx[d] = soff[li][d];
                HIPCHK(hipMemcpyAsync(s.pick_idx, idx.data(), (W + 1) * 8, hipMemcpyHostToDevice, stream));
                launch_pick(s.spos, s.pick_idx, W + 1, s.sum, stream);
                HIPCHK(hipMemcpyAsync(s.hsum, s.sum, (W + 1) * 8, hipMemcpyDeviceToHost, stream));
                HIPCHK(hipStreamSynchronize(stream));
                for (int d = 0; d <= W; d++) swoff[li][d] = s.hsum[d];
                for (int d = 0; d < W; d++) swin[li][d] = swoff[li][d + 1] - swoff[li][d];
                grow_plain(s.sx, s.sx_cap, swoff[li][W] * XW + 1);
                launch_scatter_flags(s.perm, s.sflag, s.spos, s.G, s.wflag, s.wpos, stream);
                KParams Q = base(s);
                ring_params(s, Q);
                Q.p_begin = s.p0; Q.p_end = s.p0 + s.np; Q.cnt = s.cnt; Q.off = s.off; Q.fp = s.fp;
                Q.wflag = s.wflag; Q.wpos = s.wpos; Q.xrec = s.sx; Q.gid_parent_base = s.level_start[L - 1];
                timed(PH_MAT, [&] { ks.materialize(Q, stream); });
            }
            exchange_counts(swin, rwin);
            for (size_t li = 0; li < NL; li++) {
                rwoff[li][0] = 0;
                for (int q = 0; q < W; q++) rwoff[li][q + 1] = rwoff[li][q] + rwin[li][q];
                grow_plain(sh[li].rx, sh[li].rx_cap, rwoff[li][W] * XW + 1);
                sendp[li] = sh[li].sx;
                recvp[li] = sh[li].rx;
            }
            timed(PH_XCHG, [&] { exchange_items(sendp, swin, swoff, recvp, rwoff, XW * 4); });
            // (D) owners: append winners (source-major) to the next level, seen-set insert
            for (size_t li = 0; li < NL; li++) {
                Shard &o = sh[li];
                const uint64_t n = rwoff[li][W];
                const uint64_t gid_nxt = o.level_start[L - 1] + o.cur_n;
                if (n) {
                    ensure_ring(o, n * (uint64_t)RECW, 0);
                    ensure_off(o.nxt_off, o.nxt_off_cap, o.nxt_n, o.nxt_n + n);
                    grow_trace(o, n);
                    grow_seen(o, o.T_count + n);
                    trace_restart(o);
                    const uint64_t tb = gid_nxt + o.nxt_n - o.tdev;  // == 0: everything earlier is flushed
                    timed(PH_OTHER, [&] {
                        for (int q = 0; q < W; q++) {
                            const uint64_t k = rwin[li][q];
                            if (!k) continue;
                            launch_accept(o.rx + rwoff[li][q] * XW, k, (uint32_t)RECW, o.R, o.rcap, o.nbase(),
                                          o.nxt_words + rwoff[li][q] * (uint64_t)RECW, o.nxt_off + o.nxt_n + rwoff[li][q],
                                          o.par + tb + rwoff[li][q], o.pslot + tb + rwoff[li][q], (uint64_t)q << 48, stream);
                        }
                        launch_insert_flagged(o.rfp, o.rflag, roff[li][W], o.seen(), stream);
                    });
                    flush_trace(o, gid_nxt + o.nxt_n + n);
                    o.nxt_n += n;
                    o.nxt_words += n * (uint64_t)RECW;
                    o.T_count += n;
                    level_new += n;
                }
            }
            // errors: first in (source shard, parent, slot) order
            std::vector<uint64_t> ebuf(2 * W, ~0ull);
            for (size_t li = 0; li < NL; li++) {
                Shard &s = sh[li];
                HIPCHK(hipMemcpyAsync(s.hsum, s.err, ERR_NSLOTS * 8, hipMemcpyDeviceToHost, stream));
                HIPCHK(hipMemcpyAsync(s.hsum + 8, s.flags, 4, hipMemcpyDeviceToHost, stream));
                HIPCHK(hipStreamSynchronize(stream));
                if ((uint32_t)s.hsum[8]) throw Fail(RMC_E_CAPACITY, "a state exceeds msg_cap = " + std::to_string(ks.MCAP) + " messages");
                unsigned long long best;
                const int kind = first_error(s.hsum, &best);
                if (kind >= 0) { ebuf[2 * s.id] = (uint64_t)kind; ebuf[2 * s.id + 1] = best; }
                HIPCHK(hipMemsetAsync(s.err, 0xFF, ERR_NSLOTS * 8, stream));
            }
            if (!virt && W > 1) {
                // gather every rank's (kind, key): ranks contribute only their own slots
                std::vector<uint64_t> g(2 * W, 0);
                for (int q = 0; q < 2 * W; q++) g[q] = (q / 2 == rank) ? ebuf[q] + 1 : 0;  // +1: ~0 -> 0
                allreduce(g.data(), 2 * W, false);
                for (int q = 0; q < 2 * W; q++) ebuf[q] = g[q] - 1;
            }
            for (int q = 0; q < W; q++) {
                if (ebuf[2 * q] == ~0ull) continue;
                uint64_t glob[2] = {level_gen, level_new};
                allreduce(glob, 2, false);
                stop_sharded(q, (int)ebuf[2 * q], ebuf[2 * q + 1], L, glob[0], glob[1], st);
                st->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                seconds += st->seconds;
                return status;
            }
        }
        uint64_t glob[2] = {level_gen, level_new};
        allreduce(glob, 2, false);
        total_generated += glob[0];
        total_distinct += glob[1];
        st->generated = glob[0];
        st->new_states = glob[1];
        for (Shard &s : sh) {
            const uint64_t gid_nxt = s.level_start[L - 1] + s.cur_n;
            st->new_bytes += s.nxt_words * 4;
            s.peak_words = std::max(s.peak_words, s.cur_words + s.nxt_words);
            end_level(s, gid_nxt, L);
            if (!s.cur_n) s.level_start.push_back(gid_nxt);  // every shard keeps the same level count
        }
        HIPCHK(hipStreamSynchronize(stream));
        if (glob[1]) {
            depth = L + 1;
        } else {
            finished = true;
            status = RMC_DONE;
            queue_at_end = 0;
        }
        st->total_generated = total_generated;
        st->total_distinct = total_distinct;
        st->queue = glob[1];
        st->status = finished ? RMC_DONE : RMC_OK;
        st->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        seconds += st->seconds;
        return st->status;
    }

    // Sharded stop: the error's shard q, kind, key (parent in q's level, slot).  Counters are
    // those at the end of the chunk (every chunk is processed by all shards together).
    void stop_sharded(int q, int kind, unsigned long long ek, int L, uint64_t gen, uint64_t nw, rmc_level_stats *st) {
        const uint64_t p = ek >> 24;
        const uint32_t slot = (uint32_t)((ek >> 8) & 0xFFFF);
        total_generated += gen;
        total_distinct += nw;
        uint64_t gid_cur = 0;
        for (Shard &s : sh)
            if (s.id == q) gid_cur = s.level_start[L - 1];
        uint64_t g[1] = {virt ? gid_cur : (q == rank ? gid_cur : 0)};
        allreduce(g, 1, false);
        err_ref = ((uint64_t)q << 48) | (g[0] + p);
        if (kind == ERR_INV || kind == ERR_EVAL) {
            status = kind == ERR_INV ? RMC_VIOLATION : RMC_EVAL_ERROR;
            violated = (int)(ek & 0xFF);
            err_last_slot = slot;
            depth = L + 1;
        } else {
            status = kind == ERR_ASSERT ? RMC_ASSERT : RMC_DEADLOCK;
            err_last_slot = KEY_NONE;
        }
        queue_at_end = 0;
        st->generated = gen;
        st->new_states = nw;
        st->total_generated = total_generated;
        st->total_distinct = total_distinct;
        st->status = status;
        finished = true;
        build_trace();
    }

    // parent reference and slot of a state (shard << 48 | local gid), from whichever rank holds it
    void fetch_par(uint64_t ref, uint64_t *par, uint16_t *slot) {
        const int q = (int)(ref >> 48);
        const uint64_t gid = ref & ((1ull << 48) - 1);
        uint64_t v[2] = {0, 0};
        for (Shard &s : sh)
            if (s.id == q) {
                if (gid >= s.tflushed) throw Fail(RMC_E_STATE, "trace entry not on the host");
                v[0] = s.hpar.get(gid) + 1;  // +1: the Init sentinel ~0 travels as 0
                v[1] = s.hslot.get(gid);
            }
        allreduce(v, 2, false);
        *par = v[0] - 1;
        *slot = (uint16_t)v[1];
    }

    // Walk parent pointers from err_ref to Init, then replay the slots from Init.
    void build_trace() {
        HIPCHK(hipStreamSynchronize(stream));  // pending trace copies
        std::vector<uint16_t> slots;
        if (err_last_slot != KEY_NONE) slots.push_back((uint16_t)err_last_slot);
        uint64_t g = err_ref;
        for (;;) {
            uint64_t par;
            uint16_t sl;
            fetch_par(g, &par, &sl);
            if (par == ~0ull) break;
            slots.push_back(sl);
            g = par;
            if (slots.size() > 100000) throw Fail(RMC_E_STATE, "corrupt parent chain");
        }
        std::reverse(slots.begin(), slots.end());
        trace.clear();
        std::vector<uint32_t> rec = init_record();
        trace.push_back({unpack(rec.data()), -1, -1, -1});
        for (uint16_t sk : slots) {
            HIPCHK(hipMemcpy(d_one, rec.data(), RECW * 4, hipMemcpyHostToDevice));
            std::vector<uint32_t> keys, recs;
            bool af = false;
            uint32_t cnt = expand_one(&keys, &recs, nullptr, &af);
            uint32_t i = 0;
            while (i < cnt && keys[i] != sk) i++;
            if (i == cnt) throw Fail(RMC_E_STATE, "trace replay: slot not enabled");
            std::memcpy(rec.data(), recs.data() + (size_t)i * RECW, RECW * 4);
            trace.push_back({unpack(rec.data()), (int32_t)key_action(sk), (int32_t)key_server(sk),
                             (int32_t)key_witness(sk)});
        }
    }

    // ---- checkpoint / resume (rmc_checkpoint, rmc_resume) --------------------------------
    struct CkptHeader {
        uint64_t magic;
        uint32_t abi, recw;
        int32_t n, v, e, r;
        uint32_t invariants, inv_order;
        int32_t check_deadlock, spec_variant, no_symmetry, msg_cap, depth, compact;
        uint64_t scheme;
        uint64_t total_generated, total_distinct, T_cap, T_count, cur_n, cur_words, n_levels, trace_n;
        uint32_t epoch, pad;
        double seconds;
        uint64_t check;  // checksum of every field above
    };
    static constexpr uint64_t CKPT_MAGIC = 0x3250434b434d52ull;  // "RMCKCP2"

    CkptHeader ckpt_header() const {
        CkptHeader h{};
        h.magic = CKPT_MAGIC;
        h.abi = RMC_ABI_VERSION;
        h.recw = (uint32_t)RECW;
        h.n = cfg.n_servers; h.v = cfg.n_vals; h.e = cfg.max_election; h.r = cfg.max_restart;
        h.invariants = cfg.invariants;
        h.inv_order = inv_order;
        h.check_deadlock = cfg.check_deadlock; h.spec_variant = cfg.spec_variant;
        h.no_symmetry = cfg.no_symmetry; h.msg_cap = ks.MCAP;
        h.scheme = scheme_hash;
        return h;
    }
    static uint64_t header_check(const CkptHeader &h) {
        const unsigned char *b = reinterpret_cast<const unsigned char *>(&h);
        uint64_t x = 0xcbf29ce484222325ull;
        for (size_t i = 0; i < offsetof(CkptHeader, check); i++) x = (x ^ b[i]) * 0x100000001b3ull;
        return x;
    }

    // device <-> file in bounded pieces through one host buffer
    template <class F>
    void stream_bytes(void *dev, uint64_t bytes, F &&io) {
        std::vector<char> buf((size_t)std::min<uint64_t>(bytes, 64ull << 20));
        for (uint64_t o = 0; o < bytes; o += buf.size()) {
            const size_t k = (size_t)std::min<uint64_t>(buf.size(), bytes - o);
            io((char *)dev + o, buf.data(), k);
        }
    }

    // Written to path + ".tmp", flushed to disk, then renamed over path: the previous checkpoint
    // survives until the new one is complete.
    void checkpoint(const char *path) {
        if (W != 1) throw Fail(RMC_E_ARG, "checkpoint: single-GPU runs only");
        if (!inited || finished) throw Fail(RMC_E_STATE, "checkpoint: between levels of a started, unfinished run");
        Shard &s = sh[0];
        HIPCHK(hipStreamSynchronize(stream));
        CkptHeader h = ckpt_header();
        h.depth = depth;
        h.compact = s.Tc ? 1 : 0;
        h.total_generated = total_generated; h.total_distinct = total_distinct;
        h.T_cap = s.T_cap; h.T_count = s.T_count; h.cur_n = s.cur_n; h.cur_words = s.cur_words;
        h.n_levels = s.level_start.size();
        h.trace_n = s.level_start.back() + s.cur_n;  // every state found so far has a global id below
        h.epoch = s.epoch;
        h.seconds = seconds;
        h.check = header_check(h);
        if (s.tflushed != h.trace_n) throw Fail(RMC_E_STATE, "checkpoint: trace not flushed");
        const std::string tmp = std::string(path) + ".tmp";
        FILE *f = std::fopen(tmp.c_str(), "wb");
        if (!f) throw Fail(RMC_E_ARG, std::string("checkpoint: cannot write ") + tmp);
        bool ok = std::fwrite(&h, sizeof h, 1, f) == 1 &&
                  std::fwrite(s.level_start.data(), 8, s.level_start.size(), f) == s.level_start.size();
        auto out = [&](void *dev, char *host, size_t k) {
            HIPCHK(hipMemcpy(host, dev, k, hipMemcpyDeviceToHost));
            ok = ok && std::fwrite(host, 1, k, f) == k;
        };
        if (s.Tc) stream_bytes(s.Tc, h.T_cap * 8, out);
        else stream_bytes(s.T, h.T_cap * 16, out);
        // the current level, linearised
        uint32_t *lin = dmalloc<uint32_t>(std::max<uint64_t>(h.cur_words, 1));
        ring_copy_out(s, s.cur_wbase, h.cur_words, lin);
        HIPCHK(hipStreamSynchronize(stream));
        stream_bytes(lin, h.cur_words * 4, out);
        dfree(lin);
        stream_bytes(s.cur_off, h.cur_n * 8, out);
        s.hpar.for_range(0, h.trace_n, [&](const uint64_t *p, uint64_t k) { ok = ok && std::fwrite(p, 8, k, f) == k; });
        s.hslot.for_range(0, h.trace_n, [&](const uint16_t *p, uint64_t k) { ok = ok && std::fwrite(p, 2, k, f) == k; });
        ok = std::fflush(f) == 0 && ok;
        ok = ok && fsync(fileno(f)) == 0;
        ok = (std::fclose(f) == 0) && ok;
        if (!ok) {
            std::remove(tmp.c_str());
            throw Fail(RMC_E_ARG, std::string("checkpoint: short write to ") + tmp);
        }
        if (std::rename(tmp.c_str(), path) != 0) throw Fail(RMC_E_ARG, std::string("checkpoint: cannot rename to ") + path);
    }

    void resume(const char *path) {
        if (W != 1) throw Fail(RMC_E_ARG, "resume: single-GPU runs only");
        if (inited) throw Fail(RMC_E_STATE, "resume: needs a context not yet initialised (rmc_create or rmc_reset)");
        FILE *f = std::fopen(path, "rb");
        if (!f) throw Fail(RMC_E_ARG, std::string("resume: cannot read ") + path);
        CkptHeader h{};
        const CkptHeader want = ckpt_header();
        bool ok = std::fread(&h, sizeof h, 1, f) == 1;
        if (!ok || h.magic != CKPT_MAGIC || h.abi != want.abi || h.recw != want.recw || h.n != want.n ||
            h.v != want.v || h.e != want.e || h.r != want.r || h.invariants != want.invariants ||
            h.inv_order != want.inv_order || h.check_deadlock != want.check_deadlock ||
            h.spec_variant != want.spec_variant || h.no_symmetry != want.no_symmetry || h.msg_cap != want.msg_cap) {
            std::fclose(f);
            throw Fail(RMC_E_ARG, std::string("resume: ") + path + " is not a checkpoint of this configuration");
        }
        if (h.scheme != want.scheme) {
            std::fclose(f);
            throw Fail(RMC_E_ARG, std::string("resume: ") + path + " was written with another fingerprint scheme");
        }
        // the header's own consistency, before anything is allocated from it
        if (h.check != header_check(h) || h.n_levels == 0 || h.n_levels > 100000 ||
            (!h.compact && (h.T_cap & (h.T_cap - 1)) != 0) || h.T_cap == 0 ||
            h.T_count >= h.T_cap || h.T_count > h.trace_n || h.cur_words > h.cur_n * (uint64_t)RECW ||
            h.cur_words < h.cur_n * (uint64_t)ks.CCW) {
            std::fclose(f);
            throw Fail(RMC_E_ARG, std::string("resume: ") + path + " has an inconsistent header");
        }
        std::vector<uint64_t> ls(h.n_levels);
        ok = std::fread(ls.data(), 8, ls.size(), f) == ls.size();
        for (size_t i = 1; ok && i < ls.size(); i++) ok = ls[i] > ls[i - 1];
        if (!ok || ls.back() + h.cur_n != h.trace_n) {
            std::fclose(f);
            throw Fail(RMC_E_ARG, std::string("resume: ") + path + " has an inconsistent level table");
        }
        Shard &s = sh[0];
        dfree(s.T);
        dfree(s.Tc);
        if (h.compact) {
            s.Tc = dmalloc<unsigned long long>(h.T_cap);
            s.ring_fixed = false;  // re-derived below
        } else {
            s.T = dmalloc<ulonglong2>(h.T_cap);
        }
        s.T_cap = h.T_cap;
        s.cur_wbase = 0;
        s.cur_words = 0;
        s.nxt_words = 0;
        ensure_ring(s, h.cur_words + 1, 0);
        ensure_off(s.cur_off, s.cur_off_cap, 0, std::max<uint64_t>(h.cur_n, 1));
        auto in = [&](void *dev, char *host, size_t k) {
            ok = ok && std::fread(host, 1, k, f) == k;
            if (ok) HIPCHK(hipMemcpy(dev, host, k, hipMemcpyHostToDevice));
        };
        if (s.Tc) stream_bytes(s.Tc, h.T_cap * 8, in);
        else stream_bytes(s.T, h.T_cap * 16, in);
        stream_bytes(s.R, h.cur_words * 4, in);
        stream_bytes(s.cur_off, h.cur_n * 8, in);
        s.hpar.reserve_to(h.trace_n);
        s.hslot.reserve_to(h.trace_n);
        for (uint64_t i = 0; ok && i < h.trace_n;) {
            const uint64_t k = std::min<uint64_t>(h.trace_n - i, HostArr<uint64_t>::B - i % HostArr<uint64_t>::B);
            ok = std::fread(s.hpar.blk[i / HostArr<uint64_t>::B].p + i % HostArr<uint64_t>::B, 8, k, f) == k;
            i += k;
        }
        for (uint64_t i = 0; ok && i < h.trace_n;) {
            const uint64_t k = std::min<uint64_t>(h.trace_n - i, HostArr<uint16_t>::B - i % HostArr<uint16_t>::B);
            ok = std::fread(s.hslot.blk[i / HostArr<uint16_t>::B].p + i % HostArr<uint16_t>::B, 2, k, f) == k;
            i += k;
        }
        std::fclose(f);
        if (!ok) throw Fail(RMC_E_ARG, std::string("resume: ") + path + " is truncated");
        s.hpar.n = s.hslot.n = h.trace_n;
        s.tflushed = h.trace_n;
        s.level_start = ls;
        s.cur_n = h.cur_n;
        s.cur_words = h.cur_words;
        s.T_count = h.T_count;
        s.epoch = std::max(s.epoch, h.epoch);
        if (s.Tc) fix_ring(s, 1);  // a compact seen set means a large run: the ring goes to its budget
        total_generated = h.total_generated;
        total_distinct = h.total_distinct;
        depth = h.depth;
        seconds = h.seconds;
        trace.clear();
        status = RMC_OK;
        violated = -1;
        err_ref = 0;
        err_last_slot = KEY_NONE;
        inited = true;
        finished = s.cur_n == 0;
        if (finished) { status = RMC_DONE; queue_at_end = 0; }
    }

    // Forget every explored state but keep all device buffers (repeat runs, benchmarks).
    void reset() {
        HIPCHK(hipStreamSynchronize(stream));
        for (Shard &s : sh) {
            if (s.Tc) HIPCHK(hipMemsetAsync(s.Tc, 0, s.T_cap * 8, stream));
            else HIPCHK(hipMemsetAsync(s.T, 0, s.T_cap * 16, stream));
            s.T_count = 0;
            s.cur_n = s.nxt_n = 0;
            s.cur_wbase = s.cur_words = s.nxt_words = 0;
            s.tflushed = 0;
            s.hpar.n = s.hslot.n = 0;
            s.level_start.clear();
        }
        HIPCHK(hipStreamSynchronize(stream));
        trace.clear();
        inited = finished = false;
        status = RMC_OK;
        depth = 0;
        total_generated = total_distinct = queue_at_end = 0;
        violated = -1;
        err_ref = 0;
        err_last_slot = KEY_NONE;
        seconds = 0;
    }

    void result(rmc_result *r) const {
        std::memset(r, 0, sizeof *r);
        r->status = finished ? status : RMC_OK;
        r->depth = depth;
        r->generated = total_generated;
        r->distinct = total_distinct;
        uint64_t q = 0;
        for (const Shard &s : sh) q += s.cur_n;
        r->queue = finished ? queue_at_end : q;
        r->violated = violated;
        r->trace_len = (uint32_t)trace.size();
        r->seconds = seconds;
        for (const Shard &s : sh) {
            r->seen_slots += s.T_cap;
            r->seen_slot_bytes = s.Tc ? 8 : 16;
            r->frontier_ring_bytes += s.rcap * 4;
            r->frontier_peak_bytes += s.peak_words * 4;
        }
    }
};

// ------------------------------------------------------------------------------------------
// C-ABI
// ------------------------------------------------------------------------------------------
template <class F>
static int guarded(rmc_ctx *c, F &&f) {
    if (!c) return RMC_E_ARG;
    try {
        return f();
    } catch (const Fail &e) {
        c->err = e.msg;
        return e.code;
    } catch (const std::exception &e) {
        c->err = e.what();
        return RMC_E_MEMORY;
    }
}

extern "C" {

int rmc_abi_version(void) { return RMC_ABI_VERSION; }

int rmc_comm_unique_id(void *out128) {
    if (!out128) return RMC_E_ARG;
#ifdef RMC_WITH_RCCL
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return RMC_E_COMM;
    static_assert(sizeof(id) <= 128, "ncclUniqueId larger than 128 bytes");
    static_assert(sizeof(rmc_config) == 120, "rmc_config layout (ABI 3) changed: update INTEGRATION.md and raftmc");
    std::memset(out128, 0, 128);
    std::memcpy(out128, &id, sizeof id);
    return RMC_OK;
#else
    return RMC_E_COMM;
#endif
}

int rmc_create(const rmc_config *cfg, void **out) {
    if (!cfg || !out) return RMC_E_ARG;
    *out = nullptr;
    rmc_ctx *c = new rmc_ctx();
    c->cfg = *cfg;
    int rc = guarded(c, [&] {
        c->setup();
        return RMC_OK;
    });
    if (rc != RMC_OK) {
        std::fprintf(stderr, "rmc_create: %s\n", c->err.c_str());
        c->release();
        delete c;
        return rc;
    }
    *out = c;
    return RMC_OK;
}

int rmc_init(void *ctx, rmc_level_stats *st) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    return guarded(c, [&] { return c->init(st); });
}

int rmc_step(void *ctx, rmc_level_stats *st) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    return guarded(c, [&] { return c->step(st); });
}

int rmc_run(void *ctx, rmc_result *res) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    return guarded(c, [&] {
        if (!c->inited) c->init(nullptr);
        std::vector<rmc_level_stats> tmp(LREC_CAP + 1);
        while (!c->finished) {
            if (!c->batch_ok() || c->step_batch(tmp.data(), c->batch_levels()) == 0) c->step(nullptr);
        }
        if (res) c->result(res);
        return c->status;
    });
}

int rmc_steps(void *ctx, rmc_level_stats *levels, uint32_t cap, uint32_t *n) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    if (!levels || !cap || !n) return RMC_E_ARG;
    *n = 0;
    return guarded(c, [&] {
        if (!c->inited) throw Fail(RMC_E_STATE, "rmc_steps before rmc_init");
        if (c->finished) return c->status == RMC_OK ? RMC_DONE : c->status;
        if (c->batch_ok() && cap > 1) {
            const int k = c->step_batch(levels, std::min<int>(c->batch_levels(), (int)cap - 1));
            if (k > 0) {
                *n = (uint32_t)k;
                return levels[k - 1].status;
            }
        }
        const int rc = c->step(levels);
        *n = 1;
        return rc;
    });
}

int rmc_set_timing(void *ctx, uint32_t phases) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    return guarded(c, [&] {
        c->timing_on = phases != 0;
        if (phases != 0) c->cfg.timing_phases = phases == 0xFFFFFFFFu ? 0u : phases;
        return RMC_OK;
    });
}

int rmc_reset(void *ctx) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    return guarded(c, [&] {
        c->reset();
        return RMC_OK;
    });
}

int rmc_checkpoint(void *ctx, const char *path) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    if (!path) return RMC_E_ARG;
    return guarded(c, [&] {
        c->checkpoint(path);
        return RMC_OK;
    });
}

int rmc_resume(void *ctx, const char *path) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    if (!path) return RMC_E_ARG;
    return guarded(c, [&] {
        c->resume(path);
        return RMC_OK;
    });
}

int rmc_run_levels(void *ctx, rmc_level_stats *levels, uint32_t cap, uint32_t *n_levels, rmc_result *res) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    return guarded(c, [&] {
        uint32_t n = 0;
        rmc_level_stats tmp;
        if (!c->inited) {
            c->init(n < cap && levels ? &levels[n] : &tmp);
            n++;
        }
        std::vector<rmc_level_stats> bt(LREC_CAP + 1);
        while (!c->finished) {
            const int k = c->batch_ok() ? c->step_batch(bt.data(), c->batch_levels()) : 0;
            if (k > 0) {
                for (int i = 0; i < k; i++, n++)
                    if (n < cap && levels) levels[n] = bt[i];
            } else {
                c->step(n < cap && levels ? &levels[n] : &tmp);
                n++;
            }
        }
        if (n_levels) *n_levels = n < cap ? n : cap;
        if (res) c->result(res);
        return c->status;
    });
}

int rmc_get_result(void *ctx, rmc_result *res) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    if (!res) return RMC_E_ARG;
    return guarded(c, [&] {
        c->result(res);
        return RMC_OK;
    });
}

int rmc_trace_len(void *ctx, uint32_t *len) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    if (!len) return RMC_E_ARG;
    return guarded(c, [&] {
        *len = (uint32_t)c->trace.size();
        return RMC_OK;
    });
}

int rmc_trace_state(void *ctx, uint32_t i, int32_t *unpacked, size_t cap, int32_t *action, int32_t *server,
                    int32_t *witness) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    return guarded(c, [&] {
        if (i >= c->trace.size()) throw Fail(RMC_E_ARG, "trace index out of range");
        const TraceStep &t = c->trace[i];
        if (t.unpacked.size() > cap) throw Fail(RMC_E_ARG, "buffer too small");
        std::memcpy(unpacked, t.unpacked.data(), t.unpacked.size() * 4);
        if (action) *action = t.action;
        if (server) *server = t.server;
        if (witness) *witness = t.witness;
        return (int)t.unpacked.size();
    });
}

const char *rmc_last_error(void *ctx) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    return c ? c->err.c_str() : "null context";
}

void rmc_destroy(void *ctx) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    if (!c) return;
    c->release();
    delete c;
}

int rmc_successors(void *ctx, const int32_t *unpacked, int32_t *out, size_t stride, uint32_t cap, uint32_t *keys,
                   uint64_t *fps, uint32_t *count) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    return guarded(c, [&] {
        std::vector<uint32_t> rec(c->RECW);
        c->pack(unpacked, rec.data());
        HIPCHK(hipMemcpy(c->d_one, rec.data(), c->RECW * 4, hipMemcpyHostToDevice));
        std::vector<uint32_t> ks, recs;
        std::vector<ulonglong2> f;
        bool af = false;
        uint32_t n = c->expand_one(&ks, &recs, &f, &af);
        if (af) {
            if (count) *count = 0;
            return RMC_ASSERT;
        }
        if (count) *count = n;
        if (n > cap) throw Fail(RMC_E_ARG, "successor buffer too small");
        for (uint32_t i = 0; i < n; i++) {
            std::vector<int32_t> u = c->unpack(recs.data() + (size_t)i * c->RECW);
            if (out) {
                if (u.size() > stride) throw Fail(RMC_E_ARG, "stride too small");
                std::memcpy(out + (size_t)i * stride, u.data(), u.size() * 4);
            }
            if (keys) keys[i] = (key_server(ks[i]) << 24) | (key_action(ks[i]) << 16) | key_witness(ks[i]);
            if (fps) { fps[2 * i] = f[i].x; fps[2 * i + 1] = f[i].y; }
        }
        return RMC_OK;
    });
}

int rmc_fingerprint(void *ctx, const int32_t *unpacked, uint64_t fp[2]) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    return guarded(c, [&] {
        std::vector<uint32_t> rec(c->RECW);
        c->pack(unpacked, rec.data());
        HIPCHK(hipMemcpy(c->d_one, rec.data(), c->RECW * 4, hipMemcpyHostToDevice));
        KParams P = c->base(c->sh[0]);
        P.front = c->d_one;
        P.fp = c->d_fp1;
        c->ks.fp_states(P, 1, c->stream);
        ulonglong2 f = c->d2h(c->d_fp1);
        fp[0] = f.x;
        fp[1] = f.y;
        return RMC_OK;
    });
}

int rmc_eval_invariant(void *ctx, const int32_t *unpacked, uint32_t bit, int32_t *value) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    return guarded(c, [&] {
        if (bit >= 7 || !value) throw Fail(RMC_E_ARG, "bad invariant bit");
        std::vector<uint32_t> rec(c->RECW);
        c->pack(unpacked, rec.data());
        HIPCHK(hipMemcpy(c->d_one, rec.data(), c->RECW * 4, hipMemcpyHostToDevice));
        KParams P = c->base(c->sh[0]);
        P.front = c->d_one;
        c->ks.inv_states(P, 1, c->d_inv, c->stream);
        int32_t iv[7];
        HIPCHK(hipMemcpyAsync(iv, c->d_inv, sizeof iv, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        *value = iv[bit];
        return iv[bit] < 0 ? RMC_EVAL_ERROR : RMC_OK;
    });
}

}  // extern "C"
