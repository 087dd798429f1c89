// rmc_engine.hip -- host orchestration of the level-synchronous GPU BFS behind the C-ABI.
//
// Replaces TLC's ModelChecker / Worker loop (run by myrun.sh:3) for Raft.tla:
//   * level L's states live in HBM as packed records (rmc_spec.h), in TLC -workers 1
//     FIFO order;
//   * a level is expanded in chunks of parents: COUNT -> scan -> HASH -> dedup
//     (seen set + first-in-TLC-order election) -> scan -> MATERIALIZE;
//   * new states are appended to the next level in the order TLC would have
//     enqueued them, so discovery order (and therefore which concrete state
//     represents a VIEW class) matches TLC with one worker;
//   * the first error in TLC order (invariant / eval error / Assert / deadlock)
//     stops the search with TLC's counters at that point and a replayable trace.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "rmc.h"
#include "rmc_kernels.h"
#include "rmc_spec.h"

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
            // per-message hash of everything but src/dst (those are positions in the pair sums)
            const uint64_t body = items[id].info & ~0xFCull;
            gmsg[id].x = mix64(SEED_MSG ^ mix64(body * 0x9e3779b97f4a7c15ULL + 1));
            gmsg[id].y = mix64((SEED_MSG + 0x632be59bd9b4e019ULL) ^ mix64(body * 0xc2b2ae3d27d4eb4fULL + 7));
        }
        if (info.empty()) { info.push_back(0); gmsg.push_back(make_ulonglong2(0, 0)); }
    }
};

template <class T>
T *dmalloc(size_t n) {
    void *p = nullptr;
    if (n == 0) n = 1;
    hipError_t e = hipMalloc(&p, n * sizeof(T));
    if (e != hipSuccess)
        throw Fail(RMC_E_MEMORY, "hipMalloc(" + std::to_string(n * sizeof(T)) + " B): " + hipGetErrorString(e));
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

enum Phase { PH_COUNT = 0, PH_HASH = 1, PH_DEDUP = 2, PH_MAT = 3, PH_XCHG = 4, PH_OTHER = 5 };

struct TraceStep {
    std::vector<int32_t> unpacked;
    int32_t action, server, witness;
};

}  // namespace

struct rmc_ctx {
    rmc_config cfg{};
    KernelSet ks{};
    Universe U;
    std::string err;
    hipStream_t stream = nullptr;
    int N = 0, V = 0, RECW = 0;

    // device tables
    uint32_t *d_info = nullptr;
    uint16_t *d_nat2id = nullptr;
    ulonglong2 *d_gmsg = nullptr;
    uint8_t *d_perms = nullptr;
    uint64_t *d_seeds = nullptr;
    int np = 0;

    // frontier
    uint32_t *d_cur = nullptr, *d_nxt = nullptr;
    uint64_t cur_n = 0, cur_cap = 0, nxt_cap = 0;

    // chunk buffers
    uint64_t chunk_parents = 0, Gcap = 0;
    uint32_t *d_cnt = nullptr, *d_off = nullptr, *d_lslot = nullptr, *d_wflag = nullptr, *d_wpos = nullptr;
    unsigned long long *d_L = nullptr;  // chunk dedup table, (epoch << 32) | j
    uint64_t Lcap_max = 0;
    uint32_t epoch = 0;
    unsigned long long *d_sum = nullptr, *h_sum = nullptr;  // per-chunk summary (G, W, errors, flags)
    std::vector<hipEvent_t> evpool;
    struct EvRec { int ph; int a, b; };
    std::vector<EvRec> evrecs;
    int evused = 0;
    ulonglong2 *d_fp = nullptr;
    void *d_tmp = nullptr;
    size_t tmp_bytes = 0;

    // seen set
    ulonglong2 *d_T = nullptr;
    uint64_t T_cap = 0, T_count = 0;

    // trace
    uint64_t *d_par = nullptr;
    uint16_t *d_pslot = nullptr;
    uint64_t trace_cap = 0;
    std::vector<uint64_t> level_start;  // gid of each level's first state

    // errors / flags
    unsigned long long *d_err = nullptr;
    uint32_t *d_flags = nullptr;

    // scratch for single-state hooks
    uint32_t *d_one = nullptr, *d_out = nullptr, *d_keys = nullptr, *d_cnt1 = nullptr;
    ulonglong2 *d_fp1 = nullptr;
    int32_t *d_inv = nullptr;

    // progress
    bool inited = false, finished = false;
    int status = RMC_OK;
    int depth = 0;
    uint64_t total_generated = 0, total_distinct = 0, queue_at_end = 0;
    int violated = -1;
    uint64_t err_gid = 0;  // state whose trace is reported
    std::vector<TraceStep> trace;
    double seconds = 0;

    hipEvent_t ev0 = nullptr, ev1 = nullptr;

    KParams base() const {
        KParams P{};
        P.d = U.d;
        P.E = cfg.max_election;
        P.R = cfg.max_restart;
        P.seeded = cfg.spec_variant == RMC_SPEC_SEEDED;
        P.check_deadlock = cfg.check_deadlock;
        P.inv_mask = cfg.invariants;
        P.t.info = d_info;
        P.t.nat2id = d_nat2id;
        P.t.gmsg = d_gmsg;
        P.t.perms = d_perms;
        P.t.seeds = d_seeds;
        P.t.np = np;
        P.T = d_T;
        P.Tmask = T_cap - 1;
        P.err = d_err;
        P.flags = d_flags;
        P.par = d_par;
        P.pslot = d_pslot;
        return P;
    }

    // ---- packing (unpacked int32 interchange <-> record) ------------------------------
    void pack(const int32_t *u, uint32_t *rec) const {
        const int n = N, Vv = V;
        std::vector<uint32_t> w(RECW, 0);
        int k = 0;
        auto L_VF = 0, L_CT = 1, L_ROLE = 2, L_CI = 3, L_LL = 4, L_LOG = 5, L_MI = 5 + n, L_NI = 5 + 2 * n,
             L_PEND = 5 + 3 * n, L_MISC = 6 + 3 * n;
        for (int i = 0; i < n; i++) w[L_VF] = setnib(w[L_VF], i, u[k + i] < 0 ? VF_NONE : (uint32_t)u[k + i]);
        k += n;
        for (int i = 0; i < n; i++) w[L_CT] = setnib(w[L_CT], i, u[k + i]);
        k += n;
        for (int i = 0; i < n; i++) w[L_ROLE] = setnib(w[L_ROLE], i, u[k + i]);
        k += n;
        for (int i = 0; i < n; i++) w[L_CI] = setnib(w[L_CI], i, u[k + i]);
        k += n;
        std::vector<int> ll(n);
        for (int i = 0; i < n; i++) { ll[i] = u[k + i]; w[L_LL] = setnib(w[L_LL], i, u[k + i]); }
        k += n;
        for (int i = 0; i < n; i++)
            for (int x = 1; x <= Vv + 1; x++) {
                const int t = u[k], v = u[k + 1];
                k += 2;
                if (x >= 2 && x <= ll[i]) w[L_LOG + i] |= (uint32_t)((t & 15) | ((v & 15) << 4)) << (8 * (x - 2));
            }
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) w[L_MI + i] = setnib(w[L_MI + i], j, u[k++]);
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) w[L_NI + i] = setnib(w[L_NI + i], j, u[k++]);
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) w[L_PEND] |= (u[k++] ? 1u : 0u) << (i * n + j);
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
        std::memcpy(rec, w.data(), (size_t)ks.CW * 4);
        uint16_t *rid = reinterpret_cast<uint16_t *>(rec + ks.CW);
        for (int q = 0; q < ks.MCAP; q++) rid[q] = q < (int)ids.size() ? ids[q] : 0;
    }

    std::vector<int32_t> unpack(const uint32_t *rec) const {
        const int n = N, Vv = V;
        const int L_VF = 0, L_CT = 1, L_ROLE = 2, L_CI = 3, L_LL = 4, L_LOG = 5, L_MI = 5 + n, L_NI = 5 + 2 * n,
                  L_PEND = 5 + 3 * n, L_MISC = 6 + 3 * n;
        const uint32_t misc = rec[L_MISC];
        const int nm = (misc >> 16) & 0xFF;
        std::vector<int32_t> o;
        o.reserve(RMC_UNPACKED_INTS(n, Vv, nm));
        for (int i = 0; i < n; i++) { uint32_t v = nib(rec[L_VF], i); o.push_back(v == VF_NONE ? -1 : (int)v); }
        for (int i = 0; i < n; i++) o.push_back(nib(rec[L_CT], i));
        for (int i = 0; i < n; i++) o.push_back(nib(rec[L_ROLE], i));
        for (int i = 0; i < n; i++) o.push_back(nib(rec[L_CI], i));
        for (int i = 0; i < n; i++) o.push_back(nib(rec[L_LL], i));
        for (int i = 0; i < n; i++)
            for (int x = 1; x <= Vv + 1; x++) {
                if (x == 1) { o.push_back(0); o.push_back(-1); continue; }
                if (x > (int)nib(rec[L_LL], i)) { o.push_back(0); o.push_back(0); continue; }
                const uint32_t b = (rec[L_LOG + i] >> (8 * (x - 2))) & 0xFF;
                o.push_back(b & 15);
                o.push_back(b >> 4);
            }
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) o.push_back(nib(rec[L_MI + i], j));
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) o.push_back(nib(rec[L_NI + i], j));
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) o.push_back((rec[L_PEND] >> (i * n + j)) & 1);
        o.push_back(misc & 15);
        o.push_back((misc >> 4) & 15);
        for (int v = 0; v < Vv; v++) o.push_back(((misc >> (8 + v)) & 1) ? 0 : -1);
        o.push_back(nm);
        const uint16_t *rid = reinterpret_cast<const uint16_t *>(rec + ks.CW);
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

    // ---- allocation -----------------------------------------------------------------
    void setup() {
        if (cfg.n_servers < 1 || cfg.n_servers > MAXN) throw Fail(RMC_E_ARG, "n_servers must be 1..5");
        if (cfg.n_vals < 0 || cfg.n_vals > MAXV) throw Fail(RMC_E_ARG, "n_vals must be 0..3");
        if (cfg.max_election < 0 || cfg.max_election > 7) throw Fail(RMC_E_ARG, "max_election must be 0..7");
        if (cfg.max_restart < 0 || cfg.max_restart > 15) throw Fail(RMC_E_ARG, "max_restart must be 0..15");
        if (cfg.invariants & RMC_INV_NO_ALL_COMMIT) throw Fail(RMC_E_ARG, "invariant NoAllCommit is not compiled");
        if (cfg.invariants & ~0x7Fu) throw Fail(RMC_E_ARG, "unknown invariant bits");
        if (cfg.world_size > 1) throw Fail(RMC_E_ARG, "multi-GPU sharding is driven by rmc_create on each rank: not in this build");
        N = cfg.n_servers;
        V = cfg.n_vals;
        int cap = cfg.msg_cap ? cfg.msg_cap : (N <= 3 ? 64 : 128);
        if (!get_kernels(N, V, cap, &ks))
            throw Fail(RMC_E_ARG, "no compiled kernels for n_servers=" + std::to_string(N) + " n_vals=" +
                                      std::to_string(V) + " msg_cap=" + std::to_string(cap));
        RECW = ks.RECW;
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
        HIPCHK(hipEventCreate(&ev0));
        HIPCHK(hipEventCreate(&ev1));

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

        Gcap = cfg.chunk_successors ? cfg.chunk_successors : (1ull << 26);
        Gcap = std::max<uint64_t>(Gcap, (uint64_t)ks.maxsucc * 64);
        if (Gcap >= (1ull << 31)) throw Fail(RMC_E_ARG, "chunk_successors must be < 2^31");
        chunk_parents = Gcap / ks.maxsucc;
        d_cnt = dmalloc<uint32_t>(chunk_parents + 1);
        d_off = dmalloc<uint32_t>(chunk_parents + 1);
        d_fp = dmalloc<ulonglong2>(Gcap);
        d_lslot = dmalloc<uint32_t>(Gcap);
        d_wflag = dmalloc<uint32_t>(Gcap + 1);
        HIPCHK(hipMemsetAsync(d_cnt, 0, (chunk_parents + 1) * 4, stream));
        HIPCHK(hipMemsetAsync(d_wflag, 0, (Gcap + 1) * 4, stream));
        d_wpos = dmalloc<uint32_t>(Gcap + 1);
        Lcap_max = next_pow2(2 * Gcap);
        d_L = dmalloc<unsigned long long>(Lcap_max);
        HIPCHK(hipMemsetAsync(d_L, 0, Lcap_max * 8, stream));
        d_sum = dmalloc<unsigned long long>(16);
        HIPCHK(hipHostMalloc((void **)&h_sum, 16 * 8, hipHostMallocDefault));
        size_t t1 = 0;
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, t1, d_cnt, d_off, (int)Gcap + 1, stream));
        tmp_bytes = t1;
        d_tmp = dmalloc<uint8_t>(tmp_bytes);

        T_cap = 1ull << (cfg.seen_log2 ? cfg.seen_log2 : 22);
        d_T = dmalloc<ulonglong2>(T_cap);
        HIPCHK(hipMemsetAsync(d_T, 0, T_cap * 16, stream));
        d_err = dmalloc<unsigned long long>(ERR_NSLOTS);
        d_flags = dmalloc<uint32_t>(4);
        reset_errors();

        cur_cap = nxt_cap = 1 << 16;
        d_cur = dmalloc<uint32_t>(cur_cap * RECW);
        d_nxt = dmalloc<uint32_t>(nxt_cap * RECW);
        trace_cap = 1 << 20;
        d_par = dmalloc<uint64_t>(trace_cap);
        d_pslot = dmalloc<uint16_t>(trace_cap);

        d_one = dmalloc<uint32_t>(RECW);
        d_out = dmalloc<uint32_t>((size_t)ks.maxsucc * RECW);
        d_keys = dmalloc<uint32_t>(ks.maxsucc);
        d_cnt1 = dmalloc<uint32_t>(4);
        d_fp1 = dmalloc<ulonglong2>(ks.maxsucc + 1);
        d_inv = dmalloc<int32_t>(7);
        HIPCHK(hipStreamSynchronize(stream));
    }

    void reset_errors() {
        HIPCHK(hipMemsetAsync(d_err, 0xFF, ERR_NSLOTS * 8, stream));
        HIPCHK(hipMemsetAsync(d_flags, 0, 16, stream));
    }

    void release() {
        dfree(d_info); dfree(d_nat2id); dfree(d_gmsg); dfree(d_perms); dfree(d_seeds);
        dfree(d_cur); dfree(d_nxt); dfree(d_cnt); dfree(d_off); dfree(d_fp); dfree(d_lslot); dfree(d_wflag);
        dfree(d_wpos); dfree(d_L); dfree(d_tmp); dfree(d_T); dfree(d_par); dfree(d_pslot); dfree(d_err);
        dfree(d_flags); dfree(d_one); dfree(d_out); dfree(d_keys); dfree(d_cnt1); dfree(d_fp1); dfree(d_inv);
        dfree(d_sum);
        if (h_sum) (void)hipHostFree(h_sum);
        h_sum = nullptr;
        for (hipEvent_t e : evpool) (void)hipEventDestroy(e);
        evpool.clear();
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        if (stream) (void)hipStreamDestroy(stream);
        ev0 = ev1 = nullptr;
        stream = nullptr;
    }

    void grow_records(uint32_t *&buf, uint64_t &cap, uint64_t used, uint64_t need) {
        if (need <= cap) return;
        uint64_t nc = std::max<uint64_t>(need + need / 2, cap * 2);
        uint32_t *nb = dmalloc<uint32_t>(nc * RECW);
        if (used) HIPCHK(hipMemcpyAsync(nb, buf, used * RECW * 4, hipMemcpyDeviceToDevice, stream));
        HIPCHK(hipStreamSynchronize(stream));
        dfree(buf);
        buf = nb;
        cap = nc;
    }

    void grow_trace(uint64_t need) {
        if (need <= trace_cap) return;
        uint64_t nc = std::max<uint64_t>(need + need / 2, trace_cap * 2);
        uint64_t *np_ = dmalloc<uint64_t>(nc);
        uint16_t *ns = dmalloc<uint16_t>(nc);
        HIPCHK(hipMemcpyAsync(np_, d_par, trace_cap * 8, hipMemcpyDeviceToDevice, stream));
        HIPCHK(hipMemcpyAsync(ns, d_pslot, trace_cap * 2, hipMemcpyDeviceToDevice, stream));
        HIPCHK(hipStreamSynchronize(stream));
        dfree(d_par);
        dfree(d_pslot);
        d_par = np_;
        d_pslot = ns;
        trace_cap = nc;
    }

    void grow_seen(uint64_t need) {
        if (need * 2 <= T_cap) return;  // keep the load factor <= 1/2
        uint64_t nc = T_cap;
        while (need * 2 > nc) nc *= 4;
        ulonglong2 *nT = dmalloc<ulonglong2>(nc);
        HIPCHK(hipMemsetAsync(nT, 0, nc * 16, stream));
        launch_rehash(d_T, T_cap, nT, nc - 1, stream);
        HIPCHK(hipStreamSynchronize(stream));
        dfree(d_T);
        d_T = nT;
        T_cap = nc;
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

    // successors of one record already in d_one: keys + records in d_out
    uint32_t expand_one(std::vector<uint32_t> *keys, std::vector<uint32_t> *recs, std::vector<ulonglong2> *fps,
                        bool *assert_fail) {
        reset_errors();
        KParams P = base();
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
        HIPCHK(hipMemcpy(e, d_err, sizeof e, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(fl, d_flags, sizeof fl, hipMemcpyDeviceToHost));
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

    // ---- BFS --------------------------------------------------------------------------
    int init(rmc_level_stats *st) {
        if (inited) throw Fail(RMC_E_STATE, "rmc_init called twice");
        auto t0 = std::chrono::steady_clock::now();
        std::vector<uint32_t> rec = init_record();
        HIPCHK(hipMemcpy(d_cur, rec.data(), RECW * 4, hipMemcpyHostToDevice));
        cur_n = 1;
        KParams P = base();
        P.front = d_cur;
        P.fp = d_fp1;
        ks.fp_states(P, 1, stream);
        launch_insert_fps(d_fp1, 1, d_T, T_cap - 1, stream);
        ks.inv_states(P, 1, d_inv, stream);
        int32_t iv[7];
        HIPCHK(hipMemcpyAsync(iv, d_inv, sizeof iv, hipMemcpyDeviceToHost, stream));
        const uint64_t none = ~0ull;
        HIPCHK(hipMemcpyAsync(d_par, &none, 8, hipMemcpyHostToDevice, stream));
        HIPCHK(hipStreamSynchronize(stream));
        T_count = 1;
        level_start = {0};
        total_generated = 1;  // TLC counts the initial state as generated
        total_distinct = 1;
        depth = 1;
        inited = true;
        status = RMC_OK;
        for (int b = 0; b < 7; b++) {
            if (!(cfg.invariants & (1u << b))) continue;
            if (iv[b] != 1) {
                status = iv[b] == 0 ? RMC_VIOLATION : RMC_EVAL_ERROR;
                violated = b;
                err_gid = 0;
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
            st->seconds = seconds;
        }
        return status;
    }

    int step(rmc_level_stats *st) {
        if (!inited) throw Fail(RMC_E_STATE, "rmc_step before rmc_init");
        if (finished) return status == RMC_OK ? RMC_DONE : status;
        auto t0 = std::chrono::steady_clock::now();
        rmc_level_stats local;
        if (!st) st = &local;
        std::memset(st, 0, sizeof *st);
        const int L = (int)level_start.size();  // expanding level L (1-based)
        st->level = L;
        st->expanded = cur_n;
        const uint64_t gid_cur = level_start[L - 1];
        const uint64_t gid_nxt = gid_cur + cur_n;
        uint64_t nxt_n = 0, level_gen = 0;
        for (uint64_t p0 = 0; p0 < cur_n; p0 += chunk_parents) {
            const uint64_t p1 = std::min(cur_n, p0 + chunk_parents), np_ = p1 - p0;
            auto params = [&] {
                KParams Q = base();
                Q.front = d_cur; Q.p_begin = p0; Q.p_end = p1; Q.cnt = d_cnt; Q.off = d_off; Q.fp = d_fp;
                Q.wflag = d_wflag; Q.wpos = d_wpos; Q.next = d_nxt; Q.next_base = nxt_n;
                Q.gid_next_base = gid_nxt; Q.gid_parent_base = gid_cur;
                return Q;
            };
            const uint32_t *Gp = d_off + np_;  // device-side successor count of the chunk
            timed(PH_COUNT, [&] {
                ks.count(params(), stream);
                // exclusive scan over np_+1 items: off[np_] = G (cnt[np_] is never read into it)
                HIPCHK(hipcub::DeviceScan::ExclusiveSum(d_tmp, tmp_bytes, d_cnt, d_off, (int)np_ + 1, stream));
            });
            // Small chunks run on an upper bound of G without a host round trip; large
            // ones read G back so that the dedup/scan passes are sized exactly.
            uint64_t Gub = np_ * (uint64_t)ks.maxsucc;
            if (Gub > (1ull << 20)) {
                Gub = d2h(Gp);
                collect_times(st);
            }
            grow_records(d_nxt, nxt_cap, nxt_n, nxt_n + Gub);
            grow_trace(gid_nxt + nxt_n + Gub);
            grow_seen(T_count + Gub);
            if (Gub) {
                timed(PH_HASH, [&] { ks.hash(params(), stream); });
                uint64_t Lcap = next_pow2(2 * Gub);
                if (Lcap > Lcap_max) Lcap = Lcap_max;
                ++epoch;
                timed(PH_DEDUP, [&] {
                    launch_dedup(d_fp, Gp, Gub, d_T, T_cap - 1, d_L, Lcap - 1, epoch, d_lslot, stream);
                    launch_winflag(d_lslot, d_L, Gp, Gub, d_wflag, stream);
                    HIPCHK(hipcub::DeviceScan::ExclusiveSum(d_tmp, tmp_bytes, d_wflag, d_wpos, (int)Gub + 1, stream));
                });
                timed(PH_MAT, [&] { ks.materialize(params(), stream); });
            }
            launch_summary(Gp, d_wpos, d_err, d_flags, d_sum, stream);
            HIPCHK(hipMemcpyAsync(h_sum, d_sum, 8 * 8, hipMemcpyDeviceToHost, stream));
            HIPCHK(hipStreamSynchronize(stream));
            HIPCHK(hipGetLastError());
            collect_times(st);
            const uint64_t G = h_sum[0], W = Gub ? h_sum[1] : 0;
            if (h_sum[2 + ERR_NSLOTS]) throw Fail(RMC_E_CAPACITY, "a state exceeds msg_cap = " + std::to_string(ks.MCAP) + " messages");
            const unsigned long long *e = h_sum + 2;
            level_gen += G;
            T_count += W;
            int kind = -1;
            unsigned long long best = ~0ull;
            // TLC order: smaller (parent, slot) first; on a tie the Assert wins (its action's batch is discarded)
            const int order[4] = {ERR_ASSERT, ERR_DEADLOCK, ERR_INV, ERR_EVAL};
            for (int q = 0; q < 4; q++) {
                const int kk = order[q];
                if (e[kk] == ~0ull) continue;
                if (kind < 0 || (e[kk] >> 8) < (best >> 8)) { kind = kk; best = e[kk]; }
            }
            if (kind >= 0) {
                stop_on_error(kind, best, p0, nxt_n, gid_cur, gid_nxt, level_gen - G, st);
                st->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                seconds += st->seconds;
                return status;
            }
            nxt_n += W;
        }
        total_generated += level_gen;
        total_distinct += nxt_n;
        st->generated = level_gen;
        st->new_states = nxt_n;
        std::swap(d_cur, d_nxt);
        std::swap(cur_cap, nxt_cap);
        cur_n = nxt_n;
        if (cur_n) {
            level_start.push_back(gid_nxt);
            depth = L + 1;
        } else {
            finished = true;
            status = RMC_DONE;
            queue_at_end = 0;
        }
        st->total_generated = total_generated;
        st->total_distinct = total_distinct;
        st->queue = cur_n;
        st->status = finished ? RMC_DONE : RMC_OK;
        st->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        seconds += st->seconds;
        return st->status;
    }

    // TLC's counters at the moment the first error (in -workers 1 order) is reported.
    void stop_on_error(int kind, unsigned long long ek, uint64_t p0, uint64_t nxt_before, uint64_t gid_cur,
                       uint64_t gid_nxt, uint64_t gen_before_chunk, rmc_level_stats *st) {
        const uint64_t p = ek >> 24;                       // level-local parent
        const uint32_t slot = (uint32_t)((ek >> 8) & 0xFFFF);
        const int which = (int)(ek & 0xFF);
        const uint32_t off_p = d2h(d_off + (p - p0));
        // successors of p, in order, to find the sub-action batch boundaries
        HIPCHK(hipMemcpy(d_one, d_cur + p * RECW, RECW * 4, hipMemcpyDeviceToDevice));
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
            uint32_t rank = 0;
            for (uint32_t k : keys) rank += k < slot;
            const uint32_t j = off_p + rank;
            winners_before = d2h(d_wpos + j);
            err_gid = gid_nxt + nxt_before + winners_before;
            total_distinct += nxt_before + winners_before + 1;
            queue_at_end = (cur_n - p - 1) + nxt_before + winners_before;
            status = kind == ERR_INV ? RMC_VIOLATION : RMC_EVAL_ERROR;
            violated = which;
            depth = (int)level_start.size() + 1;
        } else {
            if (kind == ERR_ASSERT) gen += cut;  // the failing sub-action's batch is never counted
            const uint32_t jcut = off_p + (kind == ERR_ASSERT ? cut : 0);
            winners_before = d2h(d_wpos + jcut);
            err_gid = gid_cur + p;
            total_distinct += nxt_before + winners_before;
            queue_at_end = (cur_n - p - 1) + nxt_before + winners_before;
            status = kind == ERR_ASSERT ? RMC_ASSERT : RMC_DEADLOCK;
            if (winners_before + nxt_before > 0) depth = (int)level_start.size() + 1;
        }
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

    // Walk parent pointers from err_gid to Init, then replay the slots from Init.
    void build_trace() {
        std::vector<uint16_t> slots;
        uint64_t g = err_gid;
        while (g != 0) {
            const uint64_t par = d2h(d_par + g);
            slots.push_back(d2h(d_pslot + g));
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

    // Forget every explored state but keep all device buffers (repeat runs, benchmarks).
    void reset() {
        HIPCHK(hipMemsetAsync(d_T, 0, T_cap * 16, stream));
        HIPCHK(hipStreamSynchronize(stream));
        T_count = 0;
        cur_n = 0;
        level_start.clear();
        trace.clear();
        inited = finished = false;
        status = RMC_OK;
        depth = 0;
        total_generated = total_distinct = queue_at_end = 0;
        violated = -1;
        err_gid = 0;
        seconds = 0;
    }

    void result(rmc_result *r) const {
        std::memset(r, 0, sizeof *r);
        r->status = finished ? status : RMC_OK;
        r->depth = depth;
        r->generated = total_generated;
        r->distinct = total_distinct;
        r->queue = finished ? queue_at_end : cur_n;
        r->violated = violated;
        r->trace_len = (uint32_t)trace.size();
        r->seconds = seconds;
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
        static thread_local std::string last;
        last = c->err;
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
        int rc = RMC_OK;
        while (!c->finished) rc = c->step(nullptr);
        (void)rc;
        if (res) c->result(res);
        return c->status;
    });
}

int rmc_reset(void *ctx) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    return guarded(c, [&] {
        c->reset();
        return RMC_OK;
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
        KParams P = c->base();
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
        KParams P = c->base();
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
