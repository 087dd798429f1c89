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
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include "rmc.h"
#include "rmc_kernels.h"
#include "rmc_plan.h"
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

// Host memory of the trace (parent's global id + slot key of every state the run found: ~110 GB
// at Raft.cfg): pageable blocks on transparent huge pages.  Round 2 kept it in pinned blocks (the
// device copied straight into them; pinned ahead of need by a background thread, since pinning
// runs at a few GB/s), but the process gives pinned memory back at ~9 GB/s when it exits: 12 s of
// myrun.sh's wall time after TLC's "Finished" line.  Huge-page blocks go back ~3x faster and are
// made ~2x faster (profiles/r03_teardown_probe.txt); the device copies into a few pinned staging
// buffers instead and a host thread moves each into its blocks (TraceStager).
static void *thp_alloc(size_t bytes) {
    void *p = nullptr;
    if (posix_memalign(&p, 2u << 20, bytes) != 0 || !p) throw Fail(RMC_E_MEMORY, "host memory for the trace");
    (void)madvise(p, bytes, MADV_HUGEPAGE);
    return p;
}

// Host array in huge-page blocks: the trace of every state the run found, never reallocated
// (block pointers stay valid while later blocks are added).
template <class T>
struct HostArr {
    static constexpr uint64_t B = 1ull << 22;
    std::vector<T *> blk;
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
        for (T *p : blk) std::free(p);
        blk.clear();
        n = 0;
    }
    void reserve_to(uint64_t m) {
        while ((uint64_t)blk.size() * B < m) blk.push_back(static_cast<T *>(thp_alloc(B * sizeof(T))));
    }
    T get(uint64_t i) const { return blk[i / B][i % B]; }
    void set(uint64_t i, T v) {
        reserve_to(i + 1);
        blk[i / B][i % B] = v;
        n = std::max(n, i + 1);
    }
    void extend(uint64_t at, uint64_t cnt) {  // elements [at, at + cnt) will be written (TraceStager)
        reserve_to(at + cnt);
        n = std::max(n, at + cnt);
    }
    void to_device(T *dev, uint64_t at, uint64_t cnt) const {
        for (uint64_t i = 0; i < cnt;) {
            const uint64_t g = at + i, k = std::min(cnt - i, B - g % B);
            HIPCHK(hipMemcpy(dev + i, blk[g / B] + g % B, k * sizeof(T), hipMemcpyHostToDevice));
            i += k;
        }
    }
    template <class F>
    void for_range(uint64_t at, uint64_t cnt, F &&f) const {  // f(pointer, count) over contiguous pieces
        for (uint64_t i = 0; i < cnt;) {
            const uint64_t g = at + i, k = std::min(cnt - i, B - g % B);
            f(blk[g / B] + g % B, k);
            i += k;
        }
    }
    void copy_from(const HostArr &o, uint64_t at, uint64_t cnt) {
        reserve_to(at + cnt);
        for (uint64_t i = 0; i < cnt; i++) blk[(at + i) / B][(at + i) % B] = o.get(at + i);
        n = std::max(n, at + cnt);
    }
};

// Trace flushes: device -> one of K pinned staging buffers on the copy stream, then a host thread
// waits for that copy's event and moves the entries into the HostArr blocks (whose addresses the
// caller resolved when it enqueued: the workers never touch a block vector).  The caller waits
// for a free staging buffer, so at most K pieces are in flight.  Several workers: the first touch of
// a fresh block (page faults) runs at a few GB/s per thread, and Raft.cfg's widest levels find
// ~5 GB of trace per second.
class TraceStager {
  public:
    static constexpr uint64_t S = 1ull << 22;  // entries per staging buffer
    static constexpr int K = 8, NW = 4;        // staging buffers, worker threads
    TraceStager() {
        for (int b = 0; b < K; b++) {
            HIPCHK(hipHostMalloc((void **)&par_[b], S * 8, hipHostMallocDefault));
            HIPCHK(hipHostMalloc((void **)&slot_[b], S * 2, hipHostMallocDefault));
            HIPCHK(hipEventCreateWithFlags(&ev_[b], hipEventDisableTiming));
            free_.push_back(b);
        }
        for (int t = 0; t < NW; t++) th_[t] = std::thread([this] { run(); });
    }
    ~TraceStager() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (std::thread &t : th_) t.join();
        for (int b = 0; b < K; b++) {
            (void)hipHostFree(par_[b]);
            (void)hipHostFree(slot_[b]);
            (void)hipEventDestroy(ev_[b]);
        }
    }
    // entries [at, at + cnt) of (hpar, hslot) from device memory, copied on stream `cs` after what
    // is already enqueued there
    void enqueue(const uint64_t *dpar, const uint16_t *dslot, uint64_t cnt, HostArr<uint64_t> &hpar,
                 HostArr<uint16_t> &hslot, uint64_t at, hipStream_t cs) {
        hpar.extend(at, cnt);
        hslot.extend(at, cnt);
        for (uint64_t i = 0; i < cnt;) {
            const uint64_t k = std::min(cnt - i, S);
            int b;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return !free_.empty() || failed_; });
                if (failed_) throw Fail(RMC_E_DEVICE, "trace copy to the host failed");
                b = free_.back();
                free_.pop_back();
            }
            try {
                HIPCHK(hipMemcpyAsync(par_[b], dpar + i, k * 8, hipMemcpyDeviceToHost, cs));
                HIPCHK(hipMemcpyAsync(slot_[b], dslot + i, k * 2, hipMemcpyDeviceToHost, cs));
                HIPCHK(hipEventRecord(ev_[b], cs));
            } catch (...) {
                // the buffer goes back and the stager is marked failed: drain() reports the error
                // instead of waiting for a buffer that no job will return
                {
                    std::lock_guard<std::mutex> lk(m_);
                    free_.push_back(b);
                    failed_ = true;
                }
                cv_.notify_all();
                throw;
            }
            Job j;
            j.b = b;
            hpar.for_range(at + i, k, [&](uint64_t *p, uint64_t c) { j.pp[j.np] = p; j.pc[j.np++] = c; });
            int q = 0;  // (same block size: the same pieces)
            hslot.for_range(at + i, k, [&](uint16_t *p, uint64_t c) { j.sp[q] = p; j.sc[q++] = c; });
            {
                std::lock_guard<std::mutex> lk(m_);
                jobs_.push_back(j);
            }
            cv_.notify_all();
            i += k;
        }
    }
    // every enqueued piece is in its blocks (the copy stream is synchronised first by the caller)
    void drain() {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return (jobs_.empty() && (int)free_.size() == K) || failed_; });
        if (failed_) throw Fail(RMC_E_DEVICE, "trace copy to the host failed");
    }

  private:
    struct Job {  // a piece of <= S entries spans at most two blocks (S == HostArr::B)
        int b = 0, np = 0;
        uint64_t *pp[2] = {};
        uint64_t pc[2] = {};
        uint16_t *sp[2] = {};
        uint64_t sc[2] = {};
    };
    void run() {
        std::unique_lock<std::mutex> lk(m_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || !jobs_.empty(); });
            if (jobs_.empty()) return;  // stop_
            Job j = jobs_.front();
            jobs_.erase(jobs_.begin());
            lk.unlock();
            const bool ok = hipEventSynchronize(ev_[j.b]) == hipSuccess;
            if (ok) {
                uint64_t o = 0;
                for (int t = 0; t < j.np; t++) {
                    std::memcpy(j.pp[t], par_[j.b] + o, j.pc[t] * 8);
                    std::memcpy(j.sp[t], slot_[j.b] + o, j.sc[t] * 2);
                    o += j.pc[t];
                }
            }
            lk.lock();
            if (!ok) failed_ = true;
            free_.push_back(j.b);
            cv_.notify_all();
        }
    }
    uint64_t *par_[K] = {};
    uint16_t *slot_[K] = {};
    hipEvent_t ev_[K] = {};
    std::mutex m_;
    std::condition_variable cv_;
    std::vector<int> free_;
    std::vector<Job> jobs_;
    bool stop_ = false, failed_ = false;
    std::thread th_[NW];
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
    // trace: parent's global id + slot key per local gid; the device
    // buffers hold gids from tflushed on, the host arrays everything before
    uint64_t *par = nullptr;
    uint16_t *pslot = nullptr;
    uint64_t trace_cap = 0, tflushed = 0;
    uint64_t trace_end = 0;  // gids with device trace entries (a finished run's last levels stay on the device)
    uint64_t tdev = 0;  // gid of device trace index 0 (set to tflushed when a kernel sequence starts)
    HostArr<uint64_t> hpar;
    HostArr<uint16_t> hslot;
    hipEvent_t tev = nullptr;  // the last trace flush on the copy stream
    bool tev_pending = false;
    std::vector<uint64_t> level_start;  // local gid of the first state of each level
    // chunk buffers (source side)
    uint32_t *cnt = nullptr, *lslot = nullptr, *wpos = nullptr;
    uint32_t *hcnt = nullptr;   // split chunks: successors per parent to fingerprint (KParams::hcnt)
    bool chunk_sep = false;     // the chunk being processed set self-loops apart (hcnt valid)
    bool chunk_dense = false;   // ... and laid its successor slots out densely (hoff valid)
    uint32_t *hoff = nullptr;   // split chunk: each parent's first successor slot (KParams::hoff)
    ulonglong2 *fp = nullptr;
    ESlot *E = nullptr;         // election table: tagged fingerprint + election word per slot (32 B)
    uint32_t epoch = 0;
    uint32_t lxy_epoch0 = 0;    // epoch of the last E clear (16-bit tags repeat after 65535 epochs)
    uint64_t gslots = 0, lcap = 0;  // successor slots of fp / lslot / score, election slots of E
    // fused single-shard level: sparse successor staging (slot q = chunk parent * maxsucc + rank)
    uint4 *score = nullptr;
    uint32_t *wcnt = nullptr, *wacc = nullptr, *pnm = nullptr, *wposw = nullptr, *ctick = nullptr;
    uint32_t *bw = nullptr, *bg = nullptr, *boff = nullptr, *bww = nullptr, *boffw = nullptr, *tickets = nullptr;
    uint32_t *bn = nullptr, *boffn = nullptr, *plist = nullptr;  // parents with winners (split chunks)
    uint32_t *hctx = nullptr;  // split chunks: each parent's hash context (KernelSet::ctxw words)
    // device-driven level loop: control block, per-level records, and their pinned host copies
    LevelCtl *ctl = nullptr, *hctl = nullptr;
    HostLoop *hloop = nullptr, *dloop = nullptr;  // device-loop mirror in mapped pinned memory (host / device view)
    LevelRec *lrec = nullptr, *hlrec = nullptr;
    void *tmp = nullptr;
    size_t tmp_bytes = 0;
    // sharded round (W > 1): successors to their fingerprint's owner (xs, owner-grouped; perm =
    // each item's slot, sflag = the owner's verdict), received successors (xr, rslot, rflag), the
    // owner's election table (OT / OK), the round's winners (outbox: records ob, offsets ooff,
    // sidecars oside) and the winners received from the sources (ib, iside, isz / ioff)
    XItem *xs = nullptr, *xr = nullptr;
    uint64_t xs_cap = 0, xr_cap = 0;
    uint32_t *perm = nullptr, *sflag = nullptr, *rslot = nullptr, *rflag = nullptr, *ocnt = nullptr;
    ESlot *OT = nullptr;
    uint64_t ot_cap = 0;
    uint32_t ot_round = 0;  // rounds on the owner table since it was last cleared (its tag, k_owner_elect)
    ESlot *rt_table = nullptr;  // the table the round's bids went to (E or OT) and its round: a split round's
    uint32_t rt_round = 0;      // commit decides the shard's own candidates there
    // split rounds: the fused election table (E, unused once the run is sharded) is the owner
    // table, so k_hash_probe bids the shard's own successors as it fingerprints them; rounds on it
    // since its last clear (0: not yet cleared for this use), and whether this round's own bids went in
    uint32_t lx_round = 0;
    bool lx_bid = false;
    uint32_t *ob = nullptr, *ib = nullptr;
    uint64_t ob_cap = 0, ib_cap = 0;
    uint4 *oside = nullptr, *iside = nullptr;
    uint64_t *ooff = nullptr;
    uint32_t *isz = nullptr, *ioff = nullptr;
    uint64_t os_cap = 0, is_cap = 0;
    // errors, summary
    unsigned long long *err = nullptr, *sum = nullptr, *hsum = nullptr;
    uint32_t *flags = nullptr;
    // per-round host bookkeeping (sharded path): first parent, parents, successors, global index
    // of the round's first parent in the level
    uint64_t p0 = 0, np = 0, G = 0, gblk = 0;
    uint64_t Gself = 0;  // the round's successors the shard owns itself (G: those it sends)
};

// the host-staged transport installed by rmc_set_transport (process-wide; read by rmc_create)
static rmc_transport g_transport{};
static bool g_transport_set = false;

struct rmc_ctx {
    rmc_config cfg{};
    KernelSet ks{};
    Universe U;
    std::string err;
    hipStream_t stream = nullptr;
    hipStream_t cstream = nullptr;  // trace flushes (device -> pinned host), overlapped with the level loop
    hipEvent_t flush_ev = nullptr;  // the main stream's point a flush starts from
    std::unique_ptr<TraceStager> stager;  // trace flushes to the host arrays
    int N = 0, V = 0, RECW = 0;  // RECW = the longest record (fixed-stride buffers)
    uint32_t inv_order = 0;      // invariants in cfg order (check_invs)
    int W = 1, rank = 0;  // shards in the run, this process's first shard
    bool virt = false;    // all W shards live in this process
    bool multi = false;   // the sharded protocol runs (W > 1, or one RCCL rank talking to itself)
    bool rccl = false;    // shards exchange through an RCCL communicator (not device copies)
    bool hostx = false;   // ... through the host-staged transport (rmc_set_transport)
    rmc_transport tx{};
#ifdef RMC_WITH_RCCL
    ncclComm_t comm = nullptr;
#endif
    // Init's record, fingerprint and invariant verdicts, cached by the first single-GPU Init
    uint32_t *d_init_rec = nullptr;
    ulonglong2 *d_init_fp = nullptr;
    int32_t init_iv[7] = {0};
    bool init_cached = false;

    // device tables
    uint32_t *d_info = nullptr;
    uint16_t *d_nat2id = nullptr;
    ulonglong2 *d_gmsg = nullptr;
    uint64_t *d_seeds = nullptr;
    int np = 0;
    uint64_t scheme_hash = 0;  // identifies the fingerprint scheme (seeds, message hashes): checkpoints

    std::vector<Shard> sh;
    uint64_t chunk_parents = 0, Gcap = 0, Lcap_max = 0;
    uint64_t want_chunk_parents_adopt = 0;  // resume: a checkpoint's smaller chunk size, taken over
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
    unsigned long long *d_red = nullptr, *h_red = nullptr;  // collective scratch (RED_CAP values)
    static constexpr int RED_CAP = 64 * (2 * 64 + 8) + (2 * 64 + 8);  // a W x K gathered count matrix + one row

    // progress
    bool inited = false, finished = false;
    bool device_released = false;  // rmc_release_device: only rmc_destroy may follow
    int status = RMC_OK;
    int depth = 0;
    uint64_t total_generated = 0, total_distinct = 0, queue_at_end = 0;
    int violated = -1;
    uint64_t err_ref = 0;  // global id of the state whose trace is reported
    uint32_t err_last_slot = KEY_NONE;  // sharded: slot of the violating successor (not stored anywhere)
    // W > 1, block-cyclic levels: global index g of a level lives on shard (g / B) % W at local
    // index (g / (B W)) B + g % B, B = chunk_parents; glevel = global id of each level's first
    // state; levels before L_shard were expanded replicated (global id == local gid everywhere)
    std::vector<uint64_t> glevel;
    int L_shard = 0;
    std::vector<TraceStep> trace;
    double seconds = 0;

    KParams base(const Shard &s) const {
        KParams P{};
        P.d = U.d;
        P.E = cfg.max_election;
        P.R = cfg.max_restart;
        P.seeded = cfg.spec_variant == RMC_SPEC_SEEDED;
        P.quirks = (cfg.spec_variant == RMC_SPEC_SPLIT_BRAIN ? 1u : 0u) | (cfg.spec_variant == RMC_SPEC_COMMIT_PAST_LOG ? 2u : 0u);
        P.check_deadlock = cfg.check_deadlock;
        P.inv_mask = cfg.invariants;
        P.inv_order = inv_order;
        P.t.info = d_info;
        P.t.nat2id = d_nat2id;
        P.t.gmsg = d_gmsg;
        P.t.seeds = d_seeds;
        P.t.np = np;
        P.t.bmw = (uint32_t)((U.info.size() + 31) / 32);
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
        Q.bn = s.bn; Q.boffn = s.boffn;
        Q.tickets = s.tickets; Q.ctick = s.ctick; Q.sum = s.sum;
        Q.score = s.score; Q.lslot = s.lslot; Q.ET = s.E; Q.hctx = s.hctx;
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
        // world_size == 1 with a unique id: a one-rank communicator; the sharded protocol then
        // runs through RCCL (self send/recv, one-rank all-reduce/all-to-all) -- its transport
        // exercised on a one-GPU machine
        hostx = !virt && ws > 1 && !cfg.comm_unique_id && g_transport_set;
        rccl = !virt && !hostx && (ws > 1 || (cfg.world_size == 1 && cfg.comm_unique_id));
        multi = W > 1 || rccl;
        if (hostx) tx = g_transport;
        if (rank < 0 || rank >= W) throw Fail(RMC_E_ARG, "rank out of range");
        N = cfg.n_servers;
        V = cfg.n_vals;
        int cap = cfg.msg_cap ? cfg.msg_cap : (N <= 3 ? 64 : 128);
        if (cfg.spec_variant < RMC_SPEC_RAFT || cfg.spec_variant > RMC_SPEC_COMMIT_PAST_LOG)
            throw Fail(RMC_E_ARG, "unknown spec_variant " + std::to_string(cfg.spec_variant));
        if (!get_kernels(N, V, cap, cfg.spec_variant == RMC_SPEC_BECOME_FOLLOWER, &ks))
            throw Fail(RMC_E_ARG, "no compiled kernels for n_servers=" + std::to_string(N) + " n_vals=" +
                                      std::to_string(V) + " msg_cap=" + std::to_string(cap));
        RECW = ks.RECW_MAX;
        // the sharded election key is (parent's global index << 10) | rank (k_route_place): every
        // parent's successors must fit the 10-bit rank (BecomeFollower at 5 servers: ~306)
        if (multi && ks.maxsucc > 1024)
            throw Fail(RMC_E_ARG, "sharded runs need at most 1024 successor slots per state");
        if (const char *fi = std::getenv("RMC_FAULT_INJECT")) {  // tests: "site,shard,round[,level]"
            long long r = -1;
            int lv = -1;
            if (std::sscanf(fi, "%d,%d,%lld,%d", &fi_site, &fi_shard, &r, &lv) >= 3) {
                fi_round = r;
                fi_level = lv;
            } else {
                fi_site = 0;
            }
        }
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
        HIPCHK(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&flush_ev, hipEventDisableTiming));
        stager.reset(new TraceStager());
        if (rccl) {
#ifdef RMC_WITH_RCCL
            if (!cfg.comm_unique_id)
                throw Fail(RMC_E_ARG, "world_size > 1 needs comm_unique_id (rmc_comm_unique_id) or a transport (rmc_set_transport)");
            ncclUniqueId id;
            std::memcpy(&id, cfg.comm_unique_id, sizeof id);
            if (ncclCommInitRank(&comm, W, id, rank) != ncclSuccess) throw Fail(RMC_E_COMM, "ncclCommInitRank failed");
#else
            throw Fail(RMC_E_COMM, "built without RCCL");
#endif
        }

        d_red = dmalloc<unsigned long long>(2 * RED_CAP);  // collective scratch (the chunk-size agreement below)
        HIPCHK(hipHostMalloc((void **)&h_red, RED_CAP * 8, hipHostMallocDefault));

        U.build(N, V, cfg.max_election);
        d_info = dmalloc<uint32_t>(U.info.size());
        d_nat2id = dmalloc<uint16_t>(U.nat2id.size());
        d_gmsg = dmalloc<ulonglong2>(U.gmsg.size());
        HIPCHK(hipMemcpy(d_info, U.info.data(), U.info.size() * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(d_nat2id, U.nat2id.data(), U.nat2id.size() * 2, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(d_gmsg, U.gmsg.data(), U.gmsg.size() * 16, hipMemcpyHostToDevice));

        // |Permutations(Servers)| (tla:21); 1 without SYMMETRY (the fingerprint's coset is the identity)
        np = 1;
        if (!cfg.no_symmetry)
            for (int i = 2; i <= N; i++) np *= i;
        // position constants K_f[a][b] of the fingerprint (rmc_spec.h), odd
        std::vector<uint64_t> seeds(2 * SEEDS_PER_F);
        uint64_t x = SEED_PAIR;
        for (uint64_t &v : seeds) v = splitmix(x) | 1ull;
        d_seeds = dmalloc<uint64_t>(seeds.size());
        HIPCHK(hipMemcpy(d_seeds, seeds.data(), seeds.size() * 8, hipMemcpyHostToDevice));
        // fingerprint scheme identity (checkpoints): seeds, message hashes, record codec, slot hash
        // (4: signature-coset minimum for n >= 4; 5: positional slot keys; 6: codec of (N, V); 7: content
        // matrix x position constants, signature coset for every n; 8: the compact seen set in 64-B buckets)
        scheme_hash = 0x5eed5c4e3e000008ull;
        auto mixin = [&](uint64_t v) { scheme_hash = mix64(scheme_hash ^ (v + 0x9e3779b97f4a7c15ull)); };
        for (uint64_t s : seeds) mixin(s);
        for (const ulonglong2 &g : U.gmsg) { mixin(g.x); mixin(g.y); }
        mixin((uint64_t)ks.CCW);
        mixin((uint64_t)codec_bits(N, V));  // the instance's packed layout (field widths below)
        for (int w : {bits_for(N), bits_for(V + 1), bits_for(V + 2), bits_for(V - 1)}) mixin((uint64_t)w);

        // successor slots per chunk: dense for the sharded path, sparse (parents x maxsucc) for
        // the fused single-GPU path, whose staging holds SW4 * 16 + 36 bytes per slot
        // Fewer, larger chunks.  An RCCL rank's round (2^28 slots, ~3 M parents for 3 servers and 2
        // values) pays a dozen host round trips and collectives (one-rank Raft.cfg 66.8 s at 2^26,
        // 57.4 at 2^27, 54.7 at 2^28); a one-GPU chunk (2^28 slots) a few launches and their tails
        // (Raft.cfg 55.0 s at 2^26, 52.7 at 2^27, 51.7 at 2^28).  On one GPU the slot buffers grow
        // on demand (ensure_chunk), so a small run does not pay for them; an RCCL rank allocates
        // them at create, its budgets may be explicit (bench's configs[3] leg).
        Gcap = cfg.chunk_successors ? cfg.chunk_successors : (virt ? (1ull << 23) : (1ull << 28));
        if (!cfg.chunk_successors && !virt && (cfg.seen_mem_bytes || cfg.frontier_mem_bytes)) {
            // with explicit seen-set / frontier budgets (an RCCL rank allocates its round buffers at
            // create; one GPU grows them to this size), halve the default chunk until its buffers
            // fit beside the budgets in free memory
            // (per slot: fingerprint, verdict, staging, item out and in, route and owner words, ~2 election slots)
            size_t fr = 0, tot = 0;
            HIPCHK(hipMemGetInfo(&fr, &tot));
            // (per slot: fingerprint, verdict, staging, scan word, ~2 election slots; an RCCL rank also its
            // route / owner words and items out and in)
            const uint64_t per_slot = 16 + 4 + 16 * (uint64_t)sw4() + 4 + 2 * 32 +
                                      ((rccl || hostx) ? 4 + 4 + 2 * sizeof(XItem) + 8 : 0);
            // beside the budgets: the live levels' record offsets (8 B a state; the two widest levels
            // of configs[3] hold about a third of its seen set's states) and some slack
            const uint64_t budgets = cfg.seen_mem_bytes + cfg.frontier_mem_bytes + cfg.seen_mem_bytes / 2 + (4ull << 30);
            uint64_t halvings = 0;
            while (Gcap > (1ull << 24) && budgets + Gcap * per_slot > (uint64_t)fr) {
                Gcap >>= 1;
                ++halvings;
            }
            // B = chunk_parents sets the block-cyclic level layout every rank must share (step_sharded,
            // route_pieces), and free memory differs between ranks (another process on the device,
            // rank 0's extra allocations): every rank takes the most-halved chunk
            if (rccl || hostx) {
                allreduce(&halvings, 1, true);
                Gcap = (cfg.chunk_successors ? cfg.chunk_successors : (1ull << 28)) >> halvings;
            }
        }
        Gcap = std::max<uint64_t>(Gcap, (uint64_t)ks.maxsucc * 64);
        if (Gcap >= (1ull << 30)) throw Fail(RMC_E_ARG, "chunk_successors must be < 2^30");
        chunk_parents = Gcap / ks.maxsucc;
        shard_min = multi ? (cfg.shard_min_states ? cfg.shard_min_states : (1ull << 20)) : 0;
        chunk_parents = std::min<uint64_t>(chunk_parents, (uint64_t)WTILE * WTILES_MAX);  // winner-count tiles
        Lcap_max = next_pow2(2 * Gcap);

        sh.resize(virt ? W : 1);
        for (size_t i = 0; i < sh.size(); i++) alloc_shard(sh[i], virt ? (int)i : rank);

        d_one = dmalloc<uint32_t>(RECW);
        d_out = dmalloc<uint32_t>((size_t)ks.maxsucc * RECW);
        d_keys = dmalloc<uint32_t>(ks.maxsucc);
        d_cnt1 = dmalloc<uint32_t>(4);
        d_fp1 = dmalloc<ulonglong2>(ks.maxsucc + 1);
        d_inv = dmalloc<int32_t>(7);
        d_err1 = dmalloc<unsigned long long>(ERR_NSLOTS);
        d_flags1 = dmalloc<uint32_t>(4);
        HIPCHK(hipStreamSynchronize(stream));
    }

    // Successor-slot buffers (fingerprints, election slots, staging) and the election table for
    // at least `slots` successor slots (powers of two, at most Gcap / Lcap_max).  A checker whose
    // levels all run in the device loop keeps them small; the first larger chunk grows them, and
    // so does the move of the seen set / ring to their budgets (migrate_compact, fix_ring) -- so
    // that those budgets are taken from what the full chunk buffers leave.
    void ensure_chunk(Shard &s, uint64_t slots) {
        slots = std::min<uint64_t>(std::max<uint64_t>(slots, 1), Gcap);
        if (slots <= s.gslots) return;
        const uint64_t g = std::min<uint64_t>(std::max<uint64_t>(next_pow2(slots), 2 * s.gslots), Gcap);
        const uint64_t lc = std::min<uint64_t>(next_pow2(2 * g), Lcap_max);
        HIPCHK(hipStreamSynchronize(stream));
        dfree(s.fp); dfree(s.lslot); dfree(s.score);
        s.fp = nullptr; s.lslot = nullptr; s.score = nullptr;
        s.fp = dmalloc<ulonglong2>(g);
        s.lslot = dmalloc<uint32_t>(g);
        s.score = dmalloc<uint4>(g * (uint64_t)sw4());
        // chunks of split_min parents or more are split (M_SPLIT + k_hash_probe): their parents' hash contexts
        const uint64_t hp = g / (uint64_t)ks.maxsucc + 1;
        if (split_min && hp >= split_min) {
            dfree(s.hctx);
            s.hctx = nullptr;
            s.hctx = dmalloc<uint32_t>(hp * (uint64_t)ks.ctxw);
        }
        s.gslots = g;
        if (lc > s.lcap) {
            dfree(s.E);
            s.E = nullptr;
            s.E = dmalloc<ESlot>(lc);
            // free slots; an all-ones election word is older than every epoch's (elect_key)
            launch_eslot_clear(s.E, lc, stream);
            s.lcap = lc;
            s.lxy_epoch0 = s.epoch;
        }
    }

    void alloc_shard(Shard &s, int id) {
        s.id = id;
        HIPCHK(hipEventCreateWithFlags(&s.tev, hipEventDisableTiming));
        s.cnt = dmalloc<uint32_t>(chunk_parents + 1);
        s.wpos = dmalloc<uint32_t>(Gcap + 1);
        HIPCHK(hipMemsetAsync(s.cnt, 0, (chunk_parents + 1) * 4, stream));
        // the successor-slot buffers: at their full size on the sharded path, on one GPU sized for
        // the device loop's levels and grown on demand (ensure_chunk)
        ensure_chunk(s, multi ? Gcap : dev_parents() * (uint64_t)ks.maxsucc);
        s.wcnt = dmalloc<uint32_t>(chunk_parents + 1);
        s.wacc = dmalloc<uint32_t>(chunk_parents + 1);
        s.pnm = dmalloc<uint32_t>(chunk_parents + 1);
        s.hcnt = dmalloc<uint32_t>(chunk_parents + 1);
        s.hoff = dmalloc<uint32_t>(chunk_parents + 1);
        s.wposw = dmalloc<uint32_t>(chunk_parents + 1);
        s.ctick = dmalloc<uint32_t>(33 * 32);
        HIPCHK(hipMemsetAsync(s.ctick, 0, 33 * 32 * 4, stream));
        HIPCHK(hipMemsetAsync(s.wacc, 0, (chunk_parents + 1) * 4, stream));
        s.bw = dmalloc<uint32_t>(WTILES_MAX);
        s.bg = dmalloc<uint32_t>(WTILES_MAX);
        s.boff = dmalloc<uint32_t>(WTILES_MAX);
        s.bww = dmalloc<uint32_t>(WTILES_MAX);
        s.boffw = dmalloc<uint32_t>(WTILES_MAX);
        s.bn = dmalloc<uint32_t>(WTILES_MAX);
        s.boffn = dmalloc<uint32_t>(WTILES_MAX);
        s.plist = dmalloc<uint32_t>(chunk_parents + 1);
        s.tickets = dmalloc<uint32_t>(4);
        HIPCHK(hipMemsetAsync(s.tickets, 0, 16, stream));
        s.ctl = dmalloc<LevelCtl>(2);  // level i reads ctl[i & 1], its commit writes the other
        s.lrec = dmalloc<LevelRec>(LREC_CAP);
        HIPCHK(hipHostMalloc((void **)&s.hctl, 2 * sizeof(LevelCtl), hipHostMallocDefault));
        HIPCHK(hipHostMalloc((void **)&s.hloop, sizeof(HostLoop), hipHostMallocMapped | hipHostMallocCoherent));
        HIPCHK(hipHostGetDevicePointer((void **)&s.dloop, s.hloop, 0));
        HIPCHK(hipHostMalloc((void **)&s.hlrec, sizeof(LevelRec) * LREC_CAP, hipHostMallocDefault));
        if (multi) {
            s.perm = dmalloc<uint32_t>(Gcap);
            s.sflag = dmalloc<uint32_t>(Gcap);
        }
        ensure_tmp(s, Gcap + 1);
        s.T_cap = 1ull << (cfg.seen_log2 ? cfg.seen_log2 : 22);
        s.T = dmalloc<ulonglong2>(s.T_cap);
        HIPCHK(hipMemsetAsync(s.T, 0, s.T_cap * 16, stream));
        s.err = dmalloc<unsigned long long>(ERR_NSLOTS);
        s.flags = dmalloc<uint32_t>(4);
        HIPCHK(hipMemsetAsync(s.err, 0xFF, ERR_NSLOTS * 8, stream));
        HIPCHK(hipMemsetAsync(s.flags, 0, 16, stream));
        s.sum = dmalloc<unsigned long long>(SUM_WORDS_TOTAL);
        HIPCHK(hipMemsetAsync(s.sum, 0, SUM_WORDS_TOTAL * 8, stream));  // (the self-loop stripes are 0 between launches)
        s.ocnt = reinterpret_cast<uint32_t *>(s.sum + SUM_OCNT);
        HIPCHK(hipHostMalloc((void **)&s.hsum, SUM_WORDS_TOTAL * 8, hipHostMallocDefault));
        s.rcap = 1ull << 14;
        s.R = dmalloc<uint32_t>(s.rcap);
        s.cur_off_cap = s.nxt_off_cap = 1 << 16;
        s.cur_off = dmalloc<uint64_t>(s.cur_off_cap);
        s.nxt_off = dmalloc<uint64_t>(s.nxt_off_cap);
        s.trace_cap = 1 << 20;
        s.par = dmalloc<uint64_t>(s.trace_cap);
        s.pslot = dmalloc<uint16_t>(s.trace_cap);
    }

    void free_shard(Shard &s, bool keep_host_trace = false) {
        dfree(s.R); dfree(s.cur_off); dfree(s.nxt_off); dfree(s.T); dfree(s.Tc); dfree(s.par); dfree(s.pslot);
        dfree(s.cnt);
        dfree(s.lslot); dfree(s.wpos); dfree(s.fp); dfree(s.E); dfree(s.tmp);
        dfree(s.xs); dfree(s.xr); dfree(s.perm); dfree(s.sflag); dfree(s.rslot); dfree(s.rflag);
        s.ocnt = nullptr;  // (inside sum)
        dfree(s.OT); dfree(s.ob); dfree(s.ib); dfree(s.oside); dfree(s.iside); dfree(s.ooff);
        dfree(s.isz); dfree(s.ioff);
        dfree(s.err); dfree(s.sum); dfree(s.flags);
        dfree(s.score); dfree(s.wcnt); dfree(s.wacc); dfree(s.pnm); dfree(s.hcnt); dfree(s.hoff); dfree(s.wposw); dfree(s.ctick);
        dfree(s.bw); dfree(s.bg); dfree(s.boff); dfree(s.bww); dfree(s.boffw); dfree(s.tickets);
        dfree(s.bn); dfree(s.boffn); dfree(s.plist); dfree(s.hctx);
        dfree(s.ctl); dfree(s.lrec);
        if (s.hsum) (void)hipHostFree(s.hsum);
        if (s.hctl) (void)hipHostFree(s.hctl);
        if (s.hloop) (void)hipHostFree(s.hloop);
        if (s.hlrec) (void)hipHostFree(s.hlrec);
        s.hsum = nullptr; s.hctl = nullptr; s.hloop = nullptr; s.dloop = nullptr; s.hlrec = nullptr;
        if (!keep_host_trace) {
            s.hpar.release();
            s.hslot.release();
        }
        if (s.tev) (void)hipEventDestroy(s.tev);
        s.tev = nullptr;
    }

    // Every device allocation, stream, event and communicator (and the pinned buffers); with
    // keep_host_trace the shards' host trace blocks stay (rmc_release_device: the process exits next and
    // the kernel returns them).  Idempotent: rmc_destroy after rmc_release_device frees the rest.
    void release(bool keep_host_trace = false) {
        if (stream) (void)hipStreamSynchronize(stream);
        if (cstream) (void)hipStreamSynchronize(cstream);
        stager.reset();  // (its thread finishes the pieces already copied: before the blocks go)
        for (Shard &s : sh) free_shard(s, keep_host_trace);
        if (!keep_host_trace) sh.clear();
        dfree(d_info); dfree(d_nat2id); dfree(d_gmsg); dfree(d_seeds);
        dfree(d_one); dfree(d_init_rec); dfree(d_init_fp); dfree(d_out); dfree(d_keys); dfree(d_cnt1); dfree(d_fp1); dfree(d_inv); dfree(d_err1);
        dfree(d_flags1); dfree(d_red);
        if (h_red) (void)hipHostFree(h_red);
        h_red = nullptr;
        hx_send.release();
        hx_recv.release();
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
        if (cstream) (void)hipStreamDestroy(cstream);
        cstream = nullptr;
        if (flush_ev) (void)hipEventDestroy(flush_ev);
        flush_ev = nullptr;
    }

    // ---- frontier storage --------------------------------------------------------------------
    // offsets array with `used` entries kept
    void ensure_off(uint64_t *&p, uint64_t &cap, uint64_t used, uint64_t need) {
        if (need <= cap) return;
        // room to grow (x1.5) when the device has it; near the memory budgets, what the level needs
        uint64_t nc = std::max<uint64_t>(need + need / 2, cap * 2);
        uint64_t *nb = dmalloc_try<uint64_t>(nc);
        if (!nb) nb = dmalloc_try<uint64_t>(nc = need + need / 16);
        if (!nb) nb = dmalloc<uint64_t>(nc = need);
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
        HIPCHK(hipStreamSynchronize(stream));
        HIPCHK(hipStreamSynchronize(cstream));  // pending flushes read the old buffers
        const uint64_t nc = std::max<uint64_t>(need + need / 2, s.trace_cap * 2);
        dfree(s.par);
        dfree(s.pslot);
        s.par = dmalloc<uint64_t>(nc);
        s.pslot = dmalloc<uint16_t>(nc);
        s.trace_cap = nc;
    }

    // trace entries of gids [tflushed, upto) to the host: on the copy stream, after everything
    // enqueued so far on the main stream, overlapped with what follows there
    void flush_trace(Shard &s, uint64_t upto) {
        if (upto <= s.tflushed) return;
        const uint64_t n = upto - s.tflushed, at = s.tflushed - s.tdev;
        HIPCHK(hipEventRecord(flush_ev, stream));
        HIPCHK(hipStreamWaitEvent(cstream, flush_ev, 0));
        stager->enqueue(s.par + at, s.pslot + at, n, s.hpar, s.hslot, s.tflushed, cstream);
        HIPCHK(hipEventRecord(s.tev, cstream));
        s.tev_pending = true;
        s.tflushed = upto;
    }
    // the device trace buffer starts over at the first gid not yet on the host
    void trace_restart(Shard &s) { s.tdev = s.tflushed; }
    // before a launch that writes the device trace buffer: the flushes still reading it are done
    void trace_fence(Shard &s) {
        if (!s.tev_pending) return;
        HIPCHK(hipStreamWaitEvent(stream, s.tev, 0));
        s.tev_pending = false;
    }
    // the host trace arrays are complete (every flush landed)
    void sync_trace() {
        HIPCHK(hipStreamSynchronize(cstream));
        stager->drain();
    }

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
        ensure_chunk(s, Gcap);  // the budget below is what the full chunk buffers leave
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
        ensure_chunk(s, Gcap);  // the budget below is what the full chunk buffers leave
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

    int sw4() const { return ks.N >= 4 ? 3 : 2; }  // staging uint4s per successor (Spec::SW4)

    // scan scratch for n values
    void ensure_tmp(Shard &s, uint64_t n) {
        size_t t = 0;
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, t, s.cnt, s.cnt, (int)std::min<uint64_t>(n, INT32_MAX), stream));
        if (t <= s.tmp_bytes) return;
        HIPCHK(hipStreamSynchronize(stream));
        dfree(s.tmp);
        s.tmp_bytes = t + t / 2;
        s.tmp = dmalloc<uint8_t>(s.tmp_bytes);
    }

    // owner election table of at least 2 * R slots, cleared for the round
    // The owner's election table for a round of R items: slots and keys carry the round's 16-bit tag
    // (k_owner_elect), so a round starts on the table as the last one left it -- it is cleared only
    // when it is (re)allocated and once every 65533 rounds (one memset of up to ~0.8 GB per round
    // before: ~1 s of a one-rank Raft.cfg exhaustion).  The tag only moves forward between clears,
    // also across rmc_reset, so a stale slot never reads as current and its key is never smaller.
    // rounds between clears of the owner table (RMC_OT_CLEAR_ROUNDS: tests take it down to a few)
    const uint32_t ot_clear_rounds = (uint32_t)env_int("RMC_OT_CLEAR_ROUNDS", 0xFFFD, 1, 0xFFFD);
    // split sharded rounds: 1 = the own successors bid in E inside k_hash_probe (when the table
    // fits them), 0 = never (k_local_elect into the owner table), 2 = bid there but always redo the
    // bids in the owner table (a test of that fallback)
    const int owner_lxy = env_int("RMC_OWNER_LXY", 1, 0, 2);
    // the round's tag on E as the owner table (cleared on first use and every ot_clear_rounds)
    uint32_t lx_table(Shard &s) {
        if (s.lx_round == 0 || s.lx_round >= ot_clear_rounds) {
            launch_eslot_clear(s.E, s.lcap, stream);
            s.lx_round = 1;
        } else {
            ++s.lx_round;
        }
        return s.lx_round;
    }

    uint64_t owner_table(Shard &o, uint64_t R) {
        const uint64_t need = next_pow2(std::max<uint64_t>(2 * R, 1024));
        bool clear = false;
        if (need > o.ot_cap) {
            HIPCHK(hipStreamSynchronize(stream));
            dfree(o.OT);
            o.OT = dmalloc<ESlot>(need);
            o.ot_cap = need;
            clear = true;
        }
        if (clear || o.ot_round >= ot_clear_rounds) {  // tags 2 .. 0xFFFE, increasing between clears
            launch_eslot_clear(o.OT, o.ot_cap, stream);
            o.ot_round = 1;
        } else {
            ++o.ot_round;
        }
        return need;
    }

    // copy `words` linear words from src into the shard's ring at ring position `at` (wrapping)
    void ring_copy_in(Shard &s, uint64_t at, const uint32_t *src, uint64_t words) {
        const uint64_t n1 = std::min(words, s.rcap - at);
        if (n1) HIPCHK(hipMemcpyAsync(s.R + at, src, n1 * 4, hipMemcpyDeviceToDevice, stream));
        if (words > n1) HIPCHK(hipMemcpyAsync(s.R, src + n1, (words - n1) * 4, hipMemcpyDeviceToDevice, stream));
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
    // RMC_COLL_CHECK=1 (host-staged transport): before every collective the ranks compare its
    // sequence number, call site and size (one extra all-gather each) and stop with the first
    // difference -- a rank taking another path through the protocol shows up there, not as a hang
    const bool coll_check = env_int("RMC_COLL_CHECK", 0, 0, 1) != 0;
    uint64_t coll_seq = 0;
    void coll_guard(int line, uint64_t n) {
        if (!hostx || !coll_check) return;
        uint64_t row[3] = {coll_seq++, (uint64_t)line, n};
        std::vector<uint64_t> all((size_t)W * 3);
        if (tx.allgather_u64(tx.user, row, 3, all.data()) != 0) throw Fail(RMC_E_COMM, "transport allgather failed");
        for (int r = 0; r < W; r++)
            if (all[3 * r] != row[0] || all[3 * r + 1] != row[1] || all[3 * r + 2] != row[2])
                throw Fail(RMC_E_COMM, "collective mismatch: rank " + std::to_string(rank) + " #" +
                                           std::to_string(row[0]) + " at line " + std::to_string(row[1]) + " n " +
                                           std::to_string(row[2]) + ", rank " + std::to_string(r) + " #" +
                                           std::to_string(all[3 * r]) + " at line " + std::to_string(all[3 * r + 1]) +
                                           " n " + std::to_string(all[3 * r + 2]));
    }
    void allreduce(uint64_t *v, int n, bool is_max, int line = __builtin_LINE()) {
        if (hostx) {
            coll_guard(line, (uint64_t)n);
            if (tx.allreduce_u64(tx.user, v, n, is_max ? 1 : 0) != 0) throw Fail(RMC_E_COMM, "transport allreduce failed");
            return;
        }
        if (!rccl) return;
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

    // Every shard's row of K values on every rank: rows[li] = sh[li]'s row in, the W x K matrix
    // (row t = shard t) out.  One ncclAllGather through RCCL; virtual shards are all local.
    std::vector<uint64_t> gather_rows(const std::vector<std::vector<uint64_t>> &rows, int K, int line = __builtin_LINE()) {
        std::vector<uint64_t> M((size_t)W * K, 0);
        if (hostx) {
            coll_guard(line, (uint64_t)K);
            if (tx.allgather_u64(tx.user, rows[0].data(), K, M.data()) != 0) throw Fail(RMC_E_COMM, "transport allgather failed");
            return M;
        }
        if (!rccl) {
            for (size_t li = 0; li < sh.size(); li++)
                std::copy(rows[li].begin(), rows[li].end(), M.begin() + (size_t)sh[li].id * K);
            return M;
        }
#ifdef RMC_WITH_RCCL
        if ((size_t)W * K + K > (size_t)RED_CAP) throw Fail(RMC_E_ARG, "gather_rows: matrix exceeds the collective scratch");
        for (int k = 0; k < K; k++) h_red[k] = rows[0][k];
        HIPCHK(hipMemcpyAsync(d_red, h_red, K * 8, hipMemcpyHostToDevice, stream));
        if (ncclAllGather(d_red, d_red + K, K, ncclUint64, comm, stream) != ncclSuccess)
            throw Fail(RMC_E_COMM, "ncclAllGather failed");
        HIPCHK(hipMemcpyAsync(h_red + K, d_red + K, (size_t)W * K * 8, hipMemcpyDeviceToHost, stream));
        HIPCHK(hipStreamSynchronize(stream));
        std::copy(h_red + K, h_red + K + (size_t)W * K, M.begin());
#endif
        return M;
    }

    // One or more all-to-all-v payloads of fixed-size items, by the plans of rmc_plan.h
    // (plans[li] = sh[li]'s; P[k] the k-th payload): virtual shards copy every transfer on the
    // device, an RCCL rank posts one send and one receive per peer and payload, all in one group.
    // RMC_SELF_VIA_RCCL=1: a rank's part for itself goes through ncclSend / ncclRecv like any other
    // (the one-rank RCCL tests use it to run those calls on a one-GPU box); by default it is a
    // device copy (the successor items have no part for their own shard: k_local_elect decides those)
    const bool self_rccl = env_int("RMC_SELF_VIA_RCCL", 0, 0, 1) != 0;
    struct Payload {
        const std::vector<XPlan> *plans;
        std::vector<const void *> send;
        std::vector<void *> recv;
        size_t elem;
        bool self_in_place = false;  // a shard's items to itself are already in its receive buffer
    };
    // The host-staged transport: a rank's part for itself is a device copy (or nothing), every peer's
    // part of every payload goes to host memory in one packed buffer, the transport's
    // all-to-all-v moves the bytes, and the received parts go back to the device.
    // pinned staging for the host-staged exchange (an asynchronous copy to or from pageable memory
    // is staged by the runtime itself; pinned buffers keep every leg inside the stream)
    struct PinnedBuf {
        char *p = nullptr;
        size_t cap = 0;
        char *get(size_t n) {
            if (n > cap) {
                if (p) (void)hipHostFree(p);
                p = nullptr;
                cap = 0;
                const size_t nc = std::max<size_t>(n + n / 2, 1 << 16);
                HIPCHK(hipHostMalloc((void **)&p, nc, hipHostMallocDefault));
                cap = nc;
            }
            return p;
        }
        void release() {
            if (p) (void)hipHostFree(p);
            p = nullptr;
            cap = 0;
        }
    };
    PinnedBuf hx_send, hx_recv;
    void exchange_host(const std::vector<Payload> &P, int line) {
        for (const Payload &p : P) {
            coll_guard(line, p.elem);
            const XPlan &x = (*p.plans)[0];
            const uint64_t own = x.send_cnt[rank];
            if (own && !p.self_in_place)
                HIPCHK(hipMemcpyAsync((char *)p.recv[0] + x.recv_off[rank] * p.elem,
                                      (const char *)p.send[0] + x.send_off[rank] * p.elem, own * p.elem,
                                      hipMemcpyDeviceToDevice, stream));
            std::vector<uint64_t> so(W, 0), sb(W, 0), ro(W, 0), rb(W, 0);
            uint64_t ts = 0, tr = 0;
            for (int q = 0; q < W; q++) {
                if (q == rank) continue;
                so[q] = ts; sb[q] = x.send_cnt[q] * p.elem; ts += sb[q];
                ro[q] = tr; rb[q] = x.recv_cnt[q] * p.elem; tr += rb[q];
            }
            char *hs = hx_send.get(std::max<size_t>(ts, 1)), *hr = hx_recv.get(std::max<size_t>(tr, 1));
            for (int q = 0; q < W; q++)
                if (sb[q])
                    HIPCHK(hipMemcpyAsync(hs + so[q], (const char *)p.send[0] + x.send_off[q] * p.elem, sb[q],
                                          hipMemcpyDeviceToHost, stream));
            HIPCHK(hipStreamSynchronize(stream));
            if (tx.alltoallv(tx.user, hs, so.data(), sb.data(), hr, ro.data(), rb.data()) != 0)
                throw Fail(RMC_E_COMM, "transport alltoallv failed");
            for (int q = 0; q < W; q++)
                if (rb[q])
                    HIPCHK(hipMemcpyAsync((char *)p.recv[0] + x.recv_off[q] * p.elem, hr + ro[q], rb[q],
                                          hipMemcpyHostToDevice, stream));
            HIPCHK(hipStreamSynchronize(stream));
        }
    }

    // A shard's part for itself never goes through RCCL: a device copy (or nothing, self_in_place).
    void exchange(const std::vector<Payload> &P, int line = __builtin_LINE()) {
        if (hostx) {
            exchange_host(P, line);
            return;
        }
        if (!rccl) {
            for (const Payload &p : P)
                for (const Xfer &x : transfers(*p.plans))
                    if (!(p.self_in_place && x.from == x.to))
                        HIPCHK(hipMemcpyAsync((char *)p.recv[x.to] + x.dst_off * p.elem,
                                              (const char *)p.send[x.from] + x.src_off * p.elem, x.n * p.elem,
                                              hipMemcpyDeviceToDevice, stream));
            return;
        }
#ifdef RMC_WITH_RCCL
        if (!self_rccl)
            for (const Payload &p : P) {
                const XPlan &x = (*p.plans)[0];
                const uint64_t n = x.send_cnt[rank];
                if (n && !p.self_in_place)
                    HIPCHK(hipMemcpyAsync((char *)p.recv[0] + x.recv_off[rank] * p.elem,
                                          (const char *)p.send[0] + x.send_off[rank] * p.elem, n * p.elem,
                                          hipMemcpyDeviceToDevice, stream));
            }
        if (W == 1 && !self_rccl) return;
        if (ncclGroupStart() != ncclSuccess) throw Fail(RMC_E_COMM, "ncclGroupStart failed");
        for (const Payload &p : P) {
            const XPlan &x = (*p.plans)[0];
            for (int peer = 0; peer < W; peer++) {
                if (peer == rank && !self_rccl) continue;
                const uint64_t ns = x.send_cnt[peer], nr = x.recv_cnt[peer];
                if (ns && ncclSend((const char *)p.send[0] + x.send_off[peer] * p.elem, ns * p.elem, ncclUint8, peer,
                                   comm, stream) != ncclSuccess)
                    throw Fail(RMC_E_COMM, "ncclSend failed");
                if (nr && ncclRecv((char *)p.recv[0] + x.recv_off[peer] * p.elem, nr * p.elem, ncclUint8, peer, comm,
                                   stream) != ncclSuccess)
                    throw Fail(RMC_E_COMM, "ncclRecv failed");
            }
        }
        if (ncclGroupEnd() != ncclSuccess) throw Fail(RMC_E_COMM, "ncclGroupEnd failed");
#endif
    }

    // Fault injection (tests only, RMC_FAULT_INJECT="site,shard,round[,level]"): the allocation at
    // `site` of the sharded round fails on that shard, as a full device would make it fail.  Sites:
    // 1 send buffer, 2 receive buffer, 3 owner (seen set / election table), 4 outbox, 5 regrouped
    // winners, 6 winner inbox, 7 next-level append (ring, offsets, trace, scan scratch),
    // 8 entering the sharded layout.  Every shard must then stop with RMC_E_MEMORY in the same round.
    int fi_site = 0, fi_shard = -1, fi_level = -1;
    int64_t fi_round = -1;
    void inject(int site, int shard, uint64_t round, int level) const {
        if (site == fi_site && shard == fi_shard && (int64_t)round == fi_round && (fi_level < 0 || level == fi_level))
            throw Fail(RMC_E_MEMORY, "injected allocation failure (RMC_FAULT_INJECT site " + std::to_string(site) + ")");
    }
    bool injecting(int site, int shard, uint64_t round, int level) const {
        return site == fi_site && shard == fi_shard && (int64_t)round == fi_round && (fi_level < 0 || level == fi_level);
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
        int32_t iv[7];
        replicated = multi && shard_min > 1;
        if (!multi && init_cached) {
            // Init's record, fingerprint and invariant verdicts are fixed by the configuration:
            // one kernel puts the level in place (no copies, no host round trip)
            Shard &s = sh[0];
            std::memcpy(iv, init_iv, sizeof iv);
            s.level_start = {0};
            s.cur_wbase = s.nxt_words = 0;
            launch_init_level(s.R, d_init_rec, rw, s.cur_off, d_init_fp, s.seen(), stream);
            s.hpar.set(0, ~0ull);
            s.hslot.set(0, 0);
            s.tflushed = 1;
            s.cur_n = 1;
            s.cur_words = rw;
            s.T_count = 1;
        } else {
            init_full(rec, rw, iv);
        }
        total_generated = 1;  // TLC counts the initial state as generated
        total_distinct = 1;
        depth = 1;
        inited = true;
        status = RMC_OK;
        return init_verdict(iv, rw, t0, st);
    }

    // First Init of the run (or every Init of a sharded run): record, fingerprint and invariants
    // on the device; the single-GPU path caches them for later runs (rmc_reset).
    void init_full(const std::vector<uint32_t> &rec, uint32_t rw, int32_t *iv) {
        HIPCHK(hipMemcpy(d_one, rec.data(), RECW * 4, hipMemcpyHostToDevice));
        KParams P = base(sh[0]);
        P.front = d_one;
        P.fp = d_fp1;
        ks.fp_states(P, 1, stream);
        ks.inv_states(P, 1, d_inv, stream);
        uint32_t owner = 0;  // the shard whose seen set takes Init's fingerprint
        if (multi && !replicated) {
            launch_owner_of(d_fp1, (uint32_t)W, d_cnt1, stream);
            owner = d2h(d_cnt1);
            glevel = {0};
            L_shard = 1;
        }
        HIPCHK(hipMemcpyAsync(iv, d_inv, 7 * sizeof(int32_t), hipMemcpyDeviceToHost, stream));
        HIPCHK(hipStreamSynchronize(stream));
        if (!multi) {
            if (!d_init_rec) {
                d_init_rec = dmalloc<uint32_t>(RECW);
                d_init_fp = dmalloc<ulonglong2>(1);
            }
            HIPCHK(hipMemcpyAsync(d_init_rec, d_one, RECW * 4, hipMemcpyDeviceToDevice, stream));
            HIPCHK(hipMemcpyAsync(d_init_fp, d_fp1, 16, hipMemcpyDeviceToDevice, stream));
            std::memcpy(init_iv, iv, sizeof init_iv);
            init_cached = true;
        }
        const uint64_t zero = 0;
        for (Shard &s : sh) {
            s.level_start = {0};
            s.cur_n = 0;
            s.cur_wbase = s.cur_words = s.nxt_words = 0;
            // Init is global index 0 of level 1: block 0, shard 0 (W > 1 from the start)
            const bool holds = replicated || !multi ? &s == &sh[0] : s.id == 0;
            if (multi && !replicated && (uint32_t)s.id == owner) {
                launch_insert_fps(d_fp1, 1, s.seen(), stream);
                s.T_count = 1;
            }
            if (!holds) continue;
            HIPCHK(hipMemcpyAsync(s.R, d_one, rw * 4, hipMemcpyDeviceToDevice, stream));
            HIPCHK(hipMemcpyAsync(s.cur_off, &zero, 8, hipMemcpyHostToDevice, stream));
            if (!multi || replicated) launch_insert_fps(d_fp1, 1, s.seen(), stream);
            s.hpar.set(0, ~0ull);
            s.hslot.set(0, 0);
            s.tflushed = 1;
            s.cur_n = 1;
            s.cur_words = rw;
            if (!multi || replicated) s.T_count = 1;
        }
        HIPCHK(hipStreamSynchronize(stream));
    }

    int init_verdict(const int32_t *iv, uint32_t rw, std::chrono::steady_clock::time_point t0, rmc_level_stats *st) {
        for (uint32_t o = inv_order; o; o >>= 4) {
            const int b = (int)(o & 15u) - 1;
            if (iv[b] != 1) {
                status = iv[b] == 0 ? RMC_VIOLATION : RMC_EVAL_ERROR;
                violated = b;
                err_ref = 0;
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
        if (replicated && sh[0].cur_n >= shard_min) {
            // a failure here is this rank's alone: it is held and agreed at the sharded level's
            // first collective, so no rank waits in it for a peer that already left
            try {
                inject(8, sh[0].id, 0, (int)sh[0].level_start.size());
                enter_sharded();
            } catch (const Fail &e) {
                pending_fail = e.code;
                pending_msg = e.msg;
                replicated = false;
            }
        }
        return (!multi || replicated) ? step_single(st) : step_sharded(st);
    }

    // Replicated -> sharded, at the start of the first level with >= shard_min states.  Every
    // shard holds that level whole (RCCL: each rank its own copy; virtual: shard 0), and every
    // state seen so far in its seen set (a superset of what it owns).  Shard t keeps the blocks
    // b = t, t + W, ... of B = chunk_parents parents (the level's block-cyclic layout) in a fresh
    // ring, their offsets rebased, their trace entries moved to the local gids of that layout.
    // Earlier levels stay replicated: global id == local gid, answered by shard 0 / rank 0.
    void enter_sharded() {
        sync_trace();  // the replicated levels' trace is read below
        Shard &s0 = sh[0];
        const size_t Lz = s0.level_start.size();
        const uint64_t F = s0.cur_n, base = s0.level_start[Lz - 1], B = chunk_parents;
        HIPCHK(hipStreamSynchronize(stream));
        glevel = s0.level_start;
        L_shard = (int)Lz;
        std::vector<uint64_t> hoff(F + 1);
        if (F) HIPCHK(hipMemcpy(hoff.data(), s0.cur_off, F * 8, hipMemcpyDeviceToHost));
        hoff[F] = s0.cur_words;
        uint32_t *src = s0.R;
        const uint64_t src_cap = s0.rcap, src_wbase = s0.cur_wbase;
        // A ring already at its budget (the seen set went compact during the replicated levels)
        // is rebuilt at the budget once the old ring is gone: allocating the new one at the old
        // one's size first would need the budget twice.
        const bool was_fixed = s0.ring_fixed;
        uint64_t *src_off = s0.cur_off;
        std::vector<uint32_t *> old_rings;
        for (size_t ti = sh.size(); ti-- > 0;) {  // shard 0 last: its trace entries move in place
            Shard &t = sh[ti];
            const int id = t.id;
            uint64_t n = 0, words = 0;
            for (uint64_t b = (uint64_t)id; b * B < F; b += (uint64_t)W) {
                const uint64_t lo = b * B, hi = std::min(F, lo + B);
                n += hi - lo;
                words += hoff[hi] - hoff[lo];
            }
            uint64_t cap = std::max<uint64_t>(words + words / 2, 1ull << 14);
            uint32_t *nr = dmalloc<uint32_t>(cap);
            uint64_t *noff = dmalloc<uint64_t>(std::max<uint64_t>(n + n / 2, 1 << 16));
            uint64_t at = 0, wat = 0;
            for (uint64_t b = (uint64_t)id; b * B < F; b += (uint64_t)W) {
                const uint64_t lo = b * B, hi = std::min(F, lo + B), w = hoff[hi] - hoff[lo];
                const uint64_t from = ring_wrap(src_wbase + hoff[lo], src_cap);
                const uint64_t n1 = std::min(w, src_cap - from);
                if (n1) HIPCHK(hipMemcpyAsync(nr + wat, src + from, n1 * 4, hipMemcpyDeviceToDevice, stream));
                if (w > n1) HIPCHK(hipMemcpyAsync(nr + wat + n1, src, (w - n1) * 4, hipMemcpyDeviceToDevice, stream));
                launch_rebase(src_off + lo, hi - lo, hoff[lo] - wat, noff + at, stream);
                // trace entries: global id base + g -> local gid base + local index (at <= lo: a
                // forward in-place move on shard 0)
                for (uint64_t i = 0; i < hi - lo; i++) {
                    t.hpar.set(base + at + i, s0.hpar.get(base + lo + i));
                    t.hslot.set(base + at + i, s0.hslot.get(base + lo + i));
                }
                at += hi - lo;
                wat += w;
            }
            HIPCHK(hipStreamSynchronize(stream));
            if (&t != &s0) {
                // the seen set so far (virtual shards share one device)
                if (s0.Tc) {
                    if (!t.Tc || t.T_cap != s0.T_cap) {
                        dfree(t.T);
                        dfree(t.Tc);
                        t.T = nullptr;
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
                t.epoch = std::max(t.epoch, s0.epoch);
                dfree(t.R);
                dfree(t.cur_off);
            } else if (was_fixed && sh.size() == 1) {
                // a rank's ring already at its budget stays: its part of the level goes back to the
                // ring's start (freeing and allocating ~100 GB again took ~3 s on MI355X)
                old_off_ = s0.cur_off;
                if (words) HIPCHK(hipMemcpyAsync(s0.R, nr, words * 4, hipMemcpyDeviceToDevice, stream));
                HIPCHK(hipStreamSynchronize(stream));
                dfree(nr);
                nr = s0.R;
                cap = src_cap;
            } else {
                old_rings.push_back(s0.R);
                old_off_ = s0.cur_off;
            }
            t.R = nr;
            t.rcap = cap;
            t.ring_fixed = false;
            t.cur_off = noff;
            t.cur_off_cap = std::max<uint64_t>(n + n / 2, 1 << 16);
            t.cur_wbase = 0;
            t.cur_words = words;
            t.nxt_words = 0;
            t.cur_n = n;
            t.nxt_n = 0;
            t.tflushed = base + n;
            t.tdev = t.tflushed;
        }
        HIPCHK(hipStreamSynchronize(stream));
        for (uint32_t *r : old_rings) dfree(r);
        dfree(old_off_);
        old_off_ = nullptr;
        if (was_fixed)
            for (Shard &t : sh) fix_ring(t, sh.size());  // (a kept ring: already at its budget)
        replicated = false;
    }
    uint64_t *old_off_ = nullptr;
    int pending_fail = 0;  // a failure entering the sharded layout, agreed at the next level's start
    std::string pending_msg;

    // First error in TLC order among the error slots: smaller (parent, slot) first; on a
    // tie the Assert wins (its sub-action's batch is discarded).
    // the chunk summary's flag word (KParams::flags[0]): what stopped the level
    std::string flag_msg(unsigned long long f) const {
        if (f & 1u) return "a state exceeds msg_cap = " + std::to_string(ks.MCAP) + " messages";
        if (f & 2u) return "internal: a split chunk's parent records are not consecutive in the frontier ring";
        if (f & 4u) return "race probe: the commit's arrival counters were not all re-armed when the level finished";
        return "internal: unknown flag " + std::to_string(f);
    }
    // the return code of a chunk's flags: a state past msg_cap (bit 0) is a capacity failure, anything
    // else an internal invariant of the engine that failed (RMC_E_STATE)
    static int flag_code(unsigned long long f) { return (f & 1u) ? RMC_E_CAPACITY : RMC_E_STATE; }

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
    // `ahead` epochs could reuse a tag still in E, clear it (all tags are nonzero).
    void renew_election_tags(Shard &s, uint32_t ahead) {
        if (!s.E || s.epoch + ahead - s.lxy_epoch0 < 0xFFFFu) return;
        launch_eslot_clear(s.E, s.lcap, stream);
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
        uint64_t level_gen = 0, level_self = 0;
        s.nxt_n = 0;
        s.nxt_words = 0;
        const uint64_t MSW = (uint64_t)ks.maxsucc * (uint64_t)ks.RECW_MAX;
        for (uint64_t p0 = 0; p0 < s.cur_n; p0 += chunk_parents) {
            const uint64_t p1 = std::min(s.cur_n, p0 + chunk_parents), np_ = p1 - p0;
            // Small chunks size the next level, trace and seen set on the successor upper bound
            // without a host round trip; large ones read the winner count back before commit.
            const uint64_t Gub = np_ * (uint64_t)ks.maxsucc;
            maybe_migrate(s, s.T_count + Gub);
            // where the chunk's first record starts (the ring words before it are consumed): read here only
            // for a chunk that may size on its bound; a larger one reads it with its winner count (no round
            // trip of its own while the device idles)
            const bool may_small = Gub <= (1ull << 20);
            uint64_t consumed = (s.ring_fixed && p0 && may_small) ? d2h(s.cur_off + p0) : 0;
            // bounds that a fixed ring or a compact seen set cannot take go the exact way
            const bool small = may_small && seen_room(s, s.T_count + Gub) && ring_room(s, np_ * MSW, consumed);
            if (small) {
                ensure_ring(s, np_ * MSW, consumed);
                ensure_off(s.nxt_off, s.nxt_off_cap, s.nxt_n, s.nxt_n + Gub);
                grow_trace(s, Gub);
                grow_seen(s, s.T_count + Gub);
            }
            ensure_chunk(s, Gub);
            const uint64_t Lcap = std::min(next_pow2(2 * Gub), s.lcap);
            renew_election_tags(s, 1);
            ++s.epoch;
            trace_restart(s);
            // chunks of many parents probe and elect in a pass of their own, a lane per successor
            const bool split = split_min && np_ >= split_min;
            // a split chunk's winners go into the seen set in its commit (k_commit_items reads the
            // election words itself: no k_insert_winners pass) when the items commit takes its slots
            const bool fold = split && ks.maxsucc <= 256;
            auto params = [&] {
                KParams Q = chunk_params(s);
                Q.p_begin = p0; Q.p_end = p1; Q.next_base = s.nxt_n; Q.next_wbase = s.nxt_words;
                Q.gid_next_base = gid_nxt; Q.gid_parent_base = gid_cur;
                Q.Lmask = Lcap - 1;
                Q.epoch = s.epoch;
                // (a chunk whose 256-lane commit cannot take a parent's slots -- the BecomeFollower variant at
                // n >= 4 -- inserts its winners in a pass of its own, k_insert_winners, and leaves the verdicts
                // in lslot for k_commit_split)
                Q.split = split ? (fold ? 1 : 7) : 0;
                Q.plist = split ? s.plist : nullptr;
                // (a split chunk's self-loops are staged after the successors to fingerprint)
                Q.hcnt = split ? s.hcnt : nullptr;
                // (the dense slot layout: chunks whose winners the items commit takes -- k_insert_winners and
                // k_commit_split read the sparse one)
                Q.hoff = fold ? s.hoff : nullptr;
                s.chunk_sep = Q.hcnt != nullptr;
                s.chunk_dense = Q.hoff != nullptr;
                return Q;
            };
            // expand + fingerprint + seen-set probe + staging, one evaluation per parent (a split
            // chunk: expand + staging + hash context, then fingerprint + probe + election a lane per successor)
            // (the chunk's self-loops: counted by the fused expansion or the split chunk's winner count; the
            // fused expansion's stripes are cleared with the sum, in case an earlier chunk stopped between its
            // expansion and its commit)
            HIPCHK(hipMemsetAsync(s.sum + SUM_SELF, 0, (SUM_SELF_STRIPE + SELF_STRIDE * SELF_STRIPES - SUM_SELF) * 8, stream));
            timed(PH_HASH, [&] {
                if (split) ks.split(params(), stream);
                else ks.fused(params(), stream);
            });
            if (split) timed(PH_OTHER, [&] { ks.hash_probe(params(), np_, stream); });
            timed(PH_DEDUP, [&] {
                ks.wincount(params(), np_, stream);
                if (split) launch_nzlist(params(), np_, stream);
            });
            if (!small) {
                HIPCHK(hipMemcpyAsync(s.hsum, s.sum, 8 * 8, hipMemcpyDeviceToHost, stream));
                unsigned long long *hc = s.hsum + SUM_WORDS_TOTAL - 1;  // (a pinned word nothing else uses here)
                const bool read_consumed = s.ring_fixed && p0 && !may_small;
                if (read_consumed) HIPCHK(hipMemcpyAsync(hc, s.cur_off + p0, 8, hipMemcpyDeviceToHost, stream));
                HIPCHK(hipStreamSynchronize(stream));
                if (read_consumed) consumed = *hc;
                collect_times(st);
                const uint64_t Wub = s.hsum[1], Wwords = s.hsum[SUM_WORDS];
                ensure_ring(s, Wwords, consumed);
                ensure_off(s.nxt_off, s.nxt_off_cap, s.nxt_n, s.nxt_n + Wub);
                grow_trace(s, Wub);
                grow_seen(s, s.T_count + Wub);
            }
            trace_fence(s);
            // (timed with the winner count: PH_OTHER stays the probe pass alone)
            if (split && !fold) timed(PH_DEDUP, [&] { ks.insert(params(), np_, stream); });
            // + chunk summary; a split chunk's winners a lane per successor slot of its parents with winners
            timed(PH_MAT, [&] {
                if (split) ks.commit_split(params(), np_, stream);
                else ks.commit(params(), stream);
            });
            HIPCHK(hipMemcpyAsync(s.hsum, s.sum, (SUM_SELF + 1) * 8, hipMemcpyDeviceToHost, stream));
            HIPCHK(hipStreamSynchronize(stream));
            HIPCHK(hipGetLastError());
            collect_times(st);
            const uint64_t G = s.hsum[0], Wn = s.hsum[1], Ww = s.hsum[SUM_WORDS];
            level_self += s.hsum[SUM_SELF];
            if (s.hsum[2 + ERR_NSLOTS]) throw Fail(flag_code(s.hsum[2 + ERR_NSLOTS]), flag_msg(s.hsum[2 + ERR_NSLOTS]));
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
        st->self_loops = level_self;
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
    // device-loop submission shape (tuning knobs, read once): levels per group, groups queued ahead,
    // microseconds of waiting for a group between stream queries
    static int env_int(const char *name, int dflt, int lo, int hi) {
        const char *v = std::getenv(name);
        if (!v || !*v) return dflt;
        return std::max(lo, std::min(hi, std::atoi(v)));
    }
    // parents per host-driven chunk from which the seen-set probe and election run as their own
    // pass (k_probe; 0 = always fused into the expansion)
    const uint64_t split_min = (uint64_t)env_int("RMC_SPLIT_MIN", 1 << 16, 0, 1 << 30);
    const int dl_group = env_int("RMC_DL_GROUP", 2, 1, 64);
    const int dl_ahead = env_int("RMC_DL_AHEAD", 2, 1, 64);
    const int dl_query_us = env_int("RMC_DL_QUERY_US", 2000, 0, 1 << 30);
    int batch_levels() const { return cfg.device_levels ? (int)cfg.device_levels : LREC_CAP; }
    uint64_t dev_parents() const { return std::min<uint64_t>(chunk_parents, 1ull << 15); }
    bool batch_ok() const {
        const Shard &s = sh[0];
        const uint64_t first = s.cur_n * (uint64_t)ks.maxsucc;
        return (!multi || (replicated && s.cur_n < shard_min)) && inited && !finished && cfg.device_levels != 1 &&
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
        trace_fence(s);
        LevelCtl &h = *s.hctl;
        std::memset(&h, 0, sizeof h);
        h.cur_n = s.cur_n;
        h.gid_cur = gid0;
        h.T_count = s.T_count;
        ensure_chunk(s, DP * MS);
        h.Lmask = std::min(next_pow2(2 * s.cur_n * MS), s.lcap) - 1;
        h.cur_wbase = s.cur_wbase;
        h.cur_words = s.cur_words;
        h.off_cap = std::min(s.cur_off_cap, s.nxt_off_cap);
        h.rcap = s.rcap;
        h.trace_base = s.tdev;
        h.trace_cap = s.trace_cap;
        h.T_cap = s.Tc ? (uint64_t)((double)s.T_cap * 1.8) : s.T_cap;  // compact: load <= 0.9
        h.chunk_parents = replicated ? std::min<uint64_t>(DP, shard_min - 1) : DP;  // stop before sharding starts
        h.Lcap_max = s.lcap;
        h.level = (uint32_t)L0;
        renew_election_tags(s, K + 1);
        h.epoch = ++s.epoch;
        h.stop = CTL_RUN;
        h.batch = (uint32_t)K;
        __atomic_store_n(&s.hloop->done, 0u, __ATOMIC_RELAXED);
        __atomic_store_n(&s.hloop->stop, (uint32_t)CTL_RUN, __ATOMIC_RELEASE);
        launch_set_ctl(s.ctl, 2, h, s.sum, stream);
        uint64_t *offs[2] = {s.cur_off, s.nxt_off};
        std::vector<size_t> mark(K);
        // Levels go in groups of GL.  The loop's progress is mirrored into pinned host memory
        // (HostLoop, system-scope stores): each level's expansion reports the levels done before it
        // as it starts, finish_level reports the stop -- so nothing but kernels sits in the stream
        // (an event or a copy between groups would be a hand-off of 6-10 us idle).  Group g + 2 is enqueued only once group g has finished with the loop
        // still running, so the device always has a group queued and at most two groups of no-op
        // launches follow the last level.
        // GL = 2: the first kernel of every group submitted while the loop runs starts ~5.8 us
        // late (measured with reports at either end of a level and with a stream query right after
        // each submission); two levels per group halve that against one, and the no-op tail after
        // the last level stays at most two groups
        const int GL = dl_group, ngroups = (K + GL - 1) / GL;
        auto enqueue_group = [&](int g) {
            for (int i = g * GL; i < std::min(K, (g + 1) * GL); i++) {
                mark[i] = evrecs.size();
                KParams Q = chunk_params(s);
                Q.foff = offs[i & 1];
                Q.noff = offs[(i + 1) & 1];
                Q.ctl = s.ctl + (i & 1);
                Q.ctl_next = s.ctl + ((i + 1) & 1);
                Q.lrec = s.lrec;
                Q.hloop = s.dloop;
                Q.p_begin = 0;
                Q.p_end = DP;  // grids are sized on the bound; the kernels read the level from ctl
                timed(PH_HASH, [&] { ks.fused(Q, stream); });
                timed(PH_DEDUP, [&] { ks.wincount(Q, DP, stream); });
                timed(PH_MAT, [&] { ks.commit(Q, stream); });
            }
        };
        // true once group g has finished (or the loop stopped); a stream error ends the wait
        // The stream is queried only after dl_query_us of waiting (then every dl_query_us): a
        // hipStreamQuery while the loop runs cost ~2 % of configs[1]'s exhaustion when it was
        // issued every 256 spins (measured, tools/dl_sweep.sh).
        auto group_done = [&](int g) {
            const uint32_t need = (uint32_t)std::min(K, (g + 1) * GL);
            auto tq = std::chrono::steady_clock::now() + std::chrono::microseconds(dl_query_us);
            for (uint32_t spin = 0;; spin++) {
                if (__atomic_load_n(&s.hloop->stop, __ATOMIC_ACQUIRE) != (uint32_t)CTL_RUN) return false;
                if (__atomic_load_n(&s.hloop->done, __ATOMIC_ACQUIRE) >= need) return true;
                if ((spin & 255u) == 255u && std::chrono::steady_clock::now() >= tq) {
                    tq = std::chrono::steady_clock::now() + std::chrono::microseconds(dl_query_us);
                    const hipError_t q = hipStreamQuery(stream);
                    if (q == hipSuccess) {  // drained (the mirror may still lag: the caller reads the device's block)
                        if (__atomic_load_n(&s.hloop->stop, __ATOMIC_ACQUIRE) != (uint32_t)CTL_RUN) return false;
                        return __atomic_load_n(&s.hloop->done, __ATOMIC_ACQUIRE) >= need;
                    }
                    if (q != hipErrorNotReady) HIPCHK(q);
                }
            }
        };
        int enq = 0;
        for (; enq < std::min(dl_ahead, ngroups); enq++) enqueue_group(enq);
        for (; enq < ngroups; enq++) {
            if (!group_done(enq - dl_ahead)) break;
            enqueue_group(enq);
        }
        for (int i = enq * GL; i < K; i++) mark[i] = evrecs.size();
        HIPCHK(hipStreamSynchronize(stream));
        HIPCHK(hipGetLastError());
        // The control block and the level records as the device holds them.  The pinned mirror is
        // for the progress polls only: its last system-scope writes can still be in flight when the
        // stream reports drained, and a poll that read a lagging `done` stops enqueueing while the
        // loop still runs -- the mirror's control block is then an earlier batch's (two rank
        // processes on one MI355X: a spurious error or a count off by one about one run in ten).
        // (both in one wait: the records of every level the batch may have run; pinned targets)
        HIPCHK(hipMemcpyAsync(s.hctl, s.ctl, 2 * sizeof(LevelCtl), hipMemcpyDeviceToHost, stream));
        HIPCHK(hipMemcpyAsync(s.hlrec, s.lrec, sizeof(LevelRec) * K, hipMemcpyDeviceToHost, stream));
        HIPCHK(hipStreamSynchronize(stream));
        // the pair's newer block: more levels done, or (an error stops without advancing) the stopped one
        const LevelCtl &c0 = s.hctl[0], &c1 = s.hctl[1];
        LevelCtl c = (c1.done_levels > c0.done_levels || (c1.done_levels == c0.done_levels && c1.stop != CTL_RUN)) ? c1 : c0;
        const int D = (int)c.done_levels;
        if (D > K) throw Fail(RMC_E_STATE, "device level loop ran past its batch");
        if (c.stop == CTL_RUN) {  // enqueueing stopped first: the levels done stand, the next batch goes on
            c.stop = CTL_HOST;
            *s.hctl = c;
        }
        if (c.stop == CTL_ERROR) {  // the erroring level's summary (error keys, winners) for the host path
            HIPCHK(hipMemcpyAsync(s.hsum, s.sum, 8 * 8, hipMemcpyDeviceToHost, stream));
            HIPCHK(hipStreamSynchronize(stream));
        }
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
            st->self_loops = r.self_loops;
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
        // a run that ended without an error reads its trace only for rmc_state_path: no flush now
        s.trace_end = c.gid_cur + c.cur_n;
        if (!(finished && status == RMC_DONE)) flush_trace(s, s.trace_end);
        seconds += el;
        if (c.stop == CTL_ERROR) {
            // the level the loop stopped in is intact: report its error as the host path does
            rmc_level_stats *st = &out[D];
            st->seconds = el / nst;
            if (s.hsum[2 + ERR_NSLOTS]) throw Fail(flag_code(s.hsum[2 + ERR_NSLOTS]), flag_msg(s.hsum[2 + ERR_NSLOTS]));
            const int L = (int)s.level_start.size();
            st->level = L;
            st->expanded = s.cur_n;
            const uint64_t gid_cur = s.level_start[L - 1];
            flush_trace(s, gid_cur + s.cur_n + s.hsum[1]);  // the error level's winners
            s.T_count += s.hsum[1];
            unsigned long long best;
            const int kind = first_error(s.hsum + 2, &best);
            if (kind < 0) throw Fail(RMC_E_STATE, "device level loop stopped without an error");
            s.chunk_sep = false;  // (device-loop levels stage every successor, sparse)
            s.chunk_dense = false;
            stop_on_error(kind, best, 0, 0, gid_cur, gid_cur + s.cur_n, 0, st);
        }
        HIPCHK(hipStreamSynchronize(stream));
        return nst;
    }

    // The erroring chunk's share of TLC's counters at its first error (key ek, level-local parent
    // p of the chunk starting at p0): successors generated by the chunk's parents up to the error
    // (the whole sub-action batch of an invariant error -- TLC adds a batch before fingerprinting
    // it -- none of an Assert's), and the chunk's winners before it.
    struct ErrCounts { uint64_t gen, win; };
    ErrCounts error_counts(Shard &s, int kind, unsigned long long ek, uint64_t p0, bool route) {
        HIPCHK(hipStreamSynchronize(stream));
        const uint64_t p = ek >> 24;
        const uint32_t slot = (uint32_t)((ek >> 8) & 0xFFFF);
        const uint64_t pl = p - p0;
        uint64_t off_p = 0;
        if (pl) {
            std::vector<uint32_t> cn(pl);
            HIPCHK(hipMemcpy(cn.data(), s.cnt, pl * 4, hipMemcpyDeviceToHost));
            for (uint32_t x : cn) off_p += x;
        }
        const uint64_t wbase = (uint64_t)d2h(s.boff + pl / WTILE) + d2h(s.wpos + pl);
        // p's winners whose slot key is below `bound` (TLC order = slot-key order).  p's staged slots
        // hold its successors in TLC order -- in a split chunk that set self-loops apart (hcnt) only
        // the others, which are the only ones that can win -- each with its key (stage_succ, word 6)
        const uint32_t nslots = s.chunk_sep ? d2h(s.hcnt + pl) : d2h(s.cnt + pl);
        auto winners_below = [&](uint32_t bound) -> uint64_t {
            if (!nslots) return 0;
            std::vector<uint32_t> ls(nslots);
            std::vector<uint4> st((size_t)nslots * sw4());
            const uint64_t q0 = s.chunk_dense ? (uint64_t)d2h(s.hoff + pl) : pl * ks.maxsucc;  // its first slot
            HIPCHK(hipMemcpy(ls.data(), s.lslot + q0, nslots * 4, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(st.data(), s.score + q0 * sw4(), (size_t)nslots * sw4() * 16, hipMemcpyDeviceToHost));
            uint64_t w = 0;
            for (uint32_t r = 0; r < nslots; r++) {
                if ((st[(size_t)r * sw4() + 1].z & 0xFFFFu) >= bound) continue;
                // (LS_WIN: an owner's verdict, or a split chunk's after k_insert_winners)
                w += ls[r] == LS_WIN ||
                     (!route && ls[r] < LS_ELECT && ((uint32_t)d2h(&s.E[ls[r]].k) >> 2) == (uint32_t)(pl * ks.maxsucc + r));
            }
            return w;
        };
        // successors of p, in order, to find the sub-action batch boundaries
        record_to_one(s, p);
        std::vector<uint32_t> keys;
        bool af = false;
        expand_one(&keys, nullptr, nullptr, &af);
        const uint32_t grp = slot >> 7;  // (server, action)
        uint32_t cut = 0, batch_end = 0, before = 0;
        for (uint32_t k : keys) {
            if ((k >> 7) < grp) cut++;
            if ((k >> 7) <= grp) batch_end++;
            if (k < slot) before++;
        }
        (void)before;
        if (kind == ERR_INV || kind == ERR_EVAL) return {off_p + batch_end, wbase + winners_below(slot)};
        if (kind == ERR_ASSERT) return {off_p + cut, wbase + winners_below(grp << 7)};
        return {off_p, wbase};
    }

    // TLC's counters at the moment the first error (in -workers 1 order) is reported.
    void stop_on_error(int kind, unsigned long long ek, uint64_t p0, uint64_t nxt_before, uint64_t gid_cur,
                       uint64_t gid_nxt, uint64_t gen_before_chunk, rmc_level_stats *st) {
        Shard &s = sh[0];
        const uint64_t p = ek >> 24;
        const int which = (int)(ek & 0xFF);
        const ErrCounts ec = error_counts(s, kind, ek, p0, false);
        const uint64_t gen = gen_before_chunk + ec.gen, winners_before = ec.win;
        if (kind == ERR_INV || kind == ERR_EVAL) {
            err_ref = gid_nxt + nxt_before + winners_before;
            total_distinct += nxt_before + winners_before + 1;
            queue_at_end = (s.cur_n - p - 1) + nxt_before + winners_before;
            status = kind == ERR_INV ? RMC_VIOLATION : RMC_EVAL_ERROR;
            violated = which;
            depth = (int)s.level_start.size() + 1;
        } else {
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

    // ---- sharded level (W > 1) ------------------------------------------------------------------
    // The level is laid out block-cyclically (glevel): round c expands the global blocks cW ..
    // cW + W - 1, block cW + t on shard t, so the rounds follow the level's order, and inside a
    // round every successor carries its global key (parent's index in the level, rank among its
    // successors).  Each successor goes to its fingerprint's owner shard, which drops those its
    // seen set holds and elects the smallest key per new fingerprint: the successor TLC -workers 1
    // meets first (Raft.tla:34-38 -- the VIEW hides variables, so which representative of a class
    // is kept depends on that order).  The verdicts come back, every shard commits its winners in
    // TLC order (the fused winner count + commit), and the winners go to the shards that own their
    // global next-level indices, appended in source order -- the level's order.  Levels, counters
    // at an error and traces are those of W = 1.
    bool round_sep(const Shard &s) const { return split_min && s.np >= split_min; }
    KParams round_params(const Shard &s, uint64_t gbase) const {
        KParams Q = chunk_params(s);
        Q.p_begin = s.p0;
        Q.p_end = s.p0 + s.np;
        Q.route = 1;
        Q.gid_parent_base = gbase + s.gblk - s.p0;  // level-local parent p -> its global id
        Q.next = s.ob;
        Q.noff = s.ooff;
        Q.nbase = 0;
        Q.next_wbase = 0;
        Q.next_base = 0;
        Q.xside = s.oside;
        Q.gid_next_base = 0;
        Q.gblk = s.gblk;
        // a round of many parents: the commit visits only those with winners (k_nzlist, as a split
        // chunk of the single-GPU path; same switches), and its self-loops are set apart -- known seen
        // (the parent's fingerprint is in its owner's seen set), they are neither fingerprinted nor routed
        if (round_sep(s)) {
            Q.plist = s.plist;
            Q.hcnt = s.hcnt;
        }
        Q.trace_base = 0;
        return Q;
    }

    void grow_recv(Shard &o, uint64_t R) {
        if (R + 1 <= o.xr_cap) return;
        const uint64_t nc = std::max<uint64_t>(R + R / 2 + 1, 1024);
        HIPCHK(hipStreamSynchronize(stream));
        dfree(o.xr); dfree(o.rslot); dfree(o.rflag);
        o.xr = dmalloc<XItem>(nc);
        o.rslot = dmalloc<uint32_t>(nc);
        o.rflag = dmalloc<uint32_t>(nc);
        o.xr_cap = nc;
    }
    void grow_outbox(Shard &s, uint64_t words, uint64_t n) {
        if (words + 1 > s.ob_cap || n + 1 > s.os_cap) HIPCHK(hipStreamSynchronize(stream));
        if (words + 1 > s.ob_cap) {
            dfree(s.ob);
            s.ob_cap = std::max<uint64_t>(words + words / 2 + 1, 1 << 16);
            s.ob = dmalloc<uint32_t>(s.ob_cap);
        }
        if (n + 1 > s.os_cap) {
            dfree(s.oside); dfree(s.ooff);
            s.os_cap = std::max<uint64_t>(n + n / 2 + 1, 1 << 12);
            s.oside = dmalloc<uint4>(s.os_cap);
            s.ooff = dmalloc<uint64_t>(s.os_cap);
        }
    }
    void grow_inbox(Shard &o, uint64_t words, uint64_t n) {
        if (words + 1 > o.ib_cap || n + 1 > o.is_cap) HIPCHK(hipStreamSynchronize(stream));
        if (words + 1 > o.ib_cap) {
            dfree(o.ib);
            o.ib_cap = std::max<uint64_t>(words + words / 2 + 1, 1 << 16);
            o.ib = dmalloc<uint32_t>(o.ib_cap);
        }
        if (n + 1 > o.is_cap) {
            dfree(o.iside); dfree(o.isz); dfree(o.ioff);
            o.is_cap = std::max<uint64_t>(n + n / 2 + 1, 1 << 12);
            o.iside = dmalloc<uint4>(o.is_cap);
            o.isz = dmalloc<uint32_t>(o.is_cap);
            o.ioff = dmalloc<uint32_t>(o.is_cap);
        }
    }

    // per-shard round row: generated, winners, words, inserted, error kind + 1, error key, -failure code,
    // self-loops
    static constexpr int TAB = 8;

    int step_sharded(rmc_level_stats *st) {
        auto t0 = std::chrono::steady_clock::now();
        const int L = (int)sh[0].level_start.size();
        st->level = L;
        const uint64_t B = chunk_parents, MS = (uint64_t)ks.maxsucc;
        uint64_t Fg = 0;
        for (Shard &s : sh) { Fg += s.cur_n; s.nxt_n = 0; s.nxt_words = 0; }
        allreduce(&Fg, 1, false);
        {
            uint64_t pend = (uint64_t)(-pending_fail);
            allreduce(&pend, 1, true);
            if (pend) {
                const std::string m = pending_fail ? pending_msg : "another rank failed entering the sharded layout";
                pending_fail = 0;
                throw Fail(-(int)pend, m);
            }
        }
        st->expanded = Fg;
        const uint64_t gbase = glevel[L - 1], rounds = (Fg + B * W - 1) / (B * W);
        const size_t NL = sh.size();
        uint64_t level_gen = 0, level_new = 0, level_words = 0, level_self = 0;
        // A shard that runs out of seen-set or ring room, or meets a state past msg_cap, must not
        // leave the others waiting in a collective: it records the failure, skips its own kernels
        // and keeps exchanging; the round's table (and a last check at the round's end) carries the
        // failure to every rank, and all of them stop with it.
        std::vector<int> fail(NL, 0);
        std::string fail_msg;
        auto guard = [&](size_t li, auto &&f) {
            if (fail[li]) return;
            try {
                f();
            } catch (const Fail &e) {
                fail[li] = e.code;
                fail_msg = e.msg;
            }
        };
        auto agree = [&](uint64_t worst) {  // worst = max over shards of -code (0: all well)
            if (!worst) return;
            throw Fail(-(int)worst, fail_msg.empty() ? std::string("another shard failed (see its rank's error)") : fail_msg);
        };
        // failure agreement: a shard that fails (allocation, capacity) records it and keeps taking
        // part in every exchange; the next gathered matrix / all-reduce carries the failure to every
        // rank and all of them raise it together (agree).  Receive buffers grow before their payload
        // moves, decided from the gathered counts and capacities the same way on every rank, followed
        // by one extra all-reduce only in the rounds where some shard grows.
        auto col_max = [&](const std::vector<uint64_t> &M, int K, int col) {
            uint64_t m = 0;
            for (int t = 0; t < W; t++) m = std::max(m, M[(size_t)t * K + col]);
            return m;
        };
        auto local_worst = [&] {
            uint64_t m = 0;
            for (size_t li = 0; li < NL; li++) m = std::max(m, (uint64_t)(-fail[li]));
            return m;
        };
        auto agree_now = [&] {  // one all-reduce of the worst failure
            uint64_t worst = local_worst();
            allreduce(&worst, 1, true);
            agree(worst);
        };
        std::vector<uint64_t> hoff_buf;  // piece boundaries read back in one copy per round
        std::vector<uint64_t> consumed_(NL, 0);  // per shard: ring words of the current level no longer needed
        for (uint64_t c = 0; c < rounds; c++) {
            // (1) expand the round's block: fingerprints, staged rows; successors per owner
            for (size_t li = 0; li < NL; li++) {
                Shard &s = sh[li];
                s.p0 = c * B;
                s.np = s.cur_n > s.p0 ? std::min<uint64_t>(B, s.cur_n - s.p0) : 0;
                s.gblk = (c * (uint64_t)W + (uint64_t)s.id) * B;
                // inserted counts, self-loops, successors per owner: one memset (sum[SUM_INS .. SUM_OCNT + 32))
                HIPCHK(hipMemsetAsync(s.sum + SUM_INS, 0, (SUM_OCNT + 32 - SUM_INS) * 8, stream));
                // (before any skip: a shard with no parents this round receives items, and they must
                // not bid in E under an earlier round's tag)
                s.lx_bid = false;
                if (!s.np || fail[li]) continue;
                const bool split = split_min && s.np >= split_min;
                // (the fused election table holds a round's successors at load <= 1/2: ensure_chunk)
                s.lx_bid = owner_lxy && split && s.E && s.lcap >= 2 * s.np * MS;
                timed(PH_HASH, [&] {
                    KParams Q = round_params(s, gbase);
                    if (split) {  // fingerprints a lane per successor (route: no probe), counted per owner
                        Q.ocnt = s.ocnt;
                        Q.nown = (uint32_t)W;
                        if (s.lx_bid) {  // ... and the shard's own successors' bids
                            Q.ot_round = lx_table(s);
                            Q.OT = s.E;
                            Q.ot_mask = s.lcap - 1;
                            Q.self = (uint32_t)s.id;
                            Q.gblk = s.gblk;
                        }
                        ks.split(Q, stream);
                        ks.hash_probe(Q, s.np, stream);
                    } else {
                        ks.fused(Q, stream);
                    }
                });
                if (!split) launch_route_count(s.fp, s.cnt, s.np, (uint32_t)MS, (uint32_t)W, s.ocnt, stream);
            }
            // gathered row per shard: its successors per owner, its receive capacity, its failure
            const int K1 = W + 2;
            std::vector<std::vector<uint64_t>> rows(NL, std::vector<uint64_t>(K1, 0));
            for (size_t li = 0; li < NL; li++) {
                Shard &s = sh[li];
                HIPCHK(hipMemcpyAsync(s.hsum, s.ocnt, 64 * 4, hipMemcpyDeviceToHost, stream));
                HIPCHK(hipStreamSynchronize(stream));
                const uint32_t *hc = reinterpret_cast<const uint32_t *>(s.hsum);
                // successors the shard owns itself stay out of the exchange (k_local_elect)
                s.G = 0;
                s.Gself = s.np ? hc[s.id] : 0;
                for (int d = 0; d < W; d++) {
                    rows[li][d] = d == s.id ? 0 : hc[d];
                    s.G += rows[li][d];
                }
                guard(li, [&] {
                    inject(1, s.id, c, L);
                    if (s.G) grow_plain(s.xs, s.xs_cap, s.G);
                });
                rows[li][W] = injecting(2, s.id, c, L) ? 0 : s.xr_cap;  // site 2 forces this shard to grow
                rows[li][W + 1] = (uint64_t)(-fail[li]);
            }
            collect_times(st);
            std::vector<uint64_t> M = gather_rows(rows, K1);
            agree(col_max(M, K1, W + 1));
            {
                std::vector<uint64_t> need(W, 0), cap(W, 0);
                for (int o = 0; o < W; o++) {
                    for (int t = 0; t < W; t++) need[o] += M[(size_t)t * K1 + o];
                    cap[o] = M[(size_t)o * K1 + W];
                }
                if (!must_grow(need, cap).empty()) {
                    for (size_t li = 0; li < NL; li++) {
                        const int id = sh[li].id;
                        if (need[id] + 1 > cap[id])
                            guard(li, [&] {
                                inject(2, id, c, L);
                                grow_recv(sh[li], need[id]);
                            });
                    }
                    agree_now();
                }
            }
            std::vector<XPlan> xp(NL), xb(NL);
            for (size_t li = 0; li < NL; li++) {
                xp[li] = make_plan(M.data(), W, K1, sh[li].id);
                xb[li] = reverse_plan(xp[li]);
            }
            // (2) successors to their owners: owner-grouped items, cursors preset to the groups
            Payload items{&xp, std::vector<const void *>(NL), std::vector<void *>(NL), sizeof(XItem)};
            for (size_t li = 0; li < NL; li++) {
                Shard &s = sh[li];
                if (s.G) {
                    // (pinned words 96..127 of hsum: nothing else uses them, and a later sync of the
                    // round orders this copy before the next round writes them)
                    uint32_t *hc = reinterpret_cast<uint32_t *>(s.hsum + 96);
                    for (int d = 0; d < W; d++) hc[d] = (uint32_t)xp[li].send_off[d];
                    HIPCHK(hipMemcpyAsync(s.ocnt, hc, W * 4, hipMemcpyHostToDevice, stream));
                    timed(PH_XCHG, [&] {
                        launch_route_place(s.fp, round_sep(s) ? s.hcnt : s.cnt, s.np, (uint32_t)MS, (uint32_t)W, s.ocnt, s.gblk, s.xs, s.perm,
                                           (uint32_t)s.id, stream);
                    });
                }
                items.send[li] = s.xs;
                items.recv[li] = s.xr;
            }
            timed(PH_XCHG, [&] { exchange({items}); });
            // (3) owners: seen-set probe, smallest key per new fingerprint, verdicts, seen-set insert
            Payload verdicts{&xb, std::vector<const void *>(NL), std::vector<void *>(NL), 4};
            for (size_t li = 0; li < NL; li++) {
                Shard &o = sh[li];
                const uint64_t R = xp[li].recv_total, Rl = o.Gself;  // received / its own
                verdicts.send[li] = o.rflag;
                verdicts.recv[li] = o.sflag;
                if (!R && !Rl) continue;
                guard(li, [&] {
                    inject(3, o.id, c, L);
                    grow_seen(o, o.T_count + R + Rl);
                    // the own successors' bids are in E already (k_hash_probe) if the received
                    // ones fit beside them at load <= 1/2; otherwise every bid goes to the owner table
                    const bool lx = o.lx_bid && 2 * (R + Rl) <= o.lcap && owner_lxy != 2;
                    ESlot *OT = o.E;
                    uint64_t mask = o.lcap - 1;
                    uint32_t rnd = o.lx_round;
                    if (!lx) {
                        mask = owner_table(o, R + Rl) - 1;
                        OT = o.OT;
                        rnd = o.ot_round;
                    }
                    // every bid counts the owner's own winners on their parents (owner_bid); a split round's commit
                    // then decides the own candidates itself (no k_local_flags pass)
                    timed(PH_DEDUP, [&] {
                        const KParams Q = round_params(o, gbase);
                        if (Rl && !lx) {
                            // (bids the fingerprint pass made in E are void: they count again in the owner table)
                            if (o.lx_bid) HIPCHK(hipMemsetAsync(o.wacc, 0, o.np * 4, stream));
                            ks.local_elect(Q, o.np, o.seen(), OT, mask, rnd, (uint32_t)W, (uint32_t)o.id, o.gblk,
                                           stream);
                        }
                        if (R) {
                            launch_owner_elect(o.xr, R, o.seen(), OT, mask, rnd, o.rslot, o.wacc, o.gblk, o.np, stream);
                            launch_owner_flags(o.xr, R, o.rslot, OT, rnd, o.seen(), o.rflag, o.sum + SUM_INS, stream);
                        }
                        if (Rl && !round_sep(o))
                            ks.local_flags(Q, o.np, o.seen(), OT, rnd, (uint32_t)W, (uint32_t)o.id, o.gblk,
                                           o.sum + SUM_INS, stream);
                    });
                    o.rt_table = OT;
                    o.rt_round = rnd;
                });
                // a failed owner answers "no winner" everywhere (the round is abandoned at the next agreement)
                if (fail[li]) HIPCHK(hipMemsetAsync(o.rflag, 0, R * 4, stream));
            }
            timed(PH_XCHG, [&] { exchange({verdicts}); });
            // (4) sources: verdicts on the slots, winners per parent and their words
            for (size_t li = 0; li < NL; li++) {
                Shard &s = sh[li];
                if (!s.np || fail[li]) continue;
                timed(PH_DEDUP, [&] {
                    launch_scatter_win(s.perm, s.sflag, s.G, s.score, (uint32_t)sw4(), s.pnm, (uint32_t)MS, s.lslot,
                                       s.wacc, stream);
                    const KParams Q = round_params(s, gbase);
                    ks.wincount(Q, s.np, stream);
                    if (Q.plist) launch_nzlist(Q, s.np, stream);
                });
            }
            std::vector<uint64_t> tab((size_t)TAB * W, 0);
            std::vector<uint64_t> ins(NL, 0), wnum(NL, 0), wwords(NL, 0);
            for (size_t li = 0; li < NL; li++) {
                Shard &s = sh[li];
                HIPCHK(hipMemcpyAsync(s.hsum, s.sum, (SUM_SELF + 1) * 8, hipMemcpyDeviceToHost, stream));
                HIPCHK(hipStreamSynchronize(stream));
                ins[li] = s.hsum[9];
                if (s.np && !fail[li]) {
                    tab[TAB * s.id + 0] = s.hsum[0];
                    wnum[li] = s.hsum[1];
                    wwords[li] = s.hsum[SUM_WORDS];
                    // self-loops: a split round's set apart (k_wincount), a fused round's counted by the expansion
                    tab[TAB * s.id + 7] = s.hsum[SUM_SELF];
                }
            }
            collect_times(st);
            // (5) commit: every shard's winners, in TLC order, into its outbox (+ invariants)
            for (size_t li = 0; li < NL; li++) {
                Shard &s = sh[li];
                if (!s.np) continue;
                guard(li, [&] {
                    inject(4, s.id, c, L);
                    grow_outbox(s, wwords[li], wnum[li]);
                    if (wwords[li] >= s.rcap) ensure_ring(s, wwords[li], 0);  // P.rcap also bounds the outbox
                    timed(PH_MAT, [&] {
                        KParams Q = round_params(s, gbase);
                        if (Q.plist) {  // a lane per successor slot; the own candidates decided in the round's table
                            Q.OT = s.rt_table;
                            Q.ot_round = s.rt_round;
                            ks.commit_split(Q, s.np, stream);
                        } else {
                            ks.commit(Q, stream);
                        }
                    });
                });
            }
            for (size_t li = 0; li < NL; li++) {
                Shard &s = sh[li];
                s.T_count += ins[li];
                if (!s.np || fail[li]) continue;
                HIPCHK(hipMemcpyAsync(s.hsum, s.sum, (SUM_INS_COMMIT + 1) * 8, hipMemcpyDeviceToHost, stream));
                HIPCHK(hipStreamSynchronize(stream));
                HIPCHK(hipGetLastError());
                ins[li] += s.hsum[SUM_INS_COMMIT];  // (a split round's own winners, inserted by its commit)
                s.T_count += s.hsum[SUM_INS_COMMIT];
                if (s.hsum[2 + ERR_NSLOTS] && !fail[li]) {
                    fail[li] = flag_code(s.hsum[2 + ERR_NSLOTS]);
                    fail_msg = flag_msg(s.hsum[2 + ERR_NSLOTS]);
                }
                uint64_t *row = &tab[TAB * s.id];
                row[1] = wnum[li];
                row[2] = wwords[li];
                row[3] = ins[li];
                unsigned long long best;
                const int kind = first_error(s.hsum + 2, &best);
                if (kind >= 0) {
                    const uint64_t g = s.gblk + ((best >> 24) - s.p0);
                    row[4] = (uint64_t)kind + 1;
                    row[5] = (((g << 16) | ((best >> 8) & 0xFFFF)) << 8) | (best & 0xFF);
                }
            }
            collect_times(st);
            for (size_t li = 0; li < NL; li++) tab[TAB * sh[li].id + 6] = (uint64_t)(-fail[li]);
            allreduce(tab.data(), TAB * W, false);  // rows: each shard's own, zero elsewhere
            {
                uint64_t worst = 0;
                for (int t = 0; t < W; t++) worst = std::max(worst, tab[TAB * t + 6]);
                agree(worst);
            }
            // (6) the first error of the round in the level's order
            int ek_shard = -1;
            for (int t = 0; t < W; t++)
                if (tab[TAB * t + 4] && (ek_shard < 0 || (tab[TAB * t + 5] >> 8) < (tab[TAB * ek_shard + 5] >> 8)))
                    ek_shard = t;
            if (ek_shard >= 0) {
                sharded_stop(ek_shard, (int)tab[TAB * ek_shard + 4] - 1, tab[TAB * ek_shard + 5], L, tab, level_gen,
                             level_new, Fg, gbase, st);
                st->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                seconds += st->seconds;
                return status;
            }
            // (7) winners to the shards owning their global next-level indices (rmc_plan.h route_pieces)
            std::vector<uint64_t> A(W + 1, level_new);
            for (int t = 0; t < W; t++) A[t + 1] = A[t] + tab[TAB * t + 1];
            std::vector<std::vector<Piece>> pcs(NL);
            std::vector<PieceLayout> lay(NL);
            std::vector<std::vector<uint64_t>> pw0(NL), pw1(NL);  // word range of each piece
            {
                // every piece boundary of every local shard in one copy back (pinned scratch)
                size_t nb = 0;
                for (size_t li = 0; li < NL; li++) {
                    const Shard &s = sh[li];
                    pcs[li] = route_pieces(A[s.id], A[s.id + 1] - A[s.id], B, W);
                    nb += pcs[li].size();
                }
                if (nb > (size_t)RED_CAP) throw Fail(RMC_E_ARG, "too many winner pieces in a round");
                size_t k = 0;
                for (size_t li = 0; li < NL; li++)
                    for (const Piece &pe : pcs[li])
                        HIPCHK(hipMemcpyAsync(h_red + k++, sh[li].ooff + pe.i0, 8, hipMemcpyDeviceToHost, stream));
                // ... and, for a ring at its budget, where the current level's unexpanded records
                // start (what the append below may reuse)
                const size_t kc = k;
                for (size_t li = 0; li < NL; li++) {
                    const Shard &o = sh[li];
                    const uint64_t done = std::min(o.cur_n, (c + 1) * B);
                    if (o.ring_fixed && done < o.cur_n) {
                        if (kc + NL > (size_t)RED_CAP) throw Fail(RMC_E_ARG, "too many winner pieces in a round");
                        HIPCHK(hipMemcpyAsync(h_red + kc + li, o.cur_off + done, 8, hipMemcpyDeviceToHost, stream));
                        nb++;
                    }
                }
                if (nb) HIPCHK(hipStreamSynchronize(stream));
                for (size_t li = 0; li < NL; li++) {
                    const Shard &o = sh[li];
                    const uint64_t done = std::min(o.cur_n, (c + 1) * B);
                    consumed_[li] = !o.ring_fixed ? 0 : done < o.cur_n ? h_red[kc + li] : o.cur_words;
                }
                k = 0;
                for (size_t li = 0; li < NL; li++) {
                    const uint64_t w = A[sh[li].id + 1] - A[sh[li].id];
                    pw0[li].resize(pcs[li].size());
                    pw1[li].resize(pcs[li].size());
                    for (size_t q = 0; q < pcs[li].size(); q++) pw0[li][q] = h_red[k++];
                    for (size_t q = 0; q < pcs[li].size(); q++)
                        pw1[li][q] = pcs[li][q].i1 < w ? pw0[li][q + 1] : wwords[li];
                }
            }
            const int K2 = 2 * W + 3;
            std::vector<std::vector<uint64_t>> rows2(NL, std::vector<uint64_t>(K2, 0));
            std::vector<std::vector<uint64_t>> wlay(NL, std::vector<uint64_t>(W, 0));  // word offsets per destination
            for (size_t li = 0; li < NL; li++) {
                Shard &s = sh[li];
                const uint64_t w = A[s.id + 1] - A[s.id];
                lay[li] = piece_layout(pcs[li], W);
                std::vector<uint64_t> pwc(W, 0);
                for (size_t q = 0; q < pcs[li].size(); q++) pwc[pcs[li][q].d] += pw1[li][q] - pw0[li][q];
                if (w && !lay[li].regroup) {
                    for (size_t q = 0; q < pcs[li].size(); q++) wlay[li][pcs[li][q].d] = pw0[li][q];
                } else if (w) {
                    // a destination owns several of the pieces: group them (in order) by destination
                    uint64_t wat = 0;
                    for (int d = 0; d < W; d++) { wlay[li][d] = wat; wat += pwc[d]; }
                    guard(li, [&] {
                        inject(5, s.id, c, L);
                        grow_inbox(s, wwords[li], w);  // the inbox holds the grouped copy until the exchange
                        uint64_t at = 0;
                        wat = 0;
                        for (int d = 0; d < W; d++)
                            for (size_t q = 0; q < pcs[li].size(); q++) {
                                const Piece &pe = pcs[li][q];
                                if (pe.d != d) continue;
                                HIPCHK(hipMemcpyAsync(s.iside + at, s.oside + pe.i0, (pe.i1 - pe.i0) * 16,
                                                      hipMemcpyDeviceToDevice, stream));
                                HIPCHK(hipMemcpyAsync(s.ib + wat, s.ob + pw0[li][q], (pw1[li][q] - pw0[li][q]) * 4,
                                                      hipMemcpyDeviceToDevice, stream));
                                at += pe.i1 - pe.i0;
                                wat += pw1[li][q] - pw0[li][q];
                            }
                        // the grouped copy goes out of the outbox buffers (the inbox is refilled below)
                        HIPCHK(hipMemcpyAsync(s.oside, s.iside, w * 16, hipMemcpyDeviceToDevice, stream));
                        HIPCHK(hipMemcpyAsync(s.ob, s.ib, wwords[li] * 4, hipMemcpyDeviceToDevice, stream));
                        HIPCHK(hipStreamSynchronize(stream));
                    });
                }
                for (int d = 0; d < W; d++) {
                    rows2[li][d] = lay[li].cnt[d];
                    rows2[li][W + d] = pwc[d];
                }
                const bool force = injecting(6, s.id, c, L);  // site 6 forces this shard's inbox to grow
                rows2[li][2 * W] = force ? 0 : s.is_cap;
                rows2[li][2 * W + 1] = force ? 0 : s.ib_cap;
                rows2[li][2 * W + 2] = (uint64_t)(-fail[li]);
            }
            std::vector<uint64_t> M2 = gather_rows(rows2, K2);
            agree(col_max(M2, K2, 2 * W + 2));
            {
                std::vector<uint64_t> need_n(W, 0), need_w(W, 0), cap_n(W, 0), cap_w(W, 0);
                for (int o = 0; o < W; o++) {
                    for (int t = 0; t < W; t++) {
                        need_n[o] += M2[(size_t)t * K2 + o];
                        need_w[o] += M2[(size_t)t * K2 + W + o];
                    }
                    cap_n[o] = M2[(size_t)o * K2 + 2 * W];
                    cap_w[o] = M2[(size_t)o * K2 + 2 * W + 1];
                }
                if (!must_grow(need_n, cap_n).empty() || !must_grow(need_w, cap_w).empty()) {
                    for (size_t li = 0; li < NL; li++) {
                        const int id = sh[li].id;
                        if (need_n[id] + 1 > cap_n[id] || need_w[id] + 1 > cap_w[id])
                            guard(li, [&] {
                                inject(6, id, c, L);
                                grow_inbox(sh[li], need_w[id], need_n[id]);
                            });
                    }
                    agree_now();
                }
            }
            std::vector<XPlan> xs_(NL), xw_(NL);
            Payload sides{&xs_, std::vector<const void *>(NL), std::vector<void *>(NL), 16};
            Payload words_{&xw_, std::vector<const void *>(NL), std::vector<void *>(NL), 4, !self_rccl};
            for (size_t li = 0; li < NL; li++) {
                Shard &s = sh[li];
                xs_[li] = make_plan(M2.data(), W, K2, s.id);
                xw_[li] = make_plan(M2.data() + W, W, K2, s.id);
                for (int d = 0; d < W; d++) {  // the send layout: pieces in place, or regrouped
                    xs_[li].send_off[d] = lay[li].off[d];
                    xw_[li].send_off[d] = wlay[li][d];
                }
                sides.send[li] = s.oside;
                words_.send[li] = s.ob;
                sides.recv[li] = s.iside;
                words_.recv[li] = s.ib;
            }
            timed(PH_XCHG, [&] { exchange({sides, words_}); });
            // (8) owners append what they received, in source order, to the next level
            for (size_t li = 0; li < NL; li++) {
                Shard &o = sh[li];
                const uint64_t n = xs_[li].recv_total, words = xw_[li].recv_total;
                if (!n) continue;
                const uint64_t consumed = consumed_[li];
                guard(li, [&] {
                    inject(7, o.id, c, L);
                    ensure_ring(o, words, consumed);
                    ensure_off(o.nxt_off, o.nxt_off_cap, o.nxt_n, o.nxt_n + n);
                    grow_trace(o, n);
                    ensure_tmp(o, n + 1);
                });
                if (fail[li]) continue;
                const uint64_t gid = o.level_start[L - 1] + o.cur_n + o.nxt_n;  // local gid of the first
                trace_restart(o);
                trace_fence(o);
                timed(PH_OTHER, [&] {
                    const uint64_t at = ring_wrap(o.nbase() + o.nxt_words, o.rcap);
                    const uint64_t a = xw_[li].recv_off[o.id], sw = xw_[li].recv_cnt[o.id];
                    if (words_.self_in_place && sw) {  // this shard's own winners come from its outbox
                        ring_copy_in(o, at, o.ib, a);
                        ring_copy_in(o, ring_wrap(at + a, o.rcap), o.ob + xw_[li].send_off[o.id], sw);
                        ring_copy_in(o, ring_wrap(at + a + sw, o.rcap), o.ib + a + sw, words - a - sw);
                    } else {
                        ring_copy_in(o, at, o.ib, words);
                    }
                    launch_side_sizes(o.iside, n, o.isz, stream);
                    HIPCHK(hipMemsetAsync(o.isz + n, 0, 4, stream));
                    HIPCHK(hipcub::DeviceScan::ExclusiveSum(o.tmp, o.tmp_bytes, o.isz, o.ioff, (int)n + 1, stream));
                    launch_accept_side(o.iside, o.ioff, n, o.nxt_words, o.nxt_off + o.nxt_n, o.par + (gid - o.tdev),
                                       o.pslot + (gid - o.tdev), stream);
                });
                flush_trace(o, gid + n);
                o.nxt_n += n;
                o.nxt_words += words;
                // the live frontier after the append: the current level's words not yet reused (a ring at its
                // budget reuses the expanded rounds' words, consumed_) plus the next level's so far
                o.peak_words = std::max(o.peak_words, o.cur_words - consumed_[li] + o.nxt_words);
            }
            // an append failure rides on the next round's gathered matrix; after the level's last
            // round it is agreed here
            if (c + 1 == rounds) agree_now();
            for (int t = 0; t < W; t++) {
                level_gen += tab[TAB * t + 0];
                level_new += tab[TAB * t + 1];
                level_words += tab[TAB * t + 2];
                level_self += tab[TAB * t + 7];
            }
            // (no wait here: the next round's first read-back orders everything before it, and its
            // phase times are collected after that)
        }
        HIPCHK(hipStreamSynchronize(stream));
        collect_times(st);
        total_generated += level_gen;
        total_distinct += level_new;
        st->generated = level_gen;
        st->new_states = level_new;
        st->new_bytes = level_words * 4;
        st->self_loops = level_self;
        for (Shard &s : sh) {
            const uint64_t gid_nxt = s.level_start[L - 1] + s.cur_n;
            s.peak_words = std::max(s.peak_words, s.nxt_words);  // (the level's rounds counted the rest)
            end_level(s, gid_nxt, L);
            if (!s.cur_n) s.level_start.push_back(gid_nxt);  // every shard keeps the same level count
        }
        glevel.push_back(gbase + Fg);
        HIPCHK(hipStreamSynchronize(stream));
        if (level_new) {
            depth = L + 1;
        } else {
            finished = true;
            status = RMC_DONE;
            queue_at_end = 0;
        }
        st->total_generated = total_generated;
        st->total_distinct = total_distinct;
        st->queue = level_new;
        st->status = finished ? RMC_DONE : RMC_OK;
        st->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        seconds += st->seconds;
        return st->status;
    }

    // Sharded stop at the round's first error (shard e, kind, global key gk = (g << 16 | slot) << 8
    // | which): TLC's counters -- every earlier round, the round's shards before e (their blocks
    // come first in the level), and e's own share up to the error (error_counts).
    void sharded_stop(int e, int kind, uint64_t gk, int L, const std::vector<uint64_t> &tab, uint64_t level_gen,
                      uint64_t level_new, uint64_t Fg, uint64_t gbase, rmc_level_stats *st) {
        const uint64_t g = gk >> 24;
        const uint32_t slot = (uint32_t)((gk >> 8) & 0xFFFF);
        uint64_t loc[2] = {0, 0};
        for (Shard &s : sh)
            if (s.id == e) {
                const uint64_t p = s.p0 + (g - s.gblk);
                const unsigned long long ek = (((p << 16) | slot) << 8) | (gk & 0xFF);
                s.chunk_sep = round_sep(s);  // (a split round stages its successors but its self-loops)
            s.chunk_dense = false;       // (sparse: the owners' verdicts come back by slot index)
                const ErrCounts ec = error_counts(s, kind, ek, s.p0, true);
                loc[0] = ec.gen;
                loc[1] = ec.win;
            }
        allreduce(loc, 2, false);
        uint64_t gen = level_gen + loc[0], winb = level_new + loc[1];
        for (int t = 0; t < e; t++) {
            gen += tab[TAB * t + 0];
            winb += tab[TAB * t + 1];
        }
        err_ref = gbase + g;
        queue_at_end = (Fg - g - 1) + winb;
        if (kind == ERR_INV || kind == ERR_EVAL) {
            status = kind == ERR_INV ? RMC_VIOLATION : RMC_EVAL_ERROR;
            violated = (int)(gk & 0xFF);
            err_last_slot = slot;
            total_distinct += winb + 1;
            depth = L + 1;
        } else {
            status = kind == ERR_ASSERT ? RMC_ASSERT : RMC_DEADLOCK;
            err_last_slot = KEY_NONE;
            total_distinct += winb;
            if (winb) depth = L + 1;
        }
        total_generated += gen;
        st->generated = gen;
        st->new_states = winb + ((kind == ERR_INV || kind == ERR_EVAL) ? 1 : 0);
        st->total_generated = total_generated;
        st->total_distinct = total_distinct;
        st->queue = queue_at_end;
        st->status = status;
        finished = true;
        build_trace();
    }

    // parent's global id and slot of the state with global id G, from whichever shard holds it
    void fetch_par(uint64_t G, uint64_t *par, uint16_t *slot) {
        uint64_t v[2] = {0, 0};
        auto take = [&](const Shard &s, uint64_t gid) {
            if (gid >= s.tflushed) throw Fail(RMC_E_STATE, "trace entry not on the host");
            v[0] = s.hpar.get(gid) + 1;  // +1: the Init sentinel ~0 travels as 0
            v[1] = s.hslot.get(gid);
        };
        if (L_shard == 0 || G < glevel[L_shard - 1]) {
            if (virt || rank == 0) take(sh[0], G);  // replicated levels: global id == local gid
        } else {
            const size_t k = (size_t)(std::upper_bound(glevel.begin(), glevel.end(), G) - glevel.begin()) - 1;
            const uint64_t g = G - glevel[k], B = chunk_parents;
            const int owner = (int)((g / B) % (uint64_t)W);
            for (const Shard &s : sh)
                if (s.id == owner) take(s, s.level_start[k] + (g / (B * W)) * B + g % B);
        }
        allreduce(v, 2, false);
        *par = v[0] - 1;
        *slot = (uint16_t)v[1];
    }

    // Walk parent pointers from err_ref to Init, then replay the slots from Init.
    // The slot keys from Init down to the state with global id g (and, with gids, the global ids of
    // the states on the path, Init's 0 first).
    std::vector<uint16_t> path_slots(uint64_t g, std::vector<uint64_t> *gids) {
        // (a run that ended without an error left its last device-loop levels' entries on the device)
        for (Shard &s : sh) flush_trace(s, s.trace_end);
        sync_trace();
        HIPCHK(hipStreamSynchronize(stream));  // pending trace copies
        std::vector<uint16_t> slots;
        if (gids) gids->assign(1, g);
        for (;;) {
            uint64_t par;
            uint16_t sl;
            fetch_par(g, &par, &sl);
            if (par == ~0ull) break;
            slots.push_back(sl);
            g = par;
            if (gids) gids->push_back(g);
            if (slots.size() > 100000) throw Fail(RMC_E_STATE, "corrupt parent chain");
        }
        std::reverse(slots.begin(), slots.end());
        if (gids) std::reverse(gids->begin(), gids->end());
        return slots;
    }

    void build_trace() {
        std::vector<uint16_t> slots = path_slots(err_ref, nullptr);
        if (err_last_slot != KEY_NONE) slots.push_back((uint16_t)err_last_slot);
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
    // One file per process: the run's header (configuration, fingerprint scheme, TLC's counters,
    // and for the sharded protocol W, this process's first shard, the chunk size B that the
    // block-cyclic layout depends on, replicated / sharded mode and the global level table),
    // then one section per shard this process holds: its seen-set shard, its part of the current
    // level (records linearised + offsets) and the parent reference of every state it holds.
    // An RCCL rank of a W > 1 run writes path + ".rank<r>"; every rank resumes from its own file.
    struct CkptHeader {
        uint64_t magic;
        uint32_t abi, recw;
        int32_t n, v, e, r;
        uint32_t invariants, inv_order;
        int32_t check_deadlock, spec_variant, no_symmetry, msg_cap, depth, pad0;
        uint64_t scheme;
        uint64_t total_generated, total_distinct;
        int32_t W, first_shard, nshards, replicated, L_shard, pad1;
        uint64_t chunk_parents, shard_min, n_glevel;
        double seconds;
        uint64_t check;  // checksum of every field above
    };
    struct CkptShard {
        int32_t id, compact;
        uint32_t epoch, pad;
        uint64_t T_cap, T_count, cur_n, cur_words, n_levels, trace_n;
    };
    static constexpr uint64_t CKPT_MAGIC = 0x3450434b434d52ull;  // "RMCKCP4": data checksums

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
        h.W = multi ? W : 0;
        h.first_shard = multi ? sh[0].id : 0;
        h.nshards = (int32_t)sh.size();
        h.chunk_parents = multi ? chunk_parents : 0;
        h.shard_min = multi ? shard_min : 0;
        return h;
    }
    template <class T>
    static uint64_t fnv(const T &h, size_t bytes) {
        const unsigned char *b = reinterpret_cast<const unsigned char *>(&h);
        uint64_t x = 0xcbf29ce484222325ull;
        for (size_t i = 0; i < bytes; i++) x = (x ^ b[i]) * 0x100000001b3ull;
        return x;
    }
    static uint64_t header_check(const CkptHeader &h) { return fnv(h, offsetof(CkptHeader, check)); }
    // checksum of a shard's data sections (seen set, ring words, offsets, trace), 8 bytes at a time:
    // fast enough for a 150 GB checkpoint, and a corrupt or mismatched section fails resume
    struct DataSum {
        uint64_t h = 0x6a09e667f3bcc909ull;
        void add(const void *p, size_t k) {
            const unsigned char *b = static_cast<const unsigned char *>(p);
            size_t i = 0;
            for (; i + 8 <= k; i += 8) {
                uint64_t w;
                std::memcpy(&w, b + i, 8);
                h = (h ^ w) * 0x9e3779b97f4a7c15ull;
                h ^= h >> 29;
            }
            for (; i < k; i++) h = (h ^ b[i]) * 0x100000001b3ull;
        }
    };
    std::string ckpt_path(const char *path) const {
        return ((rccl || hostx) && W > 1) ? std::string(path) + ".rank" + std::to_string(rank) : std::string(path);
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
    void checkpoint(const char *path_arg) {
        if (!inited || finished) throw Fail(RMC_E_STATE, "checkpoint: between levels of a started, unfinished run");
        HIPCHK(hipStreamSynchronize(stream));
        sync_trace();
        const std::string path = ckpt_path(path_arg);
        CkptHeader h = ckpt_header();
        h.depth = depth;
        h.total_generated = total_generated; h.total_distinct = total_distinct;
        h.replicated = replicated ? 1 : 0;
        h.L_shard = L_shard;
        h.n_glevel = (multi && !replicated) ? glevel.size() : 0;
        h.seconds = seconds;
        h.check = header_check(h);
        std::vector<CkptShard> sc(sh.size());
        for (size_t i = 0; i < sh.size(); i++) {
            const Shard &t = sh[i];
            CkptShard &c = sc[i];
            c.id = t.id;
            c.compact = t.Tc ? 1 : 0;
            c.epoch = t.epoch;
            c.T_cap = t.T_cap; c.T_count = t.T_count; c.cur_n = t.cur_n; c.cur_words = t.cur_words;
            c.n_levels = t.level_start.size();
            c.trace_n = t.level_start.back() + t.cur_n;  // every state the shard holds has a local gid below
            if (t.tflushed != c.trace_n) throw Fail(RMC_E_STATE, "checkpoint: trace not flushed");
        }
        const std::string tmp = path + ".tmp";
        FILE *f = std::fopen(tmp.c_str(), "wb");
        if (!f) throw Fail(RMC_E_ARG, std::string("checkpoint: cannot write ") + tmp);
        bool ok = std::fwrite(&h, sizeof h, 1, f) == 1 &&
                  std::fwrite(glevel.data(), 8, h.n_glevel, f) == h.n_glevel;
        DataSum sum;
        auto out = [&](void *dev, char *host, size_t k) {
            HIPCHK(hipMemcpy(host, dev, k, hipMemcpyDeviceToHost));
            sum.add(host, k);
            ok = ok && std::fwrite(host, 1, k, f) == k;
        };
        for (size_t i = 0; ok && i < sh.size(); i++) {
            Shard &t = sh[i];
            const CkptShard &c = sc[i];
            const uint64_t chk = fnv(c, sizeof c);
            sum = DataSum{};
            ok = std::fwrite(&c, sizeof c, 1, f) == 1 && std::fwrite(&chk, 8, 1, f) == 1 &&
                 std::fwrite(t.level_start.data(), 8, c.n_levels, f) == c.n_levels;
            if (t.Tc) stream_bytes(t.Tc, c.T_cap * 8, out);
            else stream_bytes(t.T, c.T_cap * 16, out);
            // the shard's part of the current level, linearised
            uint32_t *lin = dmalloc<uint32_t>(std::max<uint64_t>(c.cur_words, 1));
            ring_copy_out(t, t.cur_wbase, c.cur_words, lin);
            HIPCHK(hipStreamSynchronize(stream));
            stream_bytes(lin, c.cur_words * 4, out);
            dfree(lin);
            stream_bytes(t.cur_off, c.cur_n * 8, out);
            t.hpar.for_range(0, c.trace_n, [&](const uint64_t *p, uint64_t k) {
                sum.add(p, k * 8);
                ok = ok && std::fwrite(p, 8, k, f) == k;
            });
            t.hslot.for_range(0, c.trace_n, [&](const uint16_t *p, uint64_t k) {
                sum.add(p, k * 2);
                ok = ok && std::fwrite(p, 2, k, f) == k;
            });
            ok = ok && std::fwrite(&sum.h, 8, 1, f) == 1;
        }
        ok = std::fflush(f) == 0 && ok;
        ok = ok && fsync(fileno(f)) == 0;
        ok = (std::fclose(f) == 0) && ok;
        if (!ok) {
            std::remove(tmp.c_str());
            throw Fail(RMC_E_ARG, std::string("checkpoint: short write to ") + tmp);
        }
        if (std::rename(tmp.c_str(), path.c_str()) != 0)
            throw Fail(RMC_E_ARG, std::string("checkpoint: cannot rename to ") + path);
    }

    // A resume that fails part way (a corrupt data section, a short file, an allocation) may have loaded
    // part of the checkpoint into the seen set and rings: the context is reset, so it starts from Init
    // (or takes another resume) as if the failed call had not been made.
    void resume(const char *path_arg) {
        if (inited) throw Fail(RMC_E_STATE, "resume: needs a context not yet initialised (rmc_create or rmc_reset)");
        try {
            resume_body(path_arg);
        } catch (...) {
            reset();
            throw;
        }
    }

    void resume_body(const char *path_arg) {
        HIPCHK(hipStreamSynchronize(stream));  // rmc_reset's clears are stream-ordered, the loads below are not
        const std::string path = ckpt_path(path_arg);
        FILE *f = std::fopen(path.c_str(), "rb");
        if (!f) throw Fail(RMC_E_ARG, std::string("resume: cannot read ") + path);
        auto fail = [&](const char *what) {
            std::fclose(f);
            throw Fail(RMC_E_ARG, std::string("resume: ") + path + what);
        };
        CkptHeader h{};
        const CkptHeader want = ckpt_header();
        bool ok = std::fread(&h, sizeof h, 1, f) == 1;
        if (!ok || h.magic != CKPT_MAGIC || h.abi != want.abi || h.recw != want.recw || h.n != want.n ||
            h.v != want.v || h.e != want.e || h.r != want.r || h.invariants != want.invariants ||
            h.inv_order != want.inv_order || h.check_deadlock != want.check_deadlock ||
            h.spec_variant != want.spec_variant || h.no_symmetry != want.no_symmetry || h.msg_cap != want.msg_cap)
            fail(" is not a checkpoint of this configuration");
        if (h.scheme != want.scheme) fail(" was written with another fingerprint scheme");
        // A sharded checkpoint written with a SMALLER chunk size than this context's is adopted (the chunk
        // buffers hold it; the block-cyclic layout needs the writer's size): the chunk follows free memory at
        // create when budgets are explicit, so a context created with more headroom than the writer had
        // resumes.  A larger stored chunk would need larger buffers than this context sized: refused below.
        // The adoption is undone if the resume fails (cp_guard).
        struct CpGuard {
            uint64_t &cp;
            const uint64_t before;
            bool keep;
            ~CpGuard() { if (!keep) cp = before; }
        } cp_guard{chunk_parents, chunk_parents, false};
        if (multi && h.chunk_parents && h.chunk_parents < want.chunk_parents)
            want_chunk_parents_adopt = h.chunk_parents;
        else
            want_chunk_parents_adopt = 0;
        if (h.W != want.W || h.first_shard != want.first_shard || h.nshards != want.nshards ||
            (h.chunk_parents != want.chunk_parents && !want_chunk_parents_adopt) || h.shard_min != want.shard_min)
            fail(" was written with another shard layout (world size, rank, virtual shards, chunk size or shard_min)");
        // the header's own consistency, before anything is allocated from it
        if (h.check != header_check(h) || h.n_glevel > 100000 || (h.replicated && h.n_glevel) ||
            (multi && !h.replicated && (h.n_glevel == 0 || h.L_shard <= 0)))
            fail(" has an inconsistent header");
        if (want_chunk_parents_adopt) chunk_parents = want_chunk_parents_adopt;  // (<= the buffers' size)
        std::vector<uint64_t> gl(h.n_glevel);
        ok = std::fread(gl.data(), 8, gl.size(), f) == gl.size();
        for (size_t i = 1; ok && i < gl.size(); i++) ok = gl[i] > gl[i - 1];
        if (!ok) fail(" has an inconsistent global level table");
        std::vector<CkptShard> sc(sh.size());
        std::vector<std::vector<uint64_t>> lss(sh.size());
        DataSum sum;
        auto in = [&](void *dev, char *host, size_t k) {
            ok = ok && std::fread(host, 1, k, f) == k;
            if (ok) {
                sum.add(host, k);
                HIPCHK(hipMemcpy(dev, host, k, hipMemcpyHostToDevice));
            }
        };
        // the current level's offsets, checked before they reach the device: level-relative, from 0,
        // increasing by one record (CCW..RECW words) at a time, the last record ending at cur_words
        // -- the kernels' ring arithmetic assumes it (ring_wrap takes x < 2 cap)
        uint64_t off_prev = 0, off_i = 0, off_words = 0;
        bool off_ok = true;
        auto in_off = [&](void *dev, char *host, size_t k) {
            ok = ok && std::fread(host, 1, k, f) == k;
            if (!ok) return;
            sum.add(host, k);
            const uint64_t *o = reinterpret_cast<const uint64_t *>(host);
            for (size_t j = 0; j < k / 8; j++, off_i++) {
                const uint64_t x = o[j];
                if (off_i == 0) off_ok = off_ok && x == 0;
                else off_ok = off_ok && x >= off_prev + (uint64_t)ks.CCW && x <= off_prev + (uint64_t)RECW;
                off_ok = off_ok && x < off_words;
                off_prev = x;
            }
            if (off_ok) HIPCHK(hipMemcpy(dev, host, k, hipMemcpyHostToDevice));
        };
        for (size_t i = 0; i < sh.size(); i++) {
            Shard &s = sh[i];
            CkptShard &c = sc[i];
            uint64_t chk = 0;
            ok = std::fread(&c, sizeof c, 1, f) == 1 && std::fread(&chk, 8, 1, f) == 1;
            if (!ok || chk != fnv(c, sizeof c) || c.id != s.id || c.n_levels == 0 || c.n_levels > 100000 ||
                (!c.compact && (c.T_cap & (c.T_cap - 1)) != 0) || (c.compact && c.T_cap % 8) || c.T_cap == 0 || c.T_count >= c.T_cap ||
                c.T_count > h.total_distinct || (!multi && c.T_count > c.trace_n) || c.cur_words > c.cur_n * (uint64_t)RECW || c.cur_words < c.cur_n * (uint64_t)ks.CCW)
                fail(" has an inconsistent shard header");
            std::vector<uint64_t> &ls = lss[i];
            ls.resize(c.n_levels);
            ok = std::fread(ls.data(), 8, ls.size(), f) == ls.size();
            // (a shard may hold no state of a small sharded level: non-decreasing there)
            for (size_t j = 1; ok && j < ls.size(); j++) ok = multi ? ls[j] >= ls[j - 1] : ls[j] > ls[j - 1];
            if (!ok || ls.back() + c.cur_n != c.trace_n) fail(" has an inconsistent level table");
            dfree(s.T);
            dfree(s.Tc);
            if (c.compact) {
                s.Tc = dmalloc<unsigned long long>(c.T_cap);
                s.ring_fixed = false;  // re-derived below
            } else {
                s.T = dmalloc<ulonglong2>(c.T_cap);
            }
            s.T_cap = c.T_cap;
            s.cur_wbase = 0;
            s.cur_words = 0;
            s.nxt_words = 0;
            ensure_ring(s, c.cur_words + 1, 0);
            ensure_off(s.cur_off, s.cur_off_cap, 0, std::max<uint64_t>(c.cur_n, 1));
            sum = DataSum{};
            if (s.Tc) stream_bytes(s.Tc, c.T_cap * 8, in);
            else stream_bytes(s.T, c.T_cap * 16, in);
            stream_bytes(s.R, c.cur_words * 4, in);
            off_prev = off_i = 0;
            off_words = c.cur_words;
            off_ok = true;
            stream_bytes(s.cur_off, c.cur_n * 8, in_off);
            if (ok && (!off_ok || (c.cur_n && (c.cur_words - off_prev < (uint64_t)ks.CCW ||
                                               c.cur_words - off_prev > (uint64_t)RECW))))
                fail(" has inconsistent frontier offsets");
            s.hpar.reserve_to(c.trace_n);
            s.hslot.reserve_to(c.trace_n);
            for (uint64_t j = 0; ok && j < c.trace_n;) {
                const uint64_t k = std::min<uint64_t>(c.trace_n - j, HostArr<uint64_t>::B - j % HostArr<uint64_t>::B);
                ok = std::fread(s.hpar.blk[j / HostArr<uint64_t>::B] + j % HostArr<uint64_t>::B, 8, k, f) == k;
                j += k;
            }
            for (uint64_t j = 0; ok && j < c.trace_n;) {
                const uint64_t k = std::min<uint64_t>(c.trace_n - j, HostArr<uint16_t>::B - j % HostArr<uint16_t>::B);
                ok = std::fread(s.hslot.blk[j / HostArr<uint16_t>::B] + j % HostArr<uint16_t>::B, 2, k, f) == k;
                j += k;
            }
            s.hpar.for_range(0, c.trace_n, [&](const uint64_t *p, uint64_t k) { sum.add(p, k * 8); });
            s.hslot.for_range(0, c.trace_n, [&](const uint16_t *p, uint64_t k) { sum.add(p, k * 2); });
            uint64_t want_sum = 0;
            ok = ok && std::fread(&want_sum, 8, 1, f) == 1;
            if (!ok) fail(" is truncated");
            if (want_sum != sum.h) fail(" has a corrupt data section (checksum mismatch)");
        }
        std::fclose(f);
        for (size_t i = 0; i < sh.size(); i++) {
            Shard &s = sh[i];
            const CkptShard &c = sc[i];
            s.hpar.n = s.hslot.n = c.trace_n;
            s.tflushed = s.tdev = s.trace_end = c.trace_n;
            s.level_start = lss[i];
            s.cur_n = c.cur_n;
            s.nxt_n = 0;
            s.cur_words = c.cur_words;
            s.T_count = c.T_count;
            s.epoch = std::max(s.epoch, c.epoch);
        }
        // a compact seen set means a large run: the rings go to their budget (shared by the
        // shards of this process, as enter_sharded leaves them)
        for (Shard &s : sh)
            if (s.Tc) fix_ring(s, sh.size());
        if (multi) {
            replicated = h.replicated != 0;
            glevel = gl;
            L_shard = h.L_shard;
        }
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
        finished = sh[0].cur_n == 0 && (replicated || !multi);
        if (finished) { status = RMC_DONE; queue_at_end = 0; }
        cp_guard.keep = true;
    }

    // Forget every explored state but keep all device buffers (repeat runs, benchmarks).
    void reset() {
        HIPCHK(hipStreamSynchronize(stream));
        sync_trace();
        for (Shard &s : sh) {
            if (s.Tc) HIPCHK(hipMemsetAsync(s.Tc, 0, s.T_cap * 8, stream));
            else HIPCHK(hipMemsetAsync(s.T, 0, s.T_cap * 16, stream));
            s.T_count = 0;
            s.cur_n = s.nxt_n = 0;
            s.cur_wbase = s.cur_words = s.nxt_words = 0;
            s.tflushed = s.trace_end = 0;
            s.hpar.n = s.hslot.n = 0;
            s.level_start.clear();
            if (s.lx_round) {
                // E served as a sharded run's owner table: its owner keys (top 16 bits <= 0xFFFD) are
                // smaller than any fused election word (elect_key: 0xFFFF...), so the next run's fused
                // levels would keep them and drop states -- back to the fused table's empty state
                launch_eslot_clear(s.E, s.lcap, stream);
                s.lxy_epoch0 = s.epoch;
            }
            s.lx_round = 0;  // the fused levels of the next run use E again
        }
        // (the clears are stream-ordered before the next run's first kernel: no wait here)
        trace.clear();
        inited = finished = false;
        status = RMC_OK;
        depth = 0;
        total_generated = total_distinct = queue_at_end = 0;
        violated = -1;
        err_ref = 0;
        err_last_slot = KEY_NONE;
        seconds = 0;
        glevel.clear();
        L_shard = 0;
        replicated = false;
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
    if (c->device_released) {
        c->err = "the context's device memory was released (rmc_release_device): only rmc_destroy may follow";
        return RMC_E_STATE;
    }
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

int rmc_set_transport(const rmc_transport *t) {
    if (t && (!t->allreduce_u64 || !t->allgather_u64 || !t->alltoallv)) return RMC_E_ARG;
    g_transport_set = t != nullptr;
    g_transport = t ? *t : rmc_transport{};
    return RMC_OK;
}

int rmc_comm_unique_id(void *out128) {
    if (!out128) return RMC_E_ARG;
#ifdef RMC_WITH_RCCL
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return RMC_E_COMM;
    static_assert(sizeof(id) <= 128, "ncclUniqueId larger than 128 bytes");
    static_assert(sizeof(rmc_config) == 120, "rmc_config layout (ABI 3/4) changed: update INTEGRATION.md and raftmc");
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

int rmc_release_device(void *ctx) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    if (!c) return RMC_E_ARG;
    c->release(true);
    c->device_released = true;
    return RMC_OK;
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

int rmc_state_path(void *ctx, uint64_t gid, uint32_t *keys, uint64_t *gids, uint32_t cap, uint32_t *len) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    return guarded(c, [&] {
        if (!c->inited) throw Fail(RMC_E_STATE, "state_path: no run");
        if (gid >= c->total_distinct) throw Fail(RMC_E_ARG, "state_path: no state with that id");
        std::vector<uint64_t> g;
        const std::vector<uint16_t> sl = c->path_slots(gid, &g);
        if (len) *len = (uint32_t)g.size();
        if (g.size() > cap) throw Fail(RMC_E_ARG, "state_path: buffer too small");
        for (size_t i = 0; i < g.size(); i++) {
            if (gids) gids[i] = g[i];
            if (keys) {
                const uint32_t k = i ? sl[i - 1] : 0u;
                keys[i] = i ? (key_server(k) << 24) | (key_action(k) << 16) | key_witness(k) : 0u;
            }
        }
        return RMC_OK;
    });
}

int rmc_fingerprints(void *ctx, const int32_t *unpacked, size_t stride, uint64_t n, uint64_t *fps) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    return guarded(c, [&] {
        if (!unpacked || !fps) throw Fail(RMC_E_ARG, "fingerprints: null buffer");
        std::vector<uint32_t> rec((size_t)c->RECW * (n ? n : 1), 0u);
        for (uint64_t i = 0; i < n; i++) c->pack(unpacked + i * stride, rec.data() + i * c->RECW);
        uint32_t *d_rec = dmalloc<uint32_t>(rec.size());
        ulonglong2 *d_fp = dmalloc<ulonglong2>(n ? n : 1);
        try {
            HIPCHK(hipMemcpy(d_rec, rec.data(), rec.size() * 4, hipMemcpyHostToDevice));
            KParams P = c->base(c->sh[0]);
            P.front = d_rec;
            P.fp = d_fp;
            if (n) c->ks.fp_states(P, n, c->stream);
            HIPCHK(hipMemcpyAsync(fps, d_fp, n * 16, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
        } catch (...) {
            dfree(d_rec);
            dfree(d_fp);
            throw;
        }
        dfree(d_rec);
        dfree(d_fp);
        return RMC_OK;
    });
}

int rmc_seen_contains(void *ctx, const uint64_t *fps, uint64_t n, uint8_t *out) {
    rmc_ctx *c = (rmc_ctx *)ctx;
    return guarded(c, [&] {
        if (!fps || !out) throw Fail(RMC_E_ARG, "seen_contains: null buffer");
        if (c->rccl || c->hostx) throw Fail(RMC_E_STATE, "seen_contains: the seen set is spread over the ranks");
        HIPCHK(hipStreamSynchronize(c->stream));
        ulonglong2 *d_fp = dmalloc<ulonglong2>(n ? n : 1);
        uint8_t *d_out = dmalloc<uint8_t>(n ? n : 1);
        try {
            HIPCHK(hipMemcpy(d_fp, fps, n * 16, hipMemcpyHostToDevice));
            std::vector<Seen> seens;
            for (const Shard &sh : c->sh) seens.push_back(sh.seen());
            // a fingerprint lives in its owner's shard (fp_owner); one shard: every fingerprint
            for (size_t i = 0; i < seens.size(); i++)
                launch_seen_query(d_fp, n, seens[i], (uint32_t)c->sh.size(), (uint32_t)c->sh[i].id, d_out, c->stream);
            HIPCHK(hipMemcpyAsync(out, d_out, n, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
        } catch (...) {
            dfree(d_fp);
            dfree(d_out);
            throw;
        }
        dfree(d_fp);
        dfree(d_out);
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
