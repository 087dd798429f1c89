/*
 * TEST INFRASTRUCTURE ONLY -- memory-lean prefix generator for the deep golden levels.
 *
 * The same restatement of Raft.tla as oracle/raft_oracle.c (included: its successor generator
 * gen_action, exact canonical form canon_hash, invariants) and the same level-synchronous
 * first-wins BFS as oracle/raft_mt.c (TLC -workers 1 semantics), laid out so that
 * Raft.cfg's levels 31-34 (up to ~10^9 states) fit in the build container's 62 GB:
 *
 *   - frontier states are packed records (nibble-coded core + 16-bit message ids into the sorted
 *     message universe): ~28 B + 2 B per message instead of raft_oracle.c's 160 B + 4 B per message;
 *   - the seen set is a single table of 16-B slots {exact-canonical-form hash} sized once
 *     (non-power-of-two capacity, multiply-shift home, linear probing);
 *   - successors are not stored as candidates: the expansion elects (hash -> smallest key) in a
 *     per-level table, the winners are sorted by key (parent index << 16 | rank in TLC order), and
 *     the commit re-generates each winning parent's successors (no hashing) to pack them, in TLC
 *     FIFO order, into the next level.
 *
 * Every level it reports is complete.  Only tests/golden/make_golden_prefix.py runs it (--lean);
 * the product library never links or calls it.
 */
#include "raft_oracle.c"

#include <pthread.h>

/* ------------------------------------------------------------------ message universe + codec */
typedef struct {
    int n, V, E;
    uint32_t *key; /* sorted message keys (TLC order) */
    int nkey;
    int core_nib;  /* nibbles of the packed core */
    int core_bytes;
} pcodec_t;

static int cmp_key(const void *a, const void *b) { return cmp_u32(a, b); }

static void pc_build(pcodec_t *C, int n, int V, int E) {
    C->n = n; C->V = V; C->E = E;
    size_t cap = 1u << 16;
    C->key = (uint32_t *)malloc(cap * sizeof(uint32_t));
    int k = 0;
    for (int src = 0; src < n; src++)
        for (int dst = 0; dst < n; dst++)
            for (int term = 0; term <= E; term++) {
                C->key[k++] = k_vresp(src, dst, term);
                for (int i = 1; i <= V + 1; i++) {
                    for (int lt = 0; lt <= E; lt++) C->key[k++] = k_vreq(src, dst, term, i, lt);
                    for (int sc = 0; sc <= 1; sc++) C->key[k++] = k_aresp(src, dst, term, i, sc);
                    for (int plt = 0; plt <= E; plt++)
                        for (int lc = 1; lc <= V + 1; lc++) {
                            C->key[k++] = k_areq(src, dst, term, i, plt, 0, 0, 0, lc);
                            for (int et = 0; et <= E; et++)
                                for (int ev = 0; ev < V; ev++) C->key[k++] = k_areq(src, dst, term, i, plt, 1, et, ev, lc);
                        }
                }
            }
    if ((size_t)k > cap) { fprintf(stderr, "prefix: universe overflow\n"); exit(3); }
    qsort(C->key, (size_t)k, sizeof(uint32_t), cmp_key);
    int u = 0;
    for (int i = 0; i < k; i++)
        if (u == 0 || C->key[u - 1] != C->key[i]) C->key[u++] = C->key[i];
    C->nkey = u;
    if (u >= 0xFFFF) { fprintf(stderr, "prefix: universe exceeds 16-bit ids\n"); exit(3); }
    /* vf+1 ct role ci ll per server; (lt, lv+1) per log index 1..V+1; mi, ni; pend (4 per nibble);
     * ec rc; vs+1 per value; nm (2 nibbles) */
    C->core_nib = 5 * n + 2 * n * (V + 1) + 2 * n * n + (n * n + 3) / 4 + 2 + V + 2;
    C->core_bytes = (C->core_nib + 1) / 2;
}

static int pc_id(const pcodec_t *C, uint32_t k) {
    int lo = 0, hi = C->nkey - 1;
    while (lo <= hi) {
        int mid = (lo + hi) >> 1;
        if (C->key[mid] == k) return mid;
        if (C->key[mid] < k) lo = mid + 1; else hi = mid - 1;
    }
    fprintf(stderr, "prefix: message key %08x outside the universe\n", k);
    exit(3);
}

static inline void nib_put(uint8_t *b, int *p, unsigned v) {
    if (v > 15) { fprintf(stderr, "prefix: field %u exceeds a nibble\n", v); exit(3); }
    if (*p & 1) b[*p >> 1] |= (uint8_t)(v << 4); else b[*p >> 1] = (uint8_t)v;
    (*p)++;
}
static inline unsigned nib_get(const uint8_t *b, int *p) {
    unsigned v = (*p & 1) ? (b[*p >> 1] >> 4) : (b[*p >> 1] & 15u);
    (*p)++;
    return v;
}

/* record bytes of a state */
static inline size_t pc_size(const pcodec_t *C, int nm) { return (size_t)C->core_bytes + 2 * (size_t)nm; }

static size_t pc_encode(const pcodec_t *C, const st_t *s, uint8_t *o) {
    const int n = C->n, V = C->V;
    int p = 0;
    memset(o, 0, (size_t)C->core_bytes);
    for (int i = 0; i < n; i++) {
        nib_put(o, &p, (unsigned)(s->vf[i] + 1));
        nib_put(o, &p, (unsigned)s->ct[i]);
        nib_put(o, &p, (unsigned)s->role[i]);
        nib_put(o, &p, (unsigned)s->ci[i]);
        nib_put(o, &p, (unsigned)s->ll[i]);
        for (int x = 1; x <= V + 1; x++) {
            nib_put(o, &p, (unsigned)s->lt[i][x]);
            nib_put(o, &p, (unsigned)(s->lv[i][x] + 1));
        }
    }
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) { nib_put(o, &p, (unsigned)s->mi[i][j]); nib_put(o, &p, (unsigned)s->ni[i][j]); }
    for (int b = 0; b < n * n; b += 4) {
        unsigned v = 0;
        for (int q = 0; q < 4 && b + q < n * n; q++) v |= (unsigned)(s->pend[(b + q) / n][(b + q) % n] ? 1 : 0) << q;
        nib_put(o, &p, v);
    }
    nib_put(o, &p, (unsigned)s->ec);
    nib_put(o, &p, (unsigned)s->rc);
    for (int v = 0; v < V; v++) nib_put(o, &p, (unsigned)(s->vs[v] + 1));
    nib_put(o, &p, (unsigned)(s->nm & 15));
    nib_put(o, &p, (unsigned)(s->nm >> 4));
    uint16_t *ids = (uint16_t *)(o + C->core_bytes);
    for (int k = 0; k < s->nm; k++) {
        uint16_t id = (uint16_t)pc_id(C, s->m[k]);
        memcpy(ids + k, &id, 2);
    }
    return pc_size(C, s->nm);
}

static size_t pc_decode(const pcodec_t *C, const uint8_t *o, st_t *s) {
    const int n = C->n, V = C->V;
    int p = 0;
    memset(s, 0, HDR_BYTES);
    for (int i = 0; i < n; i++) {
        s->vf[i] = (int8_t)((int)nib_get(o, &p) - 1);
        s->ct[i] = (int8_t)nib_get(o, &p);
        s->role[i] = (int8_t)nib_get(o, &p);
        s->ci[i] = (int8_t)nib_get(o, &p);
        s->ll[i] = (int8_t)nib_get(o, &p);
        for (int x = 1; x <= V + 1; x++) {
            s->lt[i][x] = (int8_t)nib_get(o, &p);
            s->lv[i][x] = (int8_t)((int)nib_get(o, &p) - 1);
        }
    }
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) { s->mi[i][j] = (int8_t)nib_get(o, &p); s->ni[i][j] = (int8_t)nib_get(o, &p); }
    for (int b = 0; b < n * n; b += 4) {
        unsigned v = nib_get(o, &p);
        for (int q = 0; q < 4 && b + q < n * n; q++) s->pend[(b + q) / n][(b + q) % n] = (uint8_t)((v >> q) & 1);
    }
    s->ec = (int8_t)nib_get(o, &p);
    s->rc = (int8_t)nib_get(o, &p);
    for (int v = 0; v < V; v++) s->vs[v] = (int8_t)((int)nib_get(o, &p) - 1);
    s->nm = (int16_t)nib_get(o, &p);
    s->nm = (int16_t)(s->nm | (int16_t)(nib_get(o, &p) << 4));
    const uint16_t *ids = (const uint16_t *)(o + C->core_bytes);
    for (int k = 0; k < s->nm; k++) {
        uint16_t id;
        memcpy(&id, ids + k, 2);
        s->m[k] = C->key[id];
    }
    return pc_size(C, s->nm);
}

/* ------------------------------------------------------------------ level storage (T chunks) */
typedef struct { uint8_t *b; size_t len, cap; uint64_t *off; uint64_t n, ocap; } chunk_t;

static void ch_push(chunk_t *A, const pcodec_t *C, const st_t *s) {
    size_t sz = pc_size(C, s->nm);
    if (A->len + sz > A->cap) {
        A->cap = (A->cap ? A->cap + A->cap / 2 : (1u << 20)) + sz;
        A->b = (uint8_t *)realloc(A->b, A->cap);
        if (!A->b) { fprintf(stderr, "prefix: out of memory (level records)\n"); exit(3); }
    }
    if (A->n == A->ocap) {
        A->ocap = A->ocap ? A->ocap + A->ocap / 2 : 4096;
        A->off = (uint64_t *)realloc(A->off, A->ocap * sizeof(uint64_t));
        if (!A->off) { fprintf(stderr, "prefix: out of memory (offsets)\n"); exit(3); }
    }
    A->off[A->n++] = A->len;
    A->len += pc_encode(C, s, A->b + A->len);
}
static void ch_free(chunk_t *A) { free(A->b); free(A->off); memset(A, 0, sizeof *A); }

#define PMAXT 64
typedef struct {
    chunk_t ch[PMAXT];
    int nch;
    uint64_t base[PMAXT + 1]; /* global index of each chunk's first state */
} level_t;

static void lv_get(const level_t *L, const pcodec_t *C, uint64_t g, st_t *s) {
    int c = 0;
    while (g >= L->base[c + 1]) c++;
    const chunk_t *A = &L->ch[c];
    pc_decode(C, A->b + A->off[g - L->base[c]], s);
}
static void lv_free(level_t *L) { for (int c = 0; c < L->nch; c++) ch_free(&L->ch[c]); L->nch = 0; }

/* ------------------------------------------------------------------ hash tables */
static inline uint64_t home(uint64_t x, uint64_t cap) { return (uint64_t)(((__uint128_t)x * cap) >> 64); }

/* seen set: slot {lo | 1, hi | 1} (126 bits of the exact canonical form's hash); 1 if present */
static int sn_has(const uint64_t *K, uint64_t cap, const uint64_t h[2]) {
    const uint64_t lo = h[0] | 1, hi = h[1] | 1;  /* as the level table keeps them */
    uint64_t i = home(mix64(hi ^ 0x51ed270b7a3c5f11ULL), cap);
    for (;;) {
        const uint64_t k = __atomic_load_n(&K[2 * i], __ATOMIC_ACQUIRE);
        if (k == 0) return 0;
        if (k == lo && __atomic_load_n(&K[2 * i + 1], __ATOMIC_ACQUIRE) == hi) return 1;
        if (++i == cap) i = 0;
    }
}
static void sn_put(uint64_t *K, uint64_t cap, const uint64_t h[2]) {
    const uint64_t lo = h[0] | 1, hi = h[1] | 1;  /* as the level table keeps them */
    uint64_t i = home(mix64(hi ^ 0x51ed270b7a3c5f11ULL), cap);
    for (;;) {
        uint64_t zero = 0;
        if (__atomic_compare_exchange_n(&K[2 * i], &zero, lo, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
            __atomic_store_n(&K[2 * i + 1], hi, __ATOMIC_RELEASE);
            return;
        }
        if (++i == cap) i = 0;
    }
}

typedef struct { uint64_t lo, hi, key; } lt_t;    /* level election slot: the smallest key wins */
typedef struct { uint64_t key, lo, hi; } win_t;   /* a winner: key + its hash */

static uint64_t g_lt_fill;  /* slots claimed in the level table (overflow detection) */

static int lt_elect(lt_t *T, uint64_t cap, const uint64_t h[2], uint64_t key) {
    const uint64_t lo = h[0] | 1, hi = h[1] | 1;
    uint64_t i = home(mix64(lo ^ (hi >> 7)), cap);
    for (uint64_t probes = 0; probes < cap; probes++) {
        lt_t *s = &T[i];
        uint64_t cur = __atomic_load_n(&s->lo, __ATOMIC_ACQUIRE);
        if (cur == 0) {
            uint64_t zero = 0;
            if (__atomic_compare_exchange_n(&s->lo, &zero, lo, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
                __atomic_store_n(&s->hi, hi, __ATOMIC_RELEASE);
                __atomic_fetch_add(&g_lt_fill, 1, __ATOMIC_RELAXED);
                cur = lo;
            } else {
                cur = zero;
            }
        }
        if (cur == lo) {
            uint64_t h2;
            while ((h2 = __atomic_load_n(&s->hi, __ATOMIC_ACQUIRE)) == 0) { /* claimer's hi in flight */ }
            if (h2 == hi) {
                uint64_t old = __atomic_load_n(&s->key, __ATOMIC_RELAXED);
                while (key < old &&
                       !__atomic_compare_exchange_n(&s->key, &old, key, 1, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED)) {
                }
                return 0;
            }
        }
        if (++i == cap) i = 0;
    }
    return -1;
}

/* ------------------------------------------------------------------ the level phases */
typedef struct {
    const ocfg_t *c;
    const perms_t *P;
    const pcodec_t *C;
    const level_t *cur;
    uint64_t *seen;
    uint64_t seen_cap;
    lt_t *lt;
    uint64_t lt_cap;
    int T, tid;
    uint64_t p0, p1;          /* parents of this thread (global indices) */
    uint64_t generated, gen_msgs_max;
    int overflow;
    /* winner collection */
    uint64_t s0, s1;          /* level-table slice */
    uint64_t *cnt;            /* [T] winners of this slice per owner */
    win_t *W;                 /* all winners, grouped by owner */
    uint64_t *woff;           /* [T][T] write offsets (scanner-major) */
    uint64_t w0, w1;          /* this owner's winners */
    chunk_t *out;             /* next level's chunk of this owner */
    int violated;
    int max_nm;
} pw_t;

static void *ph_expand(void *arg) {
    pw_t *w = (pw_t *)arg;
    const ocfg_t *c = w->c;
    st_t *ps = (st_t *)malloc(sizeof(st_t));
    batch_t b;
    b.buf = (st_t *)malloc(sizeof(st_t) * BATCH_CAP);
    b.w = (int32_t *)malloc(sizeof(int32_t) * BATCH_CAP);
    b.cap = BATCH_CAP;
    w->generated = 0;
    w->overflow = 0;
    for (uint64_t i = w->p0; i < w->p1 && !w->overflow; i++) {
        lv_get(w->cur, w->C, i, ps);
        uint64_t rank = 0;
        for (int s = 0; s < c->n; s++)
            for (int ai = 0; ai < N_ORDER; ai++) {
                const int a = ACT_ORDER[ai];
                if (a == A_BF && !c->bf) continue;
                b.n = 0;
                b.assert_fail = 0;
                gen_action(c, ps, s, a, &b);
                w->generated += (uint64_t)b.n;
                for (int j = 0; j < b.n; j++, rank++) {
                    uint64_t h[2];
                    canon_hash(c, w->P, &b.buf[j], h);
                    if (sn_has(w->seen, w->seen_cap, h)) continue;
                    if (lt_elect(w->lt, w->lt_cap, h, (i << 16) | rank) < 0 ||
                        __atomic_load_n(&g_lt_fill, __ATOMIC_RELAXED) * 10 > w->lt_cap * 9) {
                        w->overflow = 1;
                        break;
                    }
                }
            }
    }
    free(ps); free(b.buf); free(b.w);
    return NULL;
}

static int owner_of(const pw_t *W0, int T, uint64_t parent) {
    int t = 0;
    while (t + 1 < T && parent >= W0[t + 1].p0) t++;
    return t;
}

static void *ph_count(void *arg) {  /* winners of this level-table slice, per owner */
    pw_t *w = (pw_t *)arg;
    pw_t *all = w - w->tid;
    for (int t = 0; t < w->T; t++) w->cnt[t] = 0;
    for (uint64_t i = w->s0; i < w->s1; i++)
        if (w->lt[i].lo) w->cnt[owner_of(all, w->T, w->lt[i].key >> 16)]++;
    return NULL;
}

static void *ph_scatter(void *arg) {
    pw_t *w = (pw_t *)arg;
    pw_t *all = w - w->tid;
    uint64_t *at = w->woff + (size_t)w->tid * w->T;
    for (uint64_t i = w->s0; i < w->s1; i++)
        if (w->lt[i].lo) {
            const int o = owner_of(all, w->T, w->lt[i].key >> 16);
            win_t *x = &w->W[at[o]++];
            x->key = w->lt[i].key; x->lo = w->lt[i].lo; x->hi = w->lt[i].hi;
        }
    return NULL;
}

static int cmp_win(const void *a, const void *b) {
    uint64_t x = ((const win_t *)a)->key, y = ((const win_t *)b)->key;
    return x < y ? -1 : x > y;
}

/* walk this owner's sorted winners in TLC order, re-generating each winning parent's successors
 * (no hashing): pass 0 sizes the next level's chunk, pass 1 packs the winners into it */
static void commit_pass(pw_t *w, int pass, st_t *ps, batch_t *b) {
    const ocfg_t *c = w->c;
    uint64_t k = w->w0;
    size_t bytes = 0;
    while (k < w->w1) {
        const uint64_t parent = w->W[k].key >> 16;
        lv_get(w->cur, w->C, parent, ps);
        uint64_t rank = 0;
        for (int s = 0; s < c->n && k < w->w1 && (w->W[k].key >> 16) == parent; s++)
            for (int ai = 0; ai < N_ORDER && k < w->w1 && (w->W[k].key >> 16) == parent; ai++) {
                const int a = ACT_ORDER[ai];
                if (a == A_BF && !c->bf) continue;
                b->n = 0;
                b->assert_fail = 0;
                gen_action(c, ps, s, a, b);
                for (int j = 0; j < b->n; j++, rank++) {
                    if (k >= w->w1 || (w->W[k].key >> 16) != parent) break;
                    if ((w->W[k].key & 0xFFFF) != rank) continue;
                    const st_t *t = &b->buf[j];
                    if (pass == 0) {
                        bytes += pc_size(w->C, t->nm);
                    } else {
                        uint64_t h[2] = {w->W[k].lo, w->W[k].hi};
                        sn_put(w->seen, w->seen_cap, h);
                        ch_push(w->out, w->C, t);
                        if (t->nm > w->max_nm) w->max_nm = t->nm;
                        if (w->violated < 0)
                            for (int i = 0; i < N_INV; i++)
                                if ((c->inv_mask & (1u << i)) && inv_eval(c, t, i) != 1) { w->violated = i; break; }
                    }
                    k++;
                }
            }
        if (k < w->w1 && (w->W[k].key >> 16) == parent) {
            fprintf(stderr, "prefix: winner rank %llu of parent %llu not generated\n",
                    (unsigned long long)(w->W[k].key & 0xFFFF), (unsigned long long)parent);
            exit(3);
        }
    }
    if (pass == 0) {  /* the chunk at its exact size: no realloc copies at the memory peak */
        chunk_t *A = w->out;
        A->cap = bytes ? bytes : 1;
        A->ocap = (w->w1 - w->w0) ? (w->w1 - w->w0) : 1;
        A->b = (uint8_t *)malloc(A->cap);
        A->off = (uint64_t *)malloc(A->ocap * sizeof(uint64_t));
        if (!A->b || !A->off) { fprintf(stderr, "prefix: out of memory (next level)\n"); exit(3); }
    }
}

static void *ph_commit(void *arg) {  /* sort this owner's winners; pack them in TLC order */
    pw_t *w = (pw_t *)arg;
    qsort(w->W + w->w0, (size_t)(w->w1 - w->w0), sizeof(win_t), cmp_win);
    st_t *ps = (st_t *)malloc(sizeof(st_t));
    batch_t b;
    b.buf = (st_t *)malloc(sizeof(st_t) * BATCH_CAP);
    b.w = (int32_t *)malloc(sizeof(int32_t) * BATCH_CAP);
    b.cap = BATCH_CAP;
    w->violated = -1;
    w->max_nm = 0;
    commit_pass(w, 0, ps, &b);
    commit_pass(w, 1, ps, &b);
    free(ps); free(b.buf); free(b.w);
    return NULL;
}

static void run_all(pw_t *W, int T, void *(*fn)(void *)) {
    pthread_t th[PMAXT];
    for (int t = 1; t < T; t++) pthread_create(&th[t], NULL, fn, &W[t]);
    fn(&W[0]);
    for (int t = 1; t < T; t++) pthread_join(th[t], NULL);
}

/* Level-synchronous first-wins BFS of (n, V, E, R), stopped at the first level boundary where
 * `max_states` distinct states are reached (0 = exhaust).  seen_slots = the seen set's capacity
 * (16 B each; must exceed every state the run finds).  Per level k (0-based, level k+1):
 * lv[k] distinct states, lg[k] successors generated expanding it, lm[k] the largest |msgs| of
 * its states.  Returns 0 exhausted, 2 stopped at max_states, 1 invariant violated, -1 capacity. */
int orc_prefix_levels(int n, int V, int E, int R, int threads, uint64_t max_states, uint64_t seen_slots,
                      uint64_t *lv, uint64_t *lg, int *lm, int lcap, uint64_t *distinct, uint64_t *generated,
                      int *depth) {
    if (threads < 1) threads = 1;
    if (threads > PMAXT) threads = PMAXT;
    ocfg_t c = {n, V, E, R, 0, 0, 1u << I_LHACE, 0, 0, 0, 0, 0, 0};
    perms_t *P = (perms_t *)malloc(sizeof(perms_t));
    make_perms(n, P);
    pcodec_t C;
    pc_build(&C, n, V, E);
    if (seen_slots < 1024) seen_slots = 1024;
    uint64_t *seen = (uint64_t *)calloc(seen_slots * 2, sizeof(uint64_t));
    if (!seen) { fprintf(stderr, "prefix: cannot allocate the seen set\n"); return -1; }
    level_t cur;
    memset(&cur, 0, sizeof cur);
    st_t *s0 = (st_t *)calloc(1, sizeof(st_t));
    init_state(&c, s0);
    uint64_t h[2];
    canon_hash(&c, P, s0, h);
    sn_put(seen, seen_slots, h);
    cur.nch = 1;
    ch_push(&cur.ch[0], &C, s0);
    cur.base[0] = 0;
    cur.base[1] = 1;
    uint64_t cur_n = 1, dist = 1, gen = 1, prev_n = 1;
    int dep = 1, verdict = 0;
    if (lcap > 0) { lv[0] = 1; lm[0] = 0; }
    pw_t *W = (pw_t *)calloc((size_t)threads, sizeof(pw_t));
    uint64_t *cnt = (uint64_t *)calloc((size_t)threads * threads, sizeof(uint64_t));
    uint64_t *woff = (uint64_t *)calloc((size_t)threads * threads, sizeof(uint64_t));
    double growth = 3.0;
    while (cur_n > 0) {
        const int T = (uint64_t)threads < cur_n ? threads : (int)cur_n;
        /* level table: every new state of the level, at load <= 0.9 */
        uint64_t lt_cap = (uint64_t)((double)cur_n * growth * 1.6) + 4096;
        lt_t *lt = NULL;
        int ok = 0;
        uint64_t lgen = 0;
        while (!ok) {
            lt = (lt_t *)malloc(lt_cap * sizeof(lt_t));
            if (!lt) { fprintf(stderr, "prefix: cannot allocate the level table\n"); return -1; }
            for (uint64_t i = 0; i < lt_cap; i++) { lt[i].lo = 0; lt[i].hi = 0; lt[i].key = ~0ull; }
            g_lt_fill = 0;
            for (int t = 0; t < T; t++) {
                W[t] = (pw_t){0};
                W[t].c = &c; W[t].P = P; W[t].C = &C; W[t].cur = &cur; W[t].seen = seen; W[t].seen_cap = seen_slots;
                W[t].lt = lt; W[t].lt_cap = lt_cap; W[t].T = T; W[t].tid = t;
                W[t].p0 = cur_n * (uint64_t)t / (uint64_t)T;
                W[t].p1 = cur_n * (uint64_t)(t + 1) / (uint64_t)T;
                W[t].cnt = cnt + (size_t)t * T; W[t].woff = woff;
            }
            run_all(W, T, ph_expand);
            ok = 1;
            lgen = 0;
            for (int t = 0; t < T; t++) { if (W[t].overflow) ok = 0; lgen += W[t].generated; }
            if (!ok) {  /* redo the level with twice the table */
                free(lt);
                lt_cap *= 2;
                fprintf(stderr, "prefix: level %d table full, retrying with %llu slots\n", dep,
                        (unsigned long long)lt_cap);
            }
        }
        gen += lgen;
        if (dep - 1 < lcap) lg[dep - 1] = lgen;
        const uint64_t nw = g_lt_fill;
        if (dist + nw > seen_slots * 9 / 10) {
            fprintf(stderr, "prefix: seen set too small (%llu slots for %llu states)\n",
                    (unsigned long long)seen_slots, (unsigned long long)(dist + nw));
            free(lt);
            verdict = -1;
            break;
        }
        /* winners grouped by owner (the thread that expanded their parent), then freed table */
        win_t *Wn = (win_t *)malloc((nw ? nw : 1) * sizeof(win_t));
        if (!Wn) { fprintf(stderr, "prefix: cannot allocate the winners\n"); return -1; }
        for (int t = 0; t < T; t++) {
            W[t].s0 = lt_cap * (uint64_t)t / (uint64_t)T;
            W[t].s1 = lt_cap * (uint64_t)(t + 1) / (uint64_t)T;
            W[t].W = Wn;
        }
        run_all(W, T, ph_count);
        uint64_t acc = 0;
        for (int o = 0; o < T; o++) {
            W[o].w0 = acc;
            for (int sc = 0; sc < T; sc++) { woff[(size_t)sc * T + o] = acc; acc += cnt[(size_t)sc * T + o]; }
            W[o].w1 = acc;
        }
        run_all(W, T, ph_scatter);
        free(lt);
        level_t nxt;
        memset(&nxt, 0, sizeof nxt);
        nxt.nch = T;
        for (int t = 0; t < T; t++) W[t].out = &nxt.ch[t];
        run_all(W, T, ph_commit);
        free(Wn);
        int mnm = 0;
        nxt.base[0] = 0;
        for (int t = 0; t < T; t++) {
            if (W[t].violated >= 0 && verdict == 0) verdict = 1;
            if (W[t].max_nm > mnm) mnm = W[t].max_nm;
            nxt.base[t + 1] = nxt.base[t] + nxt.ch[t].n;
        }
        if (nxt.base[T] != nw) { fprintf(stderr, "prefix: committed %llu of %llu winners\n",
                                         (unsigned long long)nxt.base[T], (unsigned long long)nw); exit(3); }
        lv_free(&cur);
        cur = nxt;
        prev_n = cur_n;
        cur_n = nw;
        dist += nw;
        growth = prev_n ? (double)nw / (double)prev_n : 3.0;
        if (growth < 1.0) growth = 1.0;
        if (nw && dep < lcap) { lv[dep] = nw; lm[dep] = mnm; }
        if (nw) dep++;
        fprintf(stderr, "prefix: level %d: %llu states (max |msgs| %d), %llu distinct, %llu generated\n", dep,
                (unsigned long long)nw, mnm, (unsigned long long)dist, (unsigned long long)gen);
        if (verdict) break;
        if (max_states && dist >= max_states && cur_n > 0) { verdict = 2; break; }
    }
    free(W); free(cnt); free(woff); free(seen); free(s0); free(P); free(C.key);
    lv_free(&cur);
    *distinct = dist;
    *generated = gen;
    *depth = dep;
    return verdict;
}

/* codec self-check: encode/decode round trip of every state of a small BFS (tests/test_oracle.py) */
int orc_prefix_codec_check(int n, int V, int E, int R, uint64_t max_states) {
    ocfg_t c = {n, V, E, R, 0, 0, 1u << I_LHACE, 0, 0, 0, 0, 0, 0};
    pcodec_t C;
    pc_build(&C, n, V, E);
    st_t *s = (st_t *)calloc(1, sizeof(st_t)), *t = (st_t *)calloc(1, sizeof(st_t));
    batch_t b;
    b.buf = (st_t *)malloc(sizeof(st_t) * BATCH_CAP);
    b.w = (int32_t *)malloc(sizeof(int32_t) * BATCH_CAP);
    b.cap = BATCH_CAP;
    uint8_t *rec = (uint8_t *)malloc(pc_size(&C, MCAP));
    init_state(&c, s);
    uint64_t checked = 0;
    int bad = 0;
    /* a walk over first successors of every action, plus every successor's round trip */
    for (uint64_t step = 0; step < max_states && !bad; step++) {
        int found = 0;
        for (int sv = 0; sv < n; sv++)
            for (int a = 0; a < N_ACTIONS; a++) {
                b.n = 0; b.assert_fail = 0;
                gen_action(&c, s, sv, a, &b);
                for (int j = 0; j < b.n; j++) {
                    pc_encode(&C, &b.buf[j], rec);
                    memset(t, 0x5a, sizeof(st_t));
                    pc_decode(&C, rec, t);
                    if (memcmp(t, &b.buf[j], HDR_BYTES) || memcmp(t->m, b.buf[j].m, (size_t)b.buf[j].nm * 4)) bad = 1;
                    checked++;
                }
                if (b.n && !found && ((step * 7 + (uint64_t)sv * 3 + (uint64_t)a) % 5 == 0)) { *s = b.buf[b.n - 1]; found = 1; }
            }
        if (!found) break;
    }
    free(s); free(t); free(b.buf); free(b.w); free(rec); free(C.key);
    return bad ? -1 : (int)checked;
}
