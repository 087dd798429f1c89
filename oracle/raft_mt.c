/*
 * TEST INFRASTRUCTURE ONLY -- multi-threaded CPU baseline for bench.py's cpu_baseline leg.
 *
 * The same restatement of Raft.tla as oracle/raft_oracle.c (this file includes it and reuses its
 * successor generator gen_action, exact canonical form canon_hash and invariants), run as a
 * level-synchronous breadth-first search on T host threads with TLC -workers 1 semantics
 * (FIFO order, first discovery wins, invariants on new states):
 *
 *   1. expand: thread t takes the contiguous block t of the level's states; every successor in
 *      TLC enumeration order gets its canonical 128-bit hash; those not in the seen set become
 *      candidates with key = (parent index, rank in the parent's successor list);
 *   2. elect:  candidates meet in a per-level table keyed by hash; an atomic minimum keeps the
 *      smallest key (= first in TLC order) per hash;
 *   3. commit: each thread keeps its candidates that won, in order; the blocks concatenated in
 *      thread order are the next level in TLC FIFO order; winners enter the seen set.
 *
 * Same counts as the single-threaded oracle on every configuration (tests/test_oracle.py); it
 * exists to put an honest all-cores CPU number beside the GPU one.  It is not TLC (no JVM here).
 */
#include "raft_oracle.c"

#include <pthread.h>

typedef struct {
    uint64_t lo, hi;
    uint64_t key; /* (parent << 16) | rank; ~0 = empty */
} lslot_t;

typedef struct {
    /* shared */
    const ocfg_t *c;
    const perms_t *P;
    const arena_t *cur;
    uint64_t *seen;        /* 2 words per slot, lo | 1 == 0 means empty */
    uint64_t seen_cap;
    lslot_t *lt;           /* level election table */
    uint64_t lt_cap;
    int nthreads;
    /* per thread */
    int tid;
    uint64_t p0, p1;
    uint64_t generated;
    arena_t cand;          /* candidate states, in TLC order */
    uint64_t *ch;          /* candidate hashes (2 words each) */
    uint64_t *ckey;
    uint64_t ncand, ccap;
    arena_t win;           /* winners, in TLC order */
    uint64_t nwin;
    int violated;          /* first invariant violation among the winners (-1 none) */
} worker_t;

static int seen_has(const uint64_t *K, uint64_t cap, const uint64_t h[2]) {
    uint64_t lo = h[0] | 1, hi = h[1];
    uint64_t i = (hi ^ (hi >> 29)) & (cap - 1);
    for (;;) {
        uint64_t k = __atomic_load_n(&K[2 * i], __ATOMIC_ACQUIRE);
        if (k == 0) return 0;
        if (k == lo && __atomic_load_n(&K[2 * i + 1], __ATOMIC_ACQUIRE) == hi) return 1;
        i = (i + 1) & (cap - 1);
    }
}

static void seen_put(uint64_t *K, uint64_t cap, const uint64_t h[2]) {
    uint64_t lo = h[0] | 1, hi = h[1];
    uint64_t i = (hi ^ (hi >> 29)) & (cap - 1);
    for (;;) {
        uint64_t zero = 0;
        if (__atomic_compare_exchange_n(&K[2 * i], &zero, lo, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
            __atomic_store_n(&K[2 * i + 1], hi, __ATOMIC_RELEASE);
            return;
        }
        i = (i + 1) & (cap - 1);
    }
}

/* election: the slot of hash h, claimed if free; the smallest key wins */
static lslot_t *elect(lslot_t *T, uint64_t cap, const uint64_t h[2], uint64_t key) {
    uint64_t lo = h[0] | 1, hi = h[1] | 1;  /* hi | 1: a slot's hi word is nonzero once set */
    uint64_t i = (lo ^ (lo >> 31) ^ (hi >> 7)) & (cap - 1);
    for (;;) {
        lslot_t *s = &T[i];
        uint64_t cur = __atomic_load_n(&s->lo, __ATOMIC_ACQUIRE);
        if (cur == 0) {
            uint64_t zero = 0;
            if (__atomic_compare_exchange_n(&s->lo, &zero, lo, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
                __atomic_store_n(&s->hi, hi, __ATOMIC_RELEASE);
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
                return s;
            }
        }
        i = (i + 1) & (cap - 1);
    }
}

static void *phase_expand(void *arg) {
    worker_t *w = (worker_t *)arg;
    const ocfg_t *c = w->c;
    st_t *ps = (st_t *)malloc(sizeof(st_t));
    batch_t b;
    b.buf = (st_t *)malloc(sizeof(st_t) * BATCH_CAP);
    b.w = (int32_t *)malloc(sizeof(int32_t) * BATCH_CAP);
    b.cap = BATCH_CAP;
    w->ncand = 0;
    w->generated = 0;
    for (uint64_t i = w->p0; i < w->p1; i++) {
        ar_get(w->cur, i, ps);
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
                    if (seen_has(w->seen, w->seen_cap, h)) continue;
                    if (w->ncand == w->ccap) {
                        w->ccap = w->ccap ? 2 * w->ccap : 4096;
                        w->ch = (uint64_t *)realloc(w->ch, w->ccap * 2 * sizeof(uint64_t));
                        w->ckey = (uint64_t *)realloc(w->ckey, w->ccap * sizeof(uint64_t));
                    }
                    w->ch[2 * w->ncand] = h[0];
                    w->ch[2 * w->ncand + 1] = h[1];
                    w->ckey[w->ncand] = (i << 16) | rank;
                    w->ncand++;
                    ar_push(&w->cand, &b.buf[j]);
                }
            }
    }
    free(ps); free(b.buf); free(b.w);
    return NULL;
}

static void *phase_elect(void *arg) {
    worker_t *w = (worker_t *)arg;
    for (uint64_t k = 0; k < w->ncand; k++) elect(w->lt, w->lt_cap, &w->ch[2 * k], w->ckey[k]);
    return NULL;
}

static void *phase_commit(void *arg) {
    worker_t *w = (worker_t *)arg;
    st_t *t = (st_t *)malloc(sizeof(st_t));
    w->nwin = 0;
    w->violated = -1;
    for (uint64_t k = 0; k < w->ncand; k++) {
        lslot_t *s = elect(w->lt, w->lt_cap, &w->ch[2 * k], ~0ull);  /* find (key ~0 never wins) */
        if (__atomic_load_n(&s->key, __ATOMIC_ACQUIRE) != w->ckey[k]) continue;
        ar_get(&w->cand, k, t);
        seen_put(w->seen, w->seen_cap, &w->ch[2 * k]);
        ar_push(&w->win, t);
        w->nwin++;
        if (w->violated < 0) {
            for (int i = 0; i < N_INV; i++)
                if ((w->c->inv_mask & (1u << i)) && inv_eval(w->c, t, i) != 1) { w->violated = i; break; }
        }
    }
    free(t);
    return NULL;
}

static void run_phase(worker_t *W, int T, void *(*fn)(void *)) {
    pthread_t th[256];
    for (int t = 1; t < T; t++) pthread_create(&th[t], NULL, fn, &W[t]);
    fn(&W[0]);
    for (int t = 1; t < T; t++) pthread_join(th[t], NULL);
}

static int mt_bfs(int n, int V, int E, int R, int threads, uint64_t max_states, uint64_t *lv, uint64_t *lg,
                  int lcap, uint64_t *distinct, uint64_t *generated, int *depth);

/* Exhaust (n, V, E, R) with `threads` threads; returns 0 done, 1 invariant violated, -1 error.
 * out: distinct, generated, depth. */
int orc_mt_run(int n, int V, int E, int R, int threads, uint64_t *distinct, uint64_t *generated, int *depth) {
    return mt_bfs(n, V, E, R, threads, 0, NULL, NULL, 0, distinct, generated, depth);
}

/* Prefix levels (tests/golden/make_golden_prefix.py --mt): the same BFS, stopped at the first
 * level boundary where `max_states` distinct states are reached.  Being level-synchronous, every
 * level it reports is complete: lv[k] = distinct states of level k+1 (k < depth), lg[k] = successors
 * generated expanding level k+1 (k < depth - 1, or k < depth when the run exhausted).
 * Returns 0 exhausted, 2 stopped at max_states, 1 invariant violated. */
int orc_mt_levels(int n, int V, int E, int R, int threads, uint64_t max_states, uint64_t *lv, uint64_t *lg, int lcap,
                  uint64_t *distinct, uint64_t *generated, int *depth) {
    return mt_bfs(n, V, E, R, threads, max_states, lv, lg, lcap, distinct, generated, depth);
}

static int mt_bfs(int n, int V, int E, int R, int threads, uint64_t max_states, uint64_t *lv, uint64_t *lg,
                  int lcap, uint64_t *distinct, uint64_t *generated, int *depth) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    ocfg_t c = {n, V, E, R, 0, 0, 1u << I_LHACE, 0, 0, 0, 0, 0, 0};
    perms_t *P = (perms_t *)malloc(sizeof(perms_t));
    make_perms(n, P);
    uint64_t seen_cap = 1u << 20;
    uint64_t *seen = (uint64_t *)calloc(seen_cap * 2, sizeof(uint64_t));
    arena_t cur = {0};
    st_t *s0 = (st_t *)malloc(sizeof(st_t));
    init_state(&c, s0);
    uint64_t h[2];
    canon_hash(&c, P, s0, h);
    seen_put(seen, seen_cap, h);
    ar_push(&cur, s0);
    uint64_t dist = 1, gen = 1, seen_n = 1;
    int dep = 1, verdict = 0;
    if (lcap > 0) lv[0] = 1;
    worker_t *W = (worker_t *)calloc((size_t)threads, sizeof(worker_t));
    lslot_t *lt = NULL;
    uint64_t lt_cap = 0;
    while (cur.n > 0) {
        const int T = (uint64_t)threads < cur.n ? threads : (int)cur.n;
        for (int t = 0; t < T; t++) {
            W[t].c = &c; W[t].P = P; W[t].cur = &cur; W[t].seen = seen; W[t].seen_cap = seen_cap;
            W[t].tid = t; W[t].nthreads = T;
            W[t].p0 = cur.n * (uint64_t)t / (uint64_t)T;
            W[t].p1 = cur.n * (uint64_t)(t + 1) / (uint64_t)T;
            ar_clear(&W[t].cand);
            ar_clear(&W[t].win);
        }
        run_phase(W, T, phase_expand);
        uint64_t ncand = 0;
        uint64_t lgen = 0;
        for (int t = 0; t < T; t++) { ncand += W[t].ncand; lgen += W[t].generated; }
        gen += lgen;
        if (dep - 1 < lcap) lg[dep - 1] = lgen;
        uint64_t need = 1;
        while (need < 2 * ncand + 2) need <<= 1;
        if (need > lt_cap) { free(lt); lt_cap = need; lt = (lslot_t *)malloc(lt_cap * sizeof(lslot_t)); }
        for (uint64_t i = 0; i < lt_cap; i++) { lt[i].lo = 0; lt[i].hi = 0; lt[i].key = ~0ull; }
        /* the seen set takes every winner at load <= 1/2 (winners <= candidates) */
        if ((seen_n + ncand) * 2 > seen_cap) {
            uint64_t nc = seen_cap;
            while ((seen_n + ncand) * 2 > nc) nc *= 2;
            uint64_t *ns = (uint64_t *)calloc(nc * 2, sizeof(uint64_t));
            for (uint64_t i = 0; i < seen_cap; i++)
                if (seen[2 * i]) { uint64_t hh[2] = {seen[2 * i], seen[2 * i + 1]}; seen_put(ns, nc, hh); }
            free(seen);
            seen = ns;
            seen_cap = nc;
        }
        for (int t = 0; t < T; t++) { W[t].lt = lt; W[t].lt_cap = lt_cap; W[t].seen = seen; W[t].seen_cap = seen_cap; }
        run_phase(W, T, phase_elect);
        run_phase(W, T, phase_commit);
        arena_t nxt = {0};
        uint64_t nw = 0;
        for (int t = 0; t < T; t++) {
            if (W[t].violated >= 0 && verdict == 0) verdict = 1;
            for (uint64_t k = 0; k < W[t].nwin; k++) {
                st_t tmp;
                ar_get(&W[t].win, k, &tmp);
                ar_push(&nxt, &tmp);
            }
            nw += W[t].nwin;
        }
        seen_n += nw;
        dist += nw;
        ar_free(&cur);
        cur = nxt;
        if (nw && dep < lcap) lv[dep] = nw;
        if (nw) dep++;
        if (verdict) break;
        if (max_states && dist >= max_states && cur.n > 0) { verdict = 2; break; }
    }
    for (int t = 0; t < threads; t++) { ar_free(&W[t].cand); ar_free(&W[t].win); free(W[t].ch); free(W[t].ckey); }
    free(W); free(lt); free(seen); free(s0); free(P); ar_free(&cur);
    *distinct = dist;
    *generated = gen;
    *depth = dep;
    return verdict;
}
