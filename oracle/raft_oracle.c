/*
 * TEST INFRASTRUCTURE ONLY -- C restatement of kikimo/tla-raft's hot path.
 *
 * This is the parity oracle's fast twin of oracle/raft_ref.py.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only
 * as the checker / CPU baseline; the product library (tla-raft_amd/) never links
 * or calls it.
 *
 * It restates /root/reference/Raft.tla (cited tla:N) under Raft.cfg (cfg:N) with
 * TLC -workers 1 breadth-first semantics (myrun.sh run:3 passes -deadlock):
 *   Init tla:93-105; Next tla:416-430 (server-major, disjuncts in textual order,
 *   \E witnesses in TLC's normalised order); helpers tla:41-49,70-75,271-273;
 *   invariants tla:434-499; SYMMETRY Permutations(Servers) tla:21/cfg:24;
 *   VIEW tla:38/cfg:26.
 *
 * Independence from the product: distinct states are identified here by the
 * EXACT lexicographically-minimal permuted view (bytes + sorted permuted message
 * keys), then hashed to 128 bits for the seen-set.  The GPU path instead takes
 * the minimum of a structured 128-bit hash over permutations; the two methods
 * agree unless a 128-bit collision occurs.
 *
 * Parity status: unpinned by the reference (no TLC jar, no logs, no published
 * counts: .gitignore:1-3, BASELINE.json "published": {}).  Pinned by SURVEY.md
 * Appendix C's hand-derived answers and by agreement with raft_ref.py.
 *
 * Message representation: a 32-bit key whose unsigned order equals TLC's record
 * order (field count, then (sorted field name, value) pairs):
 *   [31:30] class 0 = VoteResp (4 fields), 1 = 6-field record, 2 = AppendReq (8)
 *   [29:27] dst
 *   VoteResp   : [26:24] src  [23:21] term
 *   VoteReq    : [26]=0 [25:23] lastLogIndex [22:20] lastLogTerm [19:17] src [16:14] term
 *   AppendResp : [26]=1 [25:23] prevLogIndex [22:20] src [19] succ [18:16] term
 *   AppendReq  : [26] len(entries) [25:23] entry.term [22:21] entry.val
 *                [20:18] leaderCommit [17:15] prevLogIndex [14:12] prevLogTerm
 *                [11:9] src [8:6] term
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define MAXN 5
#define MAXV 3
#define MAXL (MAXV + 2) /* log index 1..V+1 used */
#define MCAP 160
#define MAXLEVELS 1024

enum { R_F = 0, R_C = 1, R_L = 2 };
enum { MT_VREQ = 0, MT_VRESP = 1, MT_AREQ = 2, MT_ARESP = 3 };
enum { A_BC, A_UT, A_RV, A_BL, A_CR, A_LAE, A_FAE, A_FRE, A_HAR, A_LCC, A_RS, N_ACTIONS };
/* BecomeFollower (tla:190-231): in Next only in the tla:420 variant, right after UpdateTerm */
#define A_BF 12
/* Next's disjuncts in TLC's enumeration order (tla:416-430) */
static const int ACT_ORDER[] = {A_BC, A_UT, A_BF, A_RV, A_BL, A_CR, A_LAE, A_FAE, A_FRE, A_HAR, A_LCC, A_RS};
#define N_ORDER 12
enum { V_OK = 0, V_INVARIANT = 1, V_ASSERT = 2, V_EVAL_ERROR = 3, V_DEADLOCK = 4, V_LIMIT = 5, V_CAPACITY = 6 };

/* invariant ids (bit positions of ocfg_t.inv_mask) */
enum { I_LHACE = 0, I_NOSPLIT = 1, I_RAFTCANCOMMIT = 2, I_FOLLOWERCANCOMMIT = 3, I_COMMITALL = 4,
       I_NOALLCOMMIT = 5, I_EXISTLC = 6, N_INV = 7 };

typedef struct {
    int n, V, E, R;
    int seeded;         /* RaftSeeded: Median threshold = Cardinality(Servers) */
    int check_deadlock; /* 0 = -deadlock (run:3) */
    uint32_t inv_mask;  /* bit I_* : checked invariants, in bit order */
    int record_trace;
    int order;          /* 0 = TLC -workers 1 order; 1 = reversed; 2 = seeded shuffle (order-sensitivity probe) */
    uint64_t seed;
    int bf;             /* the BecomeFollower variant (tla:420 uncommented) */
    int sb;             /* RaftSplitBrain (test variant): BecomeLeader's quorum (tla:164) is 1 */
    int cpl;            /* RaftCommitPastLog (test variant): newCommitIndex (tla:294) = Max(ci, leaderCommit) */
} ocfg_t;
/* spec flags of the C API's `seeded` argument: bit 0 RaftSeeded, bit 1 BecomeFollower variant,
 * bit 2 RaftSplitBrain, bit 3 RaftCommitPastLog */
static void set_variant(ocfg_t *c, int flags) {
    c->seeded = flags & 1; c->bf = (flags >> 1) & 1; c->sb = (flags >> 2) & 1; c->cpl = (flags >> 3) & 1;
}

typedef struct {
    int8_t vf[MAXN], ct[MAXN], role[MAXN], ci[MAXN], ll[MAXN];
    int8_t lt[MAXN][MAXL], lv[MAXN][MAXL]; /* 1-based log index */
    int8_t mi[MAXN][MAXN], ni[MAXN][MAXN];
    uint8_t pend[MAXN][MAXN];
    int8_t ec, rc, vs[MAXV];
    int16_t nm;
    uint32_t m[MCAP];
} st_t;

#define HDR_BYTES (offsetof(st_t, m))

/* ------------------------------------------------------------------ messages */
static inline uint32_t k_vresp(int src, int dst, int term) {
    return (0u << 30) | ((uint32_t)dst << 27) | ((uint32_t)src << 24) | ((uint32_t)term << 21);
}
static inline uint32_t k_vreq(int src, int dst, int term, int lli, int llt) {
    return (1u << 30) | ((uint32_t)dst << 27) | ((uint32_t)lli << 23) | ((uint32_t)llt << 20) |
           ((uint32_t)src << 17) | ((uint32_t)term << 14);
}
static inline uint32_t k_aresp(int src, int dst, int term, int pli, int succ) {
    return (1u << 30) | ((uint32_t)dst << 27) | (1u << 26) | ((uint32_t)pli << 23) | ((uint32_t)src << 20) |
           ((uint32_t)succ << 19) | ((uint32_t)term << 16);
}
static inline uint32_t k_areq(int src, int dst, int term, int pli, int plt, int elen, int et, int ev, int lc) {
    return (2u << 30) | ((uint32_t)dst << 27) | ((uint32_t)elen << 26) | ((uint32_t)et << 23) |
           ((uint32_t)ev << 21) | ((uint32_t)lc << 18) | ((uint32_t)pli << 15) | ((uint32_t)plt << 12) |
           ((uint32_t)src << 9) | ((uint32_t)term << 6);
}

typedef struct {
    int type, src, dst, term;
    int lli, llt;               /* VoteReq */
    int pli, plt, lc, elen, et, ev; /* AppendReq (pli also AppendResp) */
    int succ;                   /* AppendResp */
} msg_t;

static void k_decode(uint32_t k, msg_t *m) {
    memset(m, 0, sizeof *m);
    uint32_t cls = k >> 30;
    m->dst = (k >> 27) & 7;
    if (cls == 0) {
        m->type = MT_VRESP; m->src = (k >> 24) & 7; m->term = (k >> 21) & 7;
    } else if (cls == 1 && !((k >> 26) & 1)) {
        m->type = MT_VREQ; m->lli = (k >> 23) & 7; m->llt = (k >> 20) & 7; m->src = (k >> 17) & 7; m->term = (k >> 14) & 7;
    } else if (cls == 1) {
        m->type = MT_ARESP; m->pli = (k >> 23) & 7; m->src = (k >> 20) & 7; m->succ = (k >> 19) & 1; m->term = (k >> 16) & 7;
    } else {
        m->type = MT_AREQ; m->elen = (k >> 26) & 1; m->et = (k >> 23) & 7; m->ev = (k >> 21) & 3;
        m->lc = (k >> 18) & 7; m->pli = (k >> 15) & 7; m->plt = (k >> 12) & 7; m->src = (k >> 9) & 7; m->term = (k >> 6) & 7;
    }
}

static uint32_t k_encode(const msg_t *m) {
    switch (m->type) {
    case MT_VRESP: return k_vresp(m->src, m->dst, m->term);
    case MT_VREQ: return k_vreq(m->src, m->dst, m->term, m->lli, m->llt);
    case MT_ARESP: return k_aresp(m->src, m->dst, m->term, m->pli, m->succ);
    default: return k_areq(m->src, m->dst, m->term, m->pli, m->plt, m->elen, m->et, m->ev, m->lc);
    }
}

static uint32_t k_permute(uint32_t k, const int *pi) {
    msg_t m; k_decode(k, &m);
    m.src = pi[m.src]; m.dst = pi[m.dst];
    return k_encode(&m);
}

static int has_msg(const st_t *s, uint32_t k) {
    int lo = 0, hi = s->nm;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (s->m[mid] < k) lo = mid + 1; else hi = mid;
    }
    return lo < s->nm && s->m[lo] == k;
}

static int g_overflow = 0;

/* SendMsg (tla:43): msgs' = msgs \cup {m} */
static void add_msg(st_t *s, uint32_t k) {
    int lo = 0, hi = s->nm;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (s->m[mid] < k) lo = mid + 1; else hi = mid;
    }
    if (lo < s->nm && s->m[lo] == k) return;
    if (s->nm >= MCAP) { g_overflow = 1; return; }
    memmove(&s->m[lo + 1], &s->m[lo], (size_t)(s->nm - lo) * sizeof(uint32_t));
    s->m[lo] = k;
    s->nm++;
}

/* ------------------------------------------------------------------ state */
static void init_state(const ocfg_t *c, st_t *s) { /* Init tla:93-105 */
    memset(s, 0, sizeof *s);
    for (int i = 0; i < c->n; i++) {
        s->vf[i] = -1; s->ct[i] = 0; s->role[i] = R_F; s->ci[i] = 1; s->ll[i] = 1;
        s->lt[i][1] = 0; s->lv[i][1] = -1;
        for (int j = 0; j < c->n; j++) { s->mi[i][j] = 1; s->ni[i][j] = 2; s->pend[i][j] = 0; }
    }
    for (int v = 0; v < c->V; v++) s->vs[v] = -1;
}

static inline void copy_state(st_t *d, const st_t *s) {
    memcpy(d, s, HDR_BYTES + (size_t)s->nm * sizeof(uint32_t));
}

/* ------------------------------------------------------------------ successor emission */
typedef struct {
    st_t *buf;
    int32_t *w;   /* witness per successor */
    int n, cap;
    int assert_fail;
} batch_t;

static st_t *emit(batch_t *b, int w) {
    if (b->n >= b->cap) { fprintf(stderr, "oracle: batch overflow\n"); exit(3); }
    b->w[b->n] = w;
    return &b->buf[b->n++];
}

static int median(const ocfg_t *c, const int8_t *F) { /* Median tla:70-75 */
    int k = c->seeded ? c->n : (c->n / 2 + 1);
    int best = 127;
    for (int s = 0; s < c->n; s++) {
        int cnt = 0;
        for (int p = 0; p < c->n; p++) cnt += F[p] <= F[s];
        if (cnt >= k && F[s] < best) best = F[s];
    }
    return best;
}

static void gen_action(const ocfg_t *c, const st_t *st, int s, int a, batch_t *b) {
    int n = c->n;
    switch (a) {
    case A_BC: { /* BecomeCandidate tla:107-130 */
        if (!(st->ec < c->E)) return;
        if (!(st->role[s] == R_F || st->role[s] == R_C)) return;
        st_t *t = emit(b, 0); copy_state(t, st);
        int lli = st->ll[s], llt = st->lt[s][lli], term = st->ct[s] + 1;
        t->ec++; t->ct[s] = term; t->role[s] = R_C; t->vf[s] = s;
        for (int p = 0; p < n; p++) if (p != s) add_msg(t, k_vreq(s, p, term, lli, llt));
        return;
    }
    case A_UT: /* UpdateTerm tla:175-188 */
        for (int w = 0; w < st->nm; w++) {
            msg_t m; k_decode(st->m[w], &m);
            if (m.dst != s) continue;
            if (m.term > st->ct[s]) {
                st_t *t = emit(b, w); copy_state(t, st);
                t->role[s] = R_F; t->ct[s] = m.term; t->vf[s] = -1;
            } else if (m.term == st->ct[s] && m.type == MT_AREQ) {
                if (st->role[s] == R_L) { b->assert_fail = 1; b->n = 0; return; } /* Assert tla:185 */
                if (st->role[s] == R_C) {
                    st_t *t = emit(b, w); copy_state(t, st);
                    t->role[s] = R_F;
                }
            }
        }
        return;
    case A_BF: /* BecomeFollower tla:190-231 = FollowerUpdateTerm \/ CandidateToFollower \/
                  LeaderToFollower: role[s] enables exactly one, each over msgs in order */
        for (int w = 0; w < st->nm; w++) {
            msg_t m; k_decode(st->m[w], &m);
            if (m.dst != s) continue;
            if (st->role[s] == R_F) {        /* FollowerUpdateTerm tla:191-197: votedFor kept */
                if (m.term > st->ct[s]) { st_t *t = emit(b, w); copy_state(t, st); t->ct[s] = m.term; }
            } else if (st->role[s] == R_C) { /* CandidateToFollower tla:200-212 */
                if (m.term > st->ct[s]) {
                    st_t *t = emit(b, w); copy_state(t, st);
                    t->ct[s] = m.term; t->role[s] = R_F; t->vf[s] = -1;
                } else if (m.term == st->ct[s] && m.type == MT_AREQ) {
                    st_t *t = emit(b, w); copy_state(t, st);
                    t->role[s] = R_F;
                }
            } else if (m.term > st->ct[s]) { /* LeaderToFollower tla:215-223 */
                st_t *t = emit(b, w); copy_state(t, st);
                t->ct[s] = m.term; t->role[s] = R_F; t->vf[s] = -1;
            }
        }
        return;
    case A_RV: /* ResponseVote tla:132-155 */
        if (st->role[s] != R_F) return;
        for (int w = 0; w < st->nm; w++) {
            msg_t m; k_decode(st->m[w], &m);
            if (m.dst != s || m.type != MT_VREQ || m.term != st->ct[s]) continue;
            if (!(st->vf[s] == -1 || st->vf[s] == m.src)) continue;
            int lli = st->ll[s], llt = st->lt[s][lli];
            if (!(m.llt > llt || (m.llt == llt && m.lli >= lli))) continue;
            uint32_t g = k_vresp(s, m.src, m.term);
            if (has_msg(st, g)) continue;
            st_t *t = emit(b, w); copy_state(t, st);
            add_msg(t, g); t->vf[s] = (int8_t)m.src;
        }
        return;
    case A_BL: { /* BecomeLeader tla:157-173 */
        if (st->role[s] != R_C) return;
        int cnt = 0;
        for (int w = 0; w < st->nm; w++) {
            msg_t m; k_decode(st->m[w], &m);
            cnt += (m.dst == s && m.term == st->ct[s] && m.type == MT_VRESP);
        }
        if (!(cnt + 1 >= (c->sb ? 1 : n / 2 + 1))) return;
        st_t *t = emit(b, 0); copy_state(t, st);
        int L = st->ll[s];
        t->role[s] = R_L;
        for (int u = 0; u < n; u++) { t->mi[s][u] = (u != s) ? 1 : L; t->ni[s][u] = L + 1; t->pend[s][u] = 0; }
        return;
    }
    case A_CR: /* ClientReq tla:233-240 */
        if (st->role[s] != R_L) return;
        for (int v = 0; v < c->V; v++) {
            if (st->vs[v] != -1) continue;
            st_t *t = emit(b, v); copy_state(t, st);
            int L = st->ll[s];
            t->vs[v] = 0;
            t->ll[s] = L + 1; t->lt[s][L + 1] = st->ct[s]; t->lv[s][L + 1] = (int8_t)v;
            t->mi[s][s] = L + 1;
        }
        return;
    case A_LAE: /* LeaderAppendEntry tla:242-269 */
        if (st->role[s] != R_L) return;
        for (int d = 0; d < n; d++) {
            if (d == s) continue;
            int ni = st->ni[s][d], L = st->ll[s];
            if (!(ni <= L + 1)) continue;
            if (st->pend[s][d]) continue;
            int pli = ni - 1, plt = st->lt[s][pli];
            int elen = ni <= L, et = elen ? st->lt[s][ni] : 0, ev = elen ? st->lv[s][ni] : 0;
            uint32_t k = k_areq(s, d, st->ct[s], pli, plt, elen, et, ev, st->ci[s]);
            if (has_msg(st, k)) continue;
            st_t *t = emit(b, d); copy_state(t, st);
            t->pend[s][d] = 1; add_msg(t, k);
        }
        return;
    case A_FAE: /* FollowerAcceptEntry tla:275-300 */
    case A_FRE: /* FollowerRejectEntry tla:302-321 */
        if (st->role[s] != R_F) return;
        for (int w = 0; w < st->nm; w++) {
            msg_t m; k_decode(st->m[w], &m);
            if (m.dst != s || m.term != st->ct[s] || m.type != MT_AREQ) continue;
            int L = st->ll[s];
            int match = m.pli <= L && m.plt == st->lt[s][m.pli]; /* LogMatch tla:271-273 */
            if (a == A_FAE) {
                if (!match) continue;
                int nl = m.pli + m.elen;
                int append_new = nl > L;
                int truncated = 0;
                if (nl <= L) {
                    /* newLog # SubSeq(logs[s], 1, Len(newLog)): only the entry can differ */
                    if (m.elen && (st->lt[s][nl] != m.et || st->lv[s][nl] != m.ev)) truncated = 1;
                }
                int mn = (c->cpl || m.lc < nl) ? m.lc : nl;
                int nci = st->ci[s] > mn ? st->ci[s] : mn;
                st_t *t = emit(b, w); copy_state(t, st);
                add_msg(t, k_aresp(s, m.src, m.term, m.pli + m.elen, 1));
                t->ci[s] = (int8_t)nci;
                if (truncated || append_new) {
                    t->ll[s] = (int8_t)nl;
                    if (m.elen) { t->lt[s][nl] = (int8_t)m.et; t->lv[s][nl] = (int8_t)m.ev; }
                    for (int i = nl + 1; i < MAXL; i++) { t->lt[s][i] = 0; t->lv[s][i] = 0; }
                }
            } else {
                if (match) continue;
                uint32_t k = k_aresp(s, m.src, m.term, m.pli, 0);
                if (has_msg(st, k)) continue;
                st_t *t = emit(b, w); copy_state(t, st);
                add_msg(t, k);
            }
        }
        return;
    case A_HAR: /* HandleAppendResp tla:374-396 */
        if (st->role[s] != R_L) return;
        for (int w = 0; w < st->nm; w++) {
            msg_t m; k_decode(st->m[w], &m);
            if (m.type != MT_ARESP || m.dst != s || m.term != st->ct[s]) continue;
            if (!st->pend[s][m.src]) continue;
            if (m.succ) {
                if (!(st->mi[s][m.src] < m.pli)) continue;
                st_t *t = emit(b, w); copy_state(t, st);
                t->mi[s][m.src] = (int8_t)m.pli; t->ni[s][m.src] = (int8_t)(m.pli + 1); t->pend[s][m.src] = 0;
            } else {
                if (!(m.pli + 1 == st->ni[s][m.src])) continue;
                if (!(m.pli > st->mi[s][m.src])) continue;
                st_t *t = emit(b, w); copy_state(t, st);
                t->pend[s][m.src] = 0; t->ni[s][m.src] = (int8_t)m.pli;
            }
        }
        return;
    case A_LCC: { /* LeaderCanCommit tla:398-407 */
        if (st->role[s] != R_L) return;
        int med = median(c, st->mi[s]);
        if (!(med > st->ci[s])) return;
        st_t *t = emit(b, 0); copy_state(t, st);
        t->ci[s] = (int8_t)med;
        return;
    }
    case A_RS: /* Restart tla:409-414 */
        if (st->role[s] != R_L || !(st->rc < c->R)) return;
        {
            st_t *t = emit(b, 0); copy_state(t, st);
            t->role[s] = R_F; t->rc++;
        }
        return;
    }
}

/* ------------------------------------------------------------------ invariants */
/* returns 1 TRUE, 0 FALSE, -1 TLC evaluation error */
static int inv_lhace(const ocfg_t *c, const st_t *st) { /* LeaderHasAllCommittedEntries tla:491-499 */
    int n = c->n, any = 0;
    for (int p = 0; p < n; p++) any |= st->role[p] == R_L;
    if (!any) return 1;
    for (int l = 0; l < n; l++) {
        if (st->role[l] != R_L) continue;
        int found_bad = 0;
        for (int p = 0; p < n && !found_bad; p++) {
            if (p == l) continue;
            if (!(st->ct[p] <= st->ct[l])) continue;
            if (st->ci[p] > st->ll[l]) { found_bad = 1; break; }
            for (int i = 1; i <= st->ci[p]; i++) {
                if (i > st->ll[p]) return -1; /* logs[p][index] out of domain */
                if (st->lt[p][i] != st->lt[l][i] || st->lv[p][i] != st->lv[l][i]) { found_bad = 1; break; }
            }
        }
        if (!found_bad) return 1;
    }
    return 0;
}

static int inv_eval(const ocfg_t *c, const st_t *st, int id) {
    int n = c->n;
    switch (id) {
    case I_LHACE: return inv_lhace(c, st);
    case I_NOSPLIT: /* tla:444-448 */
        for (int a = 0; a < n; a++) for (int b = 0; b < n; b++)
            if (a != b && st->ct[a] == st->ct[b] && st->role[a] == R_L && st->role[b] == R_L) return 0;
        return 1;
    case I_RAFTCANCOMMIT: /* tla:434 */
        for (int s = 0; s < n; s++) if (st->ci[s] > 1) return 1;
        return 0;
    case I_FOLLOWERCANCOMMIT: /* tla:436-439 */
        for (int s = 0; s < n; s++) if (st->role[s] == R_F && st->ci[s] > 1) return 1;
        return 0;
    case I_COMMITALL: /* tla:442 */
        for (int s = 0; s < n; s++) if (st->ci[s] != 3) return 0;
        return 1;
    case I_EXISTLC: /* tla:483-487 */
        for (int a = 0; a < n; a++) for (int b = 0; b < n; b++)
            if (a != b && st->role[a] == R_L && st->role[b] == R_C) return 1;
        return 0;
    case I_NOALLCOMMIT: /* tla:451-481 */
        for (int s1 = 0; s1 < n; s1++) for (int s2 = 0; s2 < n; s2++) for (int s3 = 0; s3 < n; s3++) {
            if (!(s1 != s2 && s2 != s3 && st->role[s1] == R_L && st->role[s2] == R_F && st->role[s3] == R_F &&
                  st->ct[s1] == st->ct[s3] && st->ci[s1] == 2 && st->ci[s2] == 2 && st->ci[s3] == 1 &&
                  st->mi[s1][s2] == 2 && st->mi[s1][s3] == 2)) continue;
            int c1 = 0, c2 = 0, c3 = 0;
            for (int w = 0; w < st->nm; w++) {
                msg_t m; k_decode(st->m[w], &m);
                c1 |= m.dst == s3 && m.src == s1 && m.term == st->ct[s3] && m.type == MT_AREQ && m.pli == 1;
                c2 |= m.dst == s1 && m.src == s3 && m.term == st->ct[s3] && m.type == MT_ARESP && m.pli == 1 && m.succ;
                c3 |= m.dst == s3 && m.src == s1 && m.type == MT_AREQ && m.pli == 2;
            }
            if (c1 && c2 && c3) return 1;
        }
        return 0;
    }
    return 1;
}

/* ------------------------------------------------------------------ canonical form */
typedef struct { int np; int pi[120][MAXN]; int inv[120][MAXN]; } perms_t;

static void make_perms(int n, perms_t *P) {
    int a[MAXN];
    for (int i = 0; i < n; i++) a[i] = i;
    P->np = 0;
    for (;;) { /* lexicographic permutation enumeration */
        memcpy(P->pi[P->np], a, sizeof a);
        for (int i = 0; i < n; i++) P->inv[P->np][a[i]] = i;
        P->np++;
        int i = n - 2;
        while (i >= 0 && a[i] > a[i + 1]) i--;
        if (i < 0) break;
        int j = n - 1;
        while (a[j] < a[i]) j--;
        int t = a[i]; a[i] = a[j]; a[j] = t;
        for (int l = i + 1, r = n - 1; l < r; l++, r--) { t = a[l]; a[l] = a[r]; a[r] = t; }
    }
}

static int cmp_u32(const void *a, const void *b) {
    uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    return x < y ? -1 : x > y;
}

/* serialise pi(view(st)) (tla:38) into buf; returns length in bytes */
static int view_bytes(const ocfg_t *c, const st_t *st, const int *pi, const int *inv, uint8_t *buf) {
    int n = c->n, V = c->V, o = 0;
    for (int k = 0; k < n; k++) {
        int i = inv[k];
        buf[o++] = (uint8_t)(st->vf[i] < 0 ? 0xff : pi[st->vf[i]]);
        buf[o++] = (uint8_t)st->ct[i];
        buf[o++] = (uint8_t)st->ll[i];
        for (int x = 2; x <= V + 1; x++) {
            int in = x <= st->ll[i];
            buf[o++] = (uint8_t)(in ? st->lt[i][x] : 0);
            buf[o++] = (uint8_t)(in ? st->lv[i][x] : 0);
        }
        for (int l = 0; l < n; l++) buf[o++] = (uint8_t)st->mi[i][inv[l]];
        for (int l = 0; l < n; l++) buf[o++] = (uint8_t)st->ni[i][inv[l]];
        buf[o++] = (uint8_t)st->ci[i];
        buf[o++] = (uint8_t)st->role[i];
    }
    buf[o++] = (uint8_t)(st->nm & 0xff);
    buf[o++] = (uint8_t)(st->nm >> 8);
    uint32_t tmp[MCAP];
    for (int w = 0; w < st->nm; w++) tmp[w] = k_permute(st->m[w], pi);
    qsort(tmp, (size_t)st->nm, sizeof(uint32_t), cmp_u32);
    for (int w = 0; w < st->nm; w++) {
        buf[o++] = (uint8_t)(tmp[w] >> 24); buf[o++] = (uint8_t)(tmp[w] >> 16);
        buf[o++] = (uint8_t)(tmp[w] >> 8); buf[o++] = (uint8_t)tmp[w];
    }
    return o;
}

static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

static void hash128(const uint8_t *b, int len, uint64_t out[2]) {
    uint64_t h1 = 0x243f6a8885a308d3ULL ^ (uint64_t)len, h2 = 0x13198a2e03707344ULL + (uint64_t)len;
    for (int i = 0; i < len; i += 8) {
        uint64_t w = 0;
        for (int j = 0; j < 8 && i + j < len; j++) w |= (uint64_t)b[i + j] << (8 * j);
        h1 = mix64(h1 ^ w) + 0x9e3779b97f4a7c15ULL;
        h2 = mix64(h2 + w * 0xff51afd7ed558ccdULL) ^ 0xc4ceb9fe1a85ec53ULL;
    }
    out[0] = mix64(h1 ^ (h2 >> 7));
    out[1] = mix64(h2 ^ (h1 << 3));
}

#define VBUF (MAXN * (5 + 2 * MAXV + 2 * MAXN) + 2 + 4 * MCAP)

static void canon_hash(const ocfg_t *c, const perms_t *P, const st_t *st, uint64_t out[2]) {
    uint8_t best[VBUF], cur[VBUF];
    int bl = view_bytes(c, st, P->pi[0], P->inv[0], best);
    for (int p = 1; p < P->np; p++) {
        int l = view_bytes(c, st, P->pi[p], P->inv[p], cur);
        /* same length for all perms (same |msgs|) */
        if (memcmp(cur, best, (size_t)l) < 0) memcpy(best, cur, (size_t)l);
    }
    hash128(best, bl, out);
}

/* ------------------------------------------------------------------ seen set */
typedef struct { uint64_t *k; uint64_t cap, cnt; } fpset_t;

static void fps_init(fpset_t *S, uint64_t cap) {
    S->cap = cap; S->cnt = 0;
    S->k = (uint64_t *)calloc(cap * 2, sizeof(uint64_t));
    if (!S->k) { fprintf(stderr, "oracle: OOM fpset\n"); exit(3); }
}

static int fps_put_raw(uint64_t *K, uint64_t cap, const uint64_t h[2]) {
    uint64_t lo = h[0] | 1, hi = h[1];
    uint64_t i = (hi ^ (hi >> 29)) & (cap - 1);
    for (;;) {
        if (K[2 * i] == 0) { K[2 * i] = lo; K[2 * i + 1] = hi; return 1; }
        if (K[2 * i] == lo && K[2 * i + 1] == hi) return 0;
        i = (i + 1) & (cap - 1);
    }
}

/* returns 1 if new */
static int fps_put(fpset_t *S, const uint64_t h[2]) {
    if ((S->cnt + 1) * 2 > S->cap) {
        uint64_t nc = S->cap * 2;
        uint64_t *nk = (uint64_t *)calloc(nc * 2, sizeof(uint64_t));
        if (!nk) { fprintf(stderr, "oracle: OOM fpset grow\n"); exit(3); }
        for (uint64_t i = 0; i < S->cap; i++)
            if (S->k[2 * i]) { uint64_t hh[2] = {S->k[2 * i], S->k[2 * i + 1]}; fps_put_raw(nk, nc, hh); }
        free(S->k); S->k = nk; S->cap = nc;
    }
    int r = fps_put_raw(S->k, S->cap, h);
    S->cnt += r;
    return r;
}

/* ------------------------------------------------------------------ compact state arena */
typedef struct { uint8_t *b; size_t len, cap; uint64_t *off; uint64_t n, ocap; } arena_t;

static void ar_push(arena_t *A, const st_t *s) {
    size_t sz = HDR_BYTES + (size_t)s->nm * 4;
    if (A->len + sz > A->cap) {
        A->cap = (A->cap ? A->cap * 2 : (1 << 20)) + sz;
        A->b = (uint8_t *)realloc(A->b, A->cap);
        if (!A->b) { fprintf(stderr, "oracle: OOM arena\n"); exit(3); }
    }
    if (A->n == A->ocap) {
        A->ocap = A->ocap ? A->ocap * 2 : 1024;
        A->off = (uint64_t *)realloc(A->off, A->ocap * sizeof(uint64_t));
    }
    A->off[A->n++] = A->len;
    memcpy(A->b + A->len, s, sz);
    A->len += sz;
}

static void ar_get(const arena_t *A, uint64_t i, st_t *s) {
    const uint8_t *p = A->b + A->off[i];
    memcpy(s, p, HDR_BYTES);
    memcpy(s->m, p + HDR_BYTES, (size_t)s->nm * 4);
}

static void ar_clear(arena_t *A) { A->len = 0; A->n = 0; }
static void ar_free(arena_t *A) { free(A->b); free(A->off); memset(A, 0, sizeof *A); }

/* ------------------------------------------------------------------ unpacked interchange */
/* Layout (int32), documented in include/rmc.h as RMC unpacked state:
 *   votedFor[n] currentTerm[n] role[n] commitIndex[n] logLen[n]
 *   logs[n][V+1][2] (term,val; entry 1 = (0,-1); unused = 0)
 *   matchIndex[n][n] nextIndex[n][n] pendingResponse[n][n]
 *   electionCount restartCount valSent[V] nmsgs msgs[nmsgs][8]
 * message record: type(0 VoteReq,1 VoteResp,2 AppendReq,3 AppendResp) src dst term x1 x2 x3 x4
 *   VoteReq x1=lastLogIndex x2=lastLogTerm; AppendResp x1=prevLogIndex x2=succ;
 *   AppendReq x1=prevLogIndex x2=prevLogTerm x3=leaderCommit x4=entry (-1 none, else term*8+val)
 */
int orc_unpacked_ints(int n, int V, int cap) { return 5 * n + n * (V + 1) * 2 + 3 * n * n + 3 + V + 8 * cap; }

static int unpack_to(const ocfg_t *c, const st_t *s, int32_t *o, int cap_ints) {
    int n = c->n, V = c->V, k = 0;
    int need = orc_unpacked_ints(n, V, s->nm);
    if (need > cap_ints) return -need;
    for (int i = 0; i < n; i++) o[k++] = s->vf[i];
    for (int i = 0; i < n; i++) o[k++] = s->ct[i];
    for (int i = 0; i < n; i++) o[k++] = s->role[i];
    for (int i = 0; i < n; i++) o[k++] = s->ci[i];
    for (int i = 0; i < n; i++) o[k++] = s->ll[i];
    for (int i = 0; i < n; i++)
        for (int x = 1; x <= V + 1; x++) {
            int in = x <= s->ll[i];
            o[k++] = in ? s->lt[i][x] : 0;
            o[k++] = in ? s->lv[i][x] : 0;
        }
    for (int i = 0; i < n; i++) for (int j = 0; j < n; j++) o[k++] = s->mi[i][j];
    for (int i = 0; i < n; i++) for (int j = 0; j < n; j++) o[k++] = s->ni[i][j];
    for (int i = 0; i < n; i++) for (int j = 0; j < n; j++) o[k++] = s->pend[i][j];
    o[k++] = s->ec; o[k++] = s->rc;
    for (int v = 0; v < V; v++) o[k++] = s->vs[v];
    o[k++] = s->nm;
    for (int w = 0; w < s->nm; w++) {
        msg_t m; k_decode(s->m[w], &m);
        o[k++] = m.type; o[k++] = m.src; o[k++] = m.dst; o[k++] = m.term;
        switch (m.type) {
        case MT_VREQ: o[k++] = m.lli; o[k++] = m.llt; o[k++] = 0; o[k++] = 0; break;
        case MT_VRESP: o[k++] = 0; o[k++] = 0; o[k++] = 0; o[k++] = 0; break;
        case MT_ARESP: o[k++] = m.pli; o[k++] = m.succ; o[k++] = 0; o[k++] = 0; break;
        default: o[k++] = m.pli; o[k++] = m.plt; o[k++] = m.lc; o[k++] = m.elen ? m.et * 8 + m.ev : -1; break;
        }
    }
    return k;
}

static int pack_from(const ocfg_t *c, const int32_t *o, st_t *s) {
    int n = c->n, V = c->V, k = 0;
    memset(s, 0, sizeof *s);
    for (int i = 0; i < n; i++) s->vf[i] = (int8_t)o[k++];
    for (int i = 0; i < n; i++) s->ct[i] = (int8_t)o[k++];
    for (int i = 0; i < n; i++) s->role[i] = (int8_t)o[k++];
    for (int i = 0; i < n; i++) s->ci[i] = (int8_t)o[k++];
    for (int i = 0; i < n; i++) s->ll[i] = (int8_t)o[k++];
    for (int i = 0; i < n; i++)
        for (int x = 1; x <= V + 1; x++) { s->lt[i][x] = (int8_t)o[k++]; s->lv[i][x] = (int8_t)o[k++]; }
    for (int i = 0; i < n; i++) { s->lt[i][1] = 0; s->lv[i][1] = -1; }
    for (int i = 0; i < n; i++) for (int j = 0; j < n; j++) s->mi[i][j] = (int8_t)o[k++];
    for (int i = 0; i < n; i++) for (int j = 0; j < n; j++) s->ni[i][j] = (int8_t)o[k++];
    for (int i = 0; i < n; i++) for (int j = 0; j < n; j++) s->pend[i][j] = (uint8_t)o[k++];
    s->ec = (int8_t)o[k++]; s->rc = (int8_t)o[k++];
    for (int v = 0; v < V; v++) s->vs[v] = (int8_t)o[k++];
    int nm = o[k++];
    if (nm > MCAP) return -1;
    s->nm = 0;
    for (int w = 0; w < nm; w++) {
        msg_t m; memset(&m, 0, sizeof m);
        m.type = o[k]; m.src = o[k + 1]; m.dst = o[k + 2]; m.term = o[k + 3];
        switch (m.type) {
        case MT_VREQ: m.lli = o[k + 4]; m.llt = o[k + 5]; break;
        case MT_ARESP: m.pli = o[k + 4]; m.succ = o[k + 5]; break;
        case MT_AREQ: m.pli = o[k + 4]; m.plt = o[k + 5]; m.lc = o[k + 6];
            if (o[k + 7] >= 0) { m.elen = 1; m.et = o[k + 7] / 8; m.ev = o[k + 7] % 8; }
            break;
        default: break;
        }
        k += 8;
        add_msg(s, k_encode(&m));
    }
    return k;
}

/* ------------------------------------------------------------------ BFS driver */
typedef struct {
    ocfg_t c;
    perms_t P;
    int verdict;
    int violated_inv;
    uint64_t generated, distinct, queue_left;
    int depth;
    uint64_t lvl_distinct[MAXLEVELS], lvl_generated[MAXLEVELS];
    int max_nm;
    /* trace bookkeeping */
    uint64_t *parent; uint32_t *key; uint64_t tcap;
    arena_t all; /* when record_trace: every state, to print traces */
    uint64_t err_state; int err_is_parent;
    double seconds;
} orc_t;

static void rec_state(orc_t *O, uint64_t id, uint64_t parent, uint32_t key, const st_t *s) {
    if (!O->c.record_trace) return;
    if (id >= O->tcap) {
        O->tcap = O->tcap ? O->tcap * 2 : 4096;
        O->parent = (uint64_t *)realloc(O->parent, O->tcap * sizeof(uint64_t));
        O->key = (uint32_t *)realloc(O->key, O->tcap * sizeof(uint32_t));
    }
    O->parent[id] = parent; O->key[id] = key;
    ar_push(&O->all, s);
}

void *orc_create(int n, int V, int E, int R, int seeded, int check_deadlock, uint32_t inv_mask, int record_trace) {
    if (n < 1 || n > MAXN || V < 0 || V > MAXV || E < 0 || E > 7 || R < 0) return NULL;
    orc_t *O = (orc_t *)calloc(1, sizeof(orc_t));
    O->c.n = n; O->c.V = V; O->c.E = E; O->c.R = R;
    set_variant(&O->c, seeded);
    O->c.check_deadlock = check_deadlock; O->c.inv_mask = inv_mask; O->c.record_trace = record_trace;
    make_perms(n, &O->P);
    return O;
}

void orc_set_order(void *h, int order, uint64_t seed) {
    orc_t *O = (orc_t *)h;
    O->c.order = order;
    O->c.seed = seed;
}

void orc_destroy(void *h) {
    orc_t *O = (orc_t *)h;
    if (!O) return;
    free(O->parent); free(O->key); ar_free(&O->all);
    free(O);
}

static int check_invs(orc_t *O, const st_t *s, int *which) {
    for (int i = 0; i < N_INV; i++) {
        if (!(O->c.inv_mask & (1u << i))) continue;
        int r = inv_eval(&O->c, s, i);
        if (r < 0) { *which = i; return V_EVAL_ERROR; }
        if (r == 0) { *which = i; return V_INVARIANT; }
    }
    return V_OK;
}

#define BATCH_CAP 512

int orc_run(void *h, uint64_t max_states) {
    orc_t *O = (orc_t *)h;
    const ocfg_t *c = &O->c;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    arena_t cur = {0}, nxt = {0};
    fpset_t S; fps_init(&S, 1u << 20);
    st_t *s0 = (st_t *)malloc(sizeof(st_t));
    st_t *ps = (st_t *)malloc(sizeof(st_t));
    batch_t b; b.buf = (st_t *)malloc(sizeof(st_t) * BATCH_CAP); b.w = (int32_t *)malloc(sizeof(int32_t) * BATCH_CAP); b.cap = BATCH_CAP;
    init_state(c, s0);
    uint64_t h2[2];
    canon_hash(c, &O->P, s0, h2);
    fps_put(&S, h2);
    O->generated = 1; O->distinct = 1; O->depth = 1;
    O->lvl_distinct[0] = 1;
    rec_state(O, 0, UINT64_MAX, 0, s0);
    O->verdict = V_OK;
    int which = -1;
    int v = check_invs(O, s0, &which);
    if (v != V_OK) { O->verdict = v; O->violated_inv = which; O->err_state = 0; goto done; }
    ar_push(&cur, s0);
    uint64_t cur_base = 0; /* global id of cur[0] */
    for (int lvl = 1; cur.n > 0; lvl++) {
        if (lvl >= MAXLEVELS) { O->verdict = V_CAPACITY; goto done; }
        uint64_t nxt_base = O->distinct;
        uint64_t *perm = NULL;
        if (c->order) {  /* order-sensitivity probe: visit this level's states in another order */
            perm = (uint64_t *)malloc(cur.n * sizeof(uint64_t));
            for (uint64_t i = 0; i < cur.n; i++) perm[i] = c->order == 1 ? cur.n - 1 - i : i;
            if (c->order == 2) {
                uint64_t x = c->seed + (uint64_t)lvl * 0x9e3779b97f4a7c15ULL;
                for (uint64_t i = cur.n; i > 1; i--) {
                    x = mix64(x + 0x9e3779b97f4a7c15ULL);
                    uint64_t j = x % i, t = perm[i - 1]; perm[i - 1] = perm[j]; perm[j] = t;
                }
            }
        }
        for (uint64_t i = 0; i < cur.n; i++) {
            ar_get(&cur, perm ? perm[i] : i, ps);
            if (ps->nm > O->max_nm) O->max_nm = ps->nm;
            int nsucc = 0;
            for (int s = 0; s < c->n; s++) {
                for (int ai = 0; ai < N_ORDER; ai++) {
                    const int a = ACT_ORDER[ai];
                    if (a == A_BF && !c->bf) continue;
                    b.n = 0; b.assert_fail = 0;
                    gen_action(c, ps, s, a, &b);
                    if (g_overflow) { O->verdict = V_CAPACITY; goto done; }
                    if (b.assert_fail) {
                        O->verdict = V_ASSERT; O->err_state = cur_base + i; O->err_is_parent = 1;
                        O->queue_left = (cur.n - i - 1) + nxt.n;
                        goto done;
                    }
                    O->generated += (uint64_t)b.n;
                    O->lvl_generated[lvl - 1] += (uint64_t)b.n;
                    nsucc += b.n;
                    for (int jj = 0; jj < b.n; jj++) {
                        const int j = c->order == 1 ? b.n - 1 - jj : jj;
                        st_t *t = &b.buf[j];
                        canon_hash(c, &O->P, t, h2);
                        if (!fps_put(&S, h2)) continue;
                        uint64_t id = O->distinct++;
                        O->lvl_distinct[lvl]++;
                        if (lvl + 1 > O->depth) O->depth = lvl + 1;
                        uint32_t key = ((uint32_t)s << 24) | ((uint32_t)a << 16) | (uint32_t)b.w[j];
                        rec_state(O, id, cur_base + i, key, t);
                        v = check_invs(O, t, &which);
                        if (v != V_OK) {
                            O->verdict = v; O->violated_inv = which; O->err_state = id;
                            O->queue_left = (cur.n - i - 1) + nxt.n;
                            goto done;
                        }
                        ar_push(&nxt, t);
                        if (max_states && O->distinct >= max_states) { O->verdict = V_LIMIT; goto done; }
                    }
                }
            }
            if (nsucc == 0 && c->check_deadlock) {
                O->verdict = V_DEADLOCK; O->err_state = cur_base + i; O->err_is_parent = 1;
                O->queue_left = (cur.n - i - 1) + nxt.n;
                goto done;
            }
        }
        free(perm);
        arena_t tmp = cur; cur = nxt; nxt = tmp; ar_clear(&nxt);
        cur_base = nxt_base;
    }
done:
    clock_gettime(CLOCK_MONOTONIC, &t1);
    O->seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    ar_free(&cur); ar_free(&nxt); free(S.k); free(s0); free(ps); free(b.buf); free(b.w);
    return O->verdict;
}

uint64_t orc_generated(void *h) { return ((orc_t *)h)->generated; }
uint64_t orc_distinct(void *h) { return ((orc_t *)h)->distinct; }
int orc_depth(void *h) { return ((orc_t *)h)->depth; }
int orc_violated(void *h) { return ((orc_t *)h)->violated_inv; }
int orc_max_msgs(void *h) { return ((orc_t *)h)->max_nm; }
double orc_seconds(void *h) { return ((orc_t *)h)->seconds; }
uint64_t orc_queue_left(void *h) { return ((orc_t *)h)->queue_left; }

int orc_levels(void *h, uint64_t *distinct, uint64_t *generated, int cap) {
    orc_t *O = (orc_t *)h;
    int L = O->depth < cap ? O->depth : cap;
    for (int i = 0; i < L; i++) { distinct[i] = O->lvl_distinct[i]; generated[i] = O->lvl_generated[i]; }
    return O->depth;
}

/* trace: states from Init to the error state; key = server<<24 | action<<16 | witness */
int orc_trace_len(void *h) {
    orc_t *O = (orc_t *)h;
    if (!O->c.record_trace || O->verdict == V_OK) return 0;
    int len = 0;
    for (uint64_t i = O->err_state; i != UINT64_MAX; i = O->parent[i]) len++;
    return len;
}

int orc_trace_state(void *h, int idx, int32_t *out, int cap_ints, uint32_t *key) {
    orc_t *O = (orc_t *)h;
    int len = orc_trace_len(h);
    if (idx < 0 || idx >= len) return -1;
    uint64_t i = O->err_state;
    for (int k = len - 1; k > idx; k--) i = O->parent[i];
    st_t *s = (st_t *)malloc(sizeof(st_t));
    ar_get(&O->all, i, s);
    *key = O->key[i];
    int r = unpack_to(&O->c, s, out, cap_ints);
    free(s);
    return r;
}

/* ---- single-state helpers for fixtures ---- */
/* successors of an unpacked state in TLC order; returns count, -1 on Assert, -2 on capacity */
int orc_successors(int n, int V, int E, int R, int seeded, const int32_t *in, int32_t *out, int stride_ints,
                   int cap_states, uint32_t *keys) {
    ocfg_t c = {n, V, E, R, 0, 0, 1, 0, 0, 0, 0, 0, 0};
    set_variant(&c, seeded);
    st_t *st = (st_t *)malloc(sizeof(st_t));
    batch_t b; b.buf = (st_t *)malloc(sizeof(st_t) * BATCH_CAP); b.w = (int32_t *)malloc(sizeof(int32_t) * BATCH_CAP); b.cap = BATCH_CAP;
    int cnt = 0, ret = 0;
    if (pack_from(&c, in, st) < 0) { ret = -2; goto out; }
    for (int s = 0; s < n && ret == 0; s++)
        for (int ai = 0; ai < N_ORDER; ai++) {
            const int a = ACT_ORDER[ai];
            if (a == A_BF && !c.bf) continue;
            b.n = 0; b.assert_fail = 0;
            gen_action(&c, st, s, a, &b);
            if (b.assert_fail) { ret = -1; break; }
            for (int j = 0; j < b.n; j++) {
                if (cnt >= cap_states) { ret = -2; break; }
                if (unpack_to(&c, &b.buf[j], out + (size_t)cnt * stride_ints, stride_ints) < 0) { ret = -2; break; }
                keys[cnt] = ((uint32_t)s << 24) | ((uint32_t)a << 16) | (uint32_t)b.w[j];
                cnt++;
            }
            if (ret) break;
        }
out:
    free(st); free(b.buf); free(b.w);
    return ret ? ret : cnt;
}

/* Replay a path: from the unpacked state `in`, take at each step the successor whose key (as
 * orc_successors) is keys[i]; the final state goes to `out`.  Returns its unpacked length, or
 * -(i + 1) when keys[i] is not enabled (or the Assert fails) at step i, -1000000 on capacity. */
int orc_replay(int n, int V, int E, int R, int seeded, const int32_t *in, const uint32_t *keys, int nkeys,
               int32_t *out, int cap_ints) {
    ocfg_t c = {n, V, E, R, 0, 0, 1, 0, 0, 0, 0, 0, 0};
    set_variant(&c, seeded);
    st_t *st = (st_t *)malloc(sizeof(st_t));
    batch_t b; b.buf = (st_t *)malloc(sizeof(st_t) * BATCH_CAP); b.w = (int32_t *)malloc(sizeof(int32_t) * BATCH_CAP); b.cap = BATCH_CAP;
    int ret = 0;
    if (pack_from(&c, in, st) < 0) { ret = -1000000; goto out; }
    for (int i = 0; i < nkeys && ret == 0; i++) {
        const int s = (int)(keys[i] >> 24), a = (int)((keys[i] >> 16) & 0xFF), w = (int)(keys[i] & 0xFFFF);
        if (s >= n || (a == A_BF && !c.bf)) { ret = -(i + 1); break; }
        b.n = 0; b.assert_fail = 0;
        gen_action(&c, st, s, a, &b);
        int j = 0;
        while (j < b.n && b.w[j] != w) j++;
        if (b.assert_fail || j == b.n) { ret = -(i + 1); break; }
        copy_state(st, &b.buf[j]);
    }
    if (ret == 0) {
        ret = unpack_to(&c, st, out, cap_ints);
        if (ret < 0) ret = -1000000;
    }
out:
    free(st); free(b.buf); free(b.w);
    return ret;
}

int orc_canon_hash(int n, int V, const int32_t *in, uint64_t *out2) {
    ocfg_t c = {n, V, 7, 7, 0, 0, 1, 0, 0, 0, 0, 0, 0};
    perms_t *P = (perms_t *)malloc(sizeof(perms_t));
    make_perms(n, P);
    st_t *st = (st_t *)malloc(sizeof(st_t));
    int r = pack_from(&c, in, st);
    if (r >= 0) canon_hash(&c, P, st, out2);
    free(st); free(P);
    return r < 0 ? -1 : 0;
}

int orc_inv(int n, int V, const int32_t *in, int inv_id) {
    ocfg_t c = {n, V, 7, 7, 0, 0, 1, 0, 0, 0, 0, 0, 0};
    st_t *st = (st_t *)malloc(sizeof(st_t));
    int r = pack_from(&c, in, st);
    if (r >= 0) r = inv_eval(&c, st, inv_id);
    else r = -2;
    free(st);
    return r;
}

#ifdef ORC_MAIN
int main(int argc, char **argv) {
    int n = 3, V = 2, E = 3, R = 3, seeded = 0;
    uint32_t mask = 1;
    int trace = 1, order = 0;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-notrace")) trace = 0;
        else if (!strcmp(argv[i], "-order")) order = atoi(argv[++i]);
        if (!strcmp(argv[i], "-n")) n = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-V")) V = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-E")) E = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-R")) R = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-seeded")) seeded |= 1;
        else if (!strcmp(argv[i], "-bf")) seeded |= 2;
        else if (!strcmp(argv[i], "-inv")) mask = (uint32_t)strtoul(argv[++i], 0, 0);
    }
    void *h = orc_create(n, V, E, R, seeded, 0, mask, trace);
    orc_set_order(h, order, 12345);
    int v = orc_run(h, 0);
    uint64_t d[MAXLEVELS], g[MAXLEVELS];
    int L = orc_levels(h, d, g, MAXLEVELS);
    printf("verdict=%d generated=%llu distinct=%llu depth=%d max_msgs=%d trace_len=%d time=%.2fs (%.0f states/s)\n", v,
           (unsigned long long)orc_generated(h), (unsigned long long)orc_distinct(h), orc_depth(h), orc_max_msgs(h),
           orc_trace_len(h), orc_seconds(h), (double)orc_distinct(h) / orc_seconds(h));
    printf("levels");
    for (int i = 0; i < L; i++) printf(" %llu", (unsigned long long)d[i]);
    printf("\ngen/level");
    for (int i = 0; i < L; i++) printf(" %llu", (unsigned long long)g[i]);
    printf("\n");
    orc_destroy(h);
    return 0;
}
#endif
