/*
 * pg_oracle.c — plain-C restatement of kmer_numba.py's hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see pg_oracle.h).  Every function cites the
 * reference line range it restates; /root/reference/kmer_numba.py is the
 * source of truth and tests/golden/ pins this file to its outputs.
 */
#define _POSIX_C_SOURCE 200809L
#include "pg_oracle.h"

#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ---------------------------------------------------------------- tables */
/* alpha :763-768 — A0 G1 C2 T3 (either case), every other byte 4 */
static uint8_t ALPHA[256];
/* lastc :736-743 — A1 T2 G4 C8 N16 (either case), '$'32, everything else 0 */
static uint8_t LASTC[256];
/* tab_rev_bytes :191-195 — A<->T, G<->C, N->N (either case, to upper), else 'N' */
static uint8_t TABREV[256];
static int tables_ready = 0;

static void init_tables(void) {
    if (tables_ready) return;
    for (int i = 0; i < 256; i++) { ALPHA[i] = 4; LASTC[i] = 0; TABREV[i] = 'N'; }
    const char* fw = "ATGCN"; const char* rv = "TACGN";
    for (int i = 0; i < 5; i++) {
        TABREV[(uint8_t)fw[i]] = (uint8_t)rv[i];
        TABREV[(uint8_t)(fw[i] | 0x20)] = (uint8_t)rv[i];
    }
    const char* al = "AGCT";
    for (int i = 0; i < 4; i++) { ALPHA[(uint8_t)al[i]] = (uint8_t)i; ALPHA[(uint8_t)(al[i] | 0x20)] = (uint8_t)i; }
    const char* lc = "ATGCN";
    for (int i = 0; i < 5; i++) {
        LASTC[(uint8_t)lc[i]] = (uint8_t)(1u << i);
        LASTC[(uint8_t)(lc[i] | 0x20)] = (uint8_t)(1u << i);
    }
    LASTC['$'] = 32; LASTC['#'] = 0;
    tables_ready = 1;
}

#define OFFBIT 6          /* offbit :745 (log2(max lastc)+1) */
#define EDGE_OFFBIT 5     /* :1814 passes `bits`(=5) into rdbg_edge_weight's offbit slot */
#define SENTINEL ((uint64_t)-1)

static double now_s(void) {
    struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* ------------------------------------------------------ record iterator */
/* readline_jit_ :122-132 (with its `offset`) + seqio_jit_ :135-172 (FASTA). */
typedef struct {
    const uint8_t* buf; int64_t n, offset;
    int64_t pos, start; int tail_done, final_done;
    int have_qid; int64_t qid_st, qid_len;         /* qid = line[:-1] (:160)         */
    int pending; int64_t pend_st, pend_len;         /* header seen, record yielded    */
    uint8_t* seq; int64_t seq_len, seq_cap;
    /* the record most recently yielded */
    int64_t r_qid_st, r_qid_len, r_ptr;
} rec_iter;

static void it_init(rec_iter* it, const uint8_t* buf, int64_t n, int64_t offset) {
    memset(it, 0, sizeof(*it));
    it->buf = buf; it->n = n; it->offset = offset;
    it->pos = offset < 0 ? 0 : offset;
    it->seq_cap = 1 << 16; it->seq = (uint8_t*)malloc((size_t)it->seq_cap);
}
static void it_free(rec_iter* it) { free(it->seq); it->seq = NULL; }

static int next_line(rec_iter* it, int64_t* st, int64_t* ed) {
    if (it->pos < it->n) {
        const uint8_t* p = (const uint8_t*)memchr(it->buf + it->pos, 10, (size_t)(it->n - it->pos));
        if (p) {
            int64_t e = (int64_t)(p - it->buf);
            *st = it->start; *ed = e + 1; it->start = e + 1; it->pos = e + 1;
            return 1;
        }
        it->pos = it->n;
    }
    if (!it->tail_done) {
        it->tail_done = 1;
        /* `if end > start > 0: yield start, end + 1` — end is the last loop index,
         * or 0 when range(offset, len) was empty (:125-132) */
        int64_t end = (it->offset < it->n) ? it->n - 1 : 0;
        if (end > it->start && it->start > 0) { *st = it->start; *ed = end + 1; return 1; }
    }
    return 0;
}

static void seq_append(rec_iter* it, const uint8_t* p, int64_t len) {
    if (it->seq_len + len > it->seq_cap) {
        while (it->seq_len + len > it->seq_cap) it->seq_cap *= 2;
        it->seq = (uint8_t*)realloc(it->seq, (size_t)it->seq_cap);
    }
    memcpy(it->seq + it->seq_len, p, (size_t)len);
    it->seq_len += len;
}

/* yields (qid, seq, ptr); seq = it->seq[0:seq_len] valid until the next call */
static int next_record(rec_iter* it) {
    if (it->pending) {                      /* start the record whose header we hold */
        it->pending = 0; it->have_qid = 1;
        it->qid_st = it->pend_st; it->qid_len = it->pend_len; it->seq_len = 0;
    }
    int64_t st, ed;
    while (next_line(it, &st, &ed)) {
        int64_t ptr = st;                   /* ptr[0] = st (:153) */
        if (it->buf[st] == 62) {            /* header line (:155) */
            if (it->have_qid) {
                it->r_qid_st = it->qid_st; it->r_qid_len = it->qid_len; it->r_ptr = ptr;
                it->pending = 1; it->pend_st = st; it->pend_len = ed - st - 1;
                return 1;
            }
            it->have_qid = 1; it->qid_st = st; it->qid_len = ed - st - 1; it->seq_len = 0;
        } else {
            seq_append(it, it->buf + st, ed - st - 1);   /* line[:-1] (:167) */
        }
        it->r_ptr = ptr;
    }
    if (!it->final_done) {
        it->final_done = 1;
        if (it->have_qid) {                 /* :170-172 */
            it->r_qid_st = it->qid_st; it->r_qid_len = it->qid_len;
            return 1;
        }
    }
    return 0;
}

/* reverse_jit_ :197-204 */
static uint8_t* reverse_seq(const uint8_t* s, int64_t n, uint8_t** buf, int64_t* cap) {
    if (n > *cap) { *cap = n + (n >> 1) + 16; *buf = (uint8_t*)realloc(*buf, (size_t)*cap); }
    for (int64_t i = 0; i < n; i++) (*buf)[i] = TABREV[s[n - 1 - i]];
    return *buf;
}

/* --------------------------------------------------------- faithful oakht */
typedef struct {
    int64_t cap, size;
    uint64_t* keys;      /* np.empty -> fresh zeroed pages (see DESIGN.md "key-0 rule") */
    uint16_t* vals;
    uint8_t* counts;
} oakht;

static int isprime(int64_t n) {                      /* :355-366 */
    if (n <= 1 || n % 2 == 0 || n % 3 == 0) return 0;
    for (int64_t i = 5; i * i <= n; i += 6)
        if (n % i == 0 || n % (i + 2) == 0) return 0;
    return 1;
}
static int64_t find_prime(int64_t n) {               /* :369-372 */
    for (int64_t i = n; i < n + 70000000; i++) if (isprime(i)) return i;
    return n;
}
static uint64_t fnv_low4(uint64_t val) {             /* fnv :400-418, end-start == 1 */
    uint64_t a = 0xcbf29ce484222325ULL;
    for (int i = 0; i < 4; i++) { a ^= (val & 0xff); a *= 0x100000001b3ULL; val >>= 8; }
    return a;
}
static void oak_init(oakht* t, int64_t capacity) {   /* __init__ :341-352 */
    t->cap = find_prime(capacity); t->size = 0;
    t->keys = (uint64_t*)calloc((size_t)t->cap, 8);
    t->vals = (uint16_t*)calloc((size_t)t->cap, 2);
    t->counts = (uint8_t*)calloc((size_t)t->cap, 1);
}
static void oak_free(oakht* t) { free(t->keys); free(t->vals); free(t->counts); memset(t, 0, sizeof(*t)); }

static int64_t oak_pointer(const oakht* t, uint64_t key) {   /* pointer :521-538 */
    int64_t M = t->cap;
    int64_t j = (int64_t)(fnv_low4(key) % (uint64_t)M), j0 = j;
    for (int64_t k = 0; k < M; k++) {
        if (t->keys[j] == key || t->counts[j] == 0) break;
        j = (int64_t)(((uint64_t)j0 + (uint64_t)k * (uint64_t)k) % (uint64_t)M);
    }
    return j;
}
static void oak_resize(oakht* t) {                   /* resize :423-474 (extend) */
    int64_t N = t->cap;
    uint64_t* ko = t->keys; uint16_t* vo = t->vals; uint8_t* co = t->counts;
    int64_t M = find_prime((int64_t)((double)N * 1.62));
    uint64_t* kn = (uint64_t*)calloc((size_t)M, 8);
    uint16_t* vn = (uint16_t*)calloc((size_t)M, 2);
    uint8_t* cn = (uint8_t*)calloc((size_t)M, 1);
    for (int64_t i = 0; i < N; i++) {
        if (co[i] == 0) continue;
        int64_t j = (int64_t)(fnv_low4(ko[i]) % (uint64_t)M), j0 = j;
        for (int64_t k = 0; k < N; k++) {
            if (cn[j] == 0 || kn[j] == ko[i]) break;
            j = (int64_t)(((uint64_t)j0 + (uint64_t)k * (uint64_t)k) % (uint64_t)M);
        }
        kn[j] = ko[i]; vn[j] = vo[i]; cn[j] = co[i];
    }
    free(ko); free(vo); free(co);
    t->keys = kn; t->vals = vn; t->counts = cn; t->cap = M;
}
static void oak_push(oakht* t, uint64_t key, uint16_t value) {   /* __setitem__ :540-561 */
    int64_t j = oak_pointer(t, key);
    if (t->counts[j] == 0) { t->size++; t->keys[j] = key; }
    t->vals[j] = value;
    t->counts[j] = t->counts[j] < 255 ? (uint8_t)(t->counts[j] + 1) : 255;
    if ((double)t->size / (double)t->cap > 0.75) oak_resize(t);
}
static int oak_has_key(const oakht* t, uint64_t key) {          /* has_key :599-603 — no counts check */
    return t->keys[oak_pointer(t, key)] == key;
}
static uint16_t oak_get(const oakht* t, uint64_t key) {         /* get :566-575 */
    return t->vals[oak_pointer(t, key)];
}

/* add_kmer :1036-1047 — three probe sequences per occurrence */
static inline void add_kmer(oakht* t, uint64_t key, uint8_t hd, uint8_t nt) {
    uint16_t h = (uint16_t)(LASTC[hd] << OFFBIT), d = LASTC[nt];
    if (oak_has_key(t, key)) {
        uint16_t val = oak_get(t, key);
        oak_push(t, key, (uint16_t)(val | h | d));
    } else {
        oak_push(t, key, (uint16_t)(h | d));
    }
}

static uint64_t pow5(int e) { uint64_t r = 1; while (e-- > 0) r *= 5; return r; }
static uint64_t k2n(const uint8_t* s, int k) {       /* k2n_jit :975-985 */
    uint64_t N = 0, p = 1;
    for (int i = 0; i < k; i++) { N += (uint64_t)ALPHA[s[i]] * p; p *= 5; }
    return N;
}

/* ----------------------------------------------------------- k-mer walker */
/* seq2ns_jit_ :991-1033 / build_dbg :1052-1090 window enumeration, including
 * the last-window predecessor quirk (:1078-1080) and numba's binding of the
 * never-entered loop variable to 0 when n == k+1. */
typedef void (*window_fn)(void* ctx, uint64_t idx, uint64_t key, uint8_t hd, uint8_t nt);

static void walk_windows(const uint8_t* s, int64_t n, int k, window_fn fn, void* ctx) {
    if (n > k) {
        uint64_t Nu = k2n(s, k);
        uint64_t idx = 0;
        fn(ctx, idx, Nu, 35, s[k]);
        idx++;
        uint64_t shift = pow5(k - 1);
        int64_t i = 0;
        for (int64_t ii = k; ii < n - 1; ii++) {
            i = ii;
            Nu = Nu / 5 + (uint64_t)ALPHA[s[i]] * shift;
            fn(ctx, idx, Nu, s[i - k], s[i + 1]);
            idx++;
        }
        Nu = Nu / 5 + (uint64_t)ALPHA[s[i + 1]] * shift;
        int64_t hi = i - k; if (hi < 0) hi += n;          /* numba negative-index wrap */
        fn(ctx, idx, Nu, s[hi], 36);
    } else if (n == k) {
        fn(ctx, 0, k2n(s, k), 35, 36);
    } else {
        fn(ctx, 0, SENTINEL, 35, 36);
    }
}

static void dbg_window(void* ctx, uint64_t idx, uint64_t key, uint8_t hd, uint8_t nt) {
    (void)idx; add_kmer((oakht*)ctx, key, hd, nt);
}

/* ------------------------------------------------------------ edge map */
typedef struct { uint64_t n0, v0, n1, v1; int64_t count; int64_t last_walk; } edge_rec;
typedef struct {
    edge_rec* e; int64_t n, cap;        /* edge records, in creation order          */
    int64_t* slot; int64_t nslot;       /* open addressing on record ids (-1 empty) */
    int64_t* order; int64_t n_order;    /* typed-Dict iteration order                */
} edge_map;

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
static uint64_t edge_hash(uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
    return mix64(a ^ mix64(b ^ mix64(c ^ mix64(d + 0x9e3779b97f4a7c15ULL))));
}
static void em_init(edge_map* m) {
    memset(m, 0, sizeof(*m));
    m->cap = 1024; m->e = (edge_rec*)malloc(sizeof(edge_rec) * (size_t)m->cap);
    m->order = (int64_t*)malloc(sizeof(int64_t) * (size_t)m->cap);
    m->nslot = 4096; m->slot = (int64_t*)malloc(sizeof(int64_t) * (size_t)m->nslot);
    for (int64_t i = 0; i < m->nslot; i++) m->slot[i] = -1;
}
static void em_free(edge_map* m) { free(m->e); free(m->slot); free(m->order); memset(m, 0, sizeof(*m)); }
static void em_rehash(edge_map* m) {
    free(m->slot);
    m->nslot *= 2; m->slot = (int64_t*)malloc(sizeof(int64_t) * (size_t)m->nslot);
    for (int64_t i = 0; i < m->nslot; i++) m->slot[i] = -1;
    for (int64_t id = 0; id < m->n; id++) {
        edge_rec* r = &m->e[id];
        uint64_t h = edge_hash(r->n0, r->v0, r->n1, r->v1) & (uint64_t)(m->nslot - 1);
        while (m->slot[h] >= 0) h = (h + 1) & (uint64_t)(m->nslot - 1);
        m->slot[h] = id;
    }
}
/* rdbg_edge_weight :1476-1484: per-walk `visit` dedup, rdbg_edge[k12] += 1 */
static void em_count(edge_map* m, uint64_t n0, uint64_t v0, uint64_t n1, uint64_t v1, int64_t walk) {
    uint64_t h = edge_hash(n0, v0, n1, v1) & (uint64_t)(m->nslot - 1);
    while (m->slot[h] >= 0) {
        edge_rec* r = &m->e[m->slot[h]];
        if (r->n0 == n0 && r->v0 == v0 && r->n1 == n1 && r->v1 == v1) {
            if (r->last_walk != walk) { r->last_walk = walk; r->count++; }
            return;
        }
        h = (h + 1) & (uint64_t)(m->nslot - 1);
    }
    if (m->n == m->cap) {
        m->cap *= 2;
        m->e = (edge_rec*)realloc(m->e, sizeof(edge_rec) * (size_t)m->cap);
        m->order = (int64_t*)realloc(m->order, sizeof(int64_t) * (size_t)m->cap);
    }
    int64_t id = m->n++;
    m->e[id] = (edge_rec){n0, v0, n1, v1, 1, walk};
    m->slot[h] = id;
    m->order[m->n_order++] = id;
    if (m->n * 2 > m->nslot) em_rehash(m);
}

/* ------------------------------------------------------------ result */
typedef struct { int64_t hst, hlen, start, end, strand, label; } row_rec;

struct pgo_result {
    int k;
    oakht dbg, rdbg;
    int has_dbg, has_rdbg;
    int64_t n_bases, n_records;
    double t_dbg, t_rdbg;
    edge_map edges; int has_edges;
    row_rec* rows; int64_t n_rows, cap_rows;
};

static int ns_hit(int64_t N, int64_t ns, int ns_never) { return !ns_never && N > ns; }

/* seq2rdbg :1251-1266 -> seq2dbg_jit_ :1208-1228: every window of the pass
 * (both strands when rc0) to fn, with the chunk checkpoints (:1224-1225) and
 * their resume (offset = the seqio ptr of the record that crossed, :1255-1259)
 * and the -n limit (:1227). */
static void dbg_pass(const uint8_t* buf, int64_t n, int k, int rc0, int64_t ns, int ns_never, int64_t chunk,
                     window_fn fn, void* ctx, int64_t* n_bases, int64_t* n_records) {
    uint8_t* rv = NULL; int64_t rvcap = 0;
    int64_t N = 0, offset = 0;
    for (;;) {
        int64_t Nl = 0, chk = 0, ptr = 0; int done = 1;
        rec_iter it; it_init(&it, buf, n, offset);
        while (next_record(&it)) {
            const uint8_t* s = it.seq; int64_t ln = it.seq_len;
            walk_windows(s, ln, k, fn, ctx);
            Nl += ln; chk += ln; *n_bases += ln; (*n_records)++;
            if (rc0) {
                walk_windows(reverse_seq(s, ln, &rv, &rvcap), ln, k, fn, ctx);
                Nl += ln; chk += ln;
            }
            if (chk > chunk) { done = -1; ptr = it.r_ptr; break; }
            if (ns_hit(Nl, ns, ns_never)) break;
        }
        it_free(&it);
        if (done == -1) offset = ptr;                /* dump(...'_db_brkpt') + resume */
        else break;
        N += Nl;
        if (ns_hit(N, ns, ns_never)) break;
    }
    free(rv);
}

int pgo_build_graph(const uint8_t* buf, int64_t n, int k, int rc0,
                    int64_t ns, int ns_never, int64_t chunk, pgo_result** out) {
    init_tables();
    if (k < 1) k = 1;
    if (k > 27) k = 27;                               /* :1236 */
    pgo_result* r = (pgo_result*)calloc(1, sizeof(pgo_result));
    r->k = k;
    double t0 = now_s();
    oak_init(&r->dbg, 1 << 20); r->has_dbg = 1;       /* init_dict :1097-1122 */
    dbg_pass(buf, n, k, rc0, ns, ns_never, chunk, dbg_window, &r->dbg, &r->n_bases, &r->n_records);
    double t1 = now_s();
    /* dbg2rdbg :1313-1321 -> build_rdbg_jit_ :1293-1309 (slot order) */
    oak_init(&r->rdbg, 1 << 20); r->has_rdbg = 1;
    for (int64_t i = 0; i < r->dbg.cap; i++) {
        if (r->dbg.counts[i] == 0) continue;
        uint16_t hn = r->dbg.vals[i];
        int pr = __builtin_popcount((unsigned)(hn >> OFFBIT));
        int sf = __builtin_popcount((unsigned)(hn & 63));
        if (pr == 1 && sf == 1) continue;
        oak_push(&r->rdbg, r->dbg.keys[i], hn);
    }
    double t2 = now_s();
    r->t_dbg = t1 - t0; r->t_rdbg = t2 - t1;
    *out = r;
    return 0;
}

/* ------------------------------------------------- dBG of one key range */
/* The same dBG (key -> OR of add_kmer's masks, :1036-1047) for the keys in
 * [lo, hi) only (hi = 2^64-1 includes the n<k sentinel), by sorting the
 * range's occurrences instead of inserting them into an oakht: what the
 * benchmark-scale digests of inputs too large for one in-memory oakht use
 * (tests/golden/make_scale_digests.py).  The result is a set, so it does not
 * depend on the table (tests/test_oracle_golden.py checks it against
 * pgo_build_graph on every golden input). */
typedef struct { uint64_t key; uint16_t mask; uint16_t pad[3]; } kocc;
typedef struct { uint64_t lo, hi; kocc* v; int64_t n, cap; } range_ctx;

/* pass 1 (v == NULL) counts the range's occurrences, pass 2 stores them */
static void range_window(void* ctx, uint64_t idx, uint64_t key, uint8_t hd, uint8_t nt) {
    (void)idx;
    range_ctx* c = (range_ctx*)ctx;
    if (!(key >= c->lo && (key < c->hi || (c->hi == SENTINEL && key == SENTINEL)))) return;
    if (c->v && c->n < c->cap) {
        c->v[c->n].key = key;
        c->v[c->n].mask = (uint16_t)((LASTC[hd] << OFFBIT) | LASTC[nt]);
    }
    c->n++;
}

static int radix_sort_kocc(kocc* a, int64_t n) {      /* LSD, 8-bit digits, stable */
    kocc* b = (kocc*)malloc(sizeof(kocc) * (size_t)(n ? n : 1));
    if (!b) return -1;
    int64_t cnt[256];
    uint64_t all_or = 0, all_and = ~0ull;
    for (int64_t i = 0; i < n; i++) { all_or |= a[i].key; all_and &= a[i].key; }
    kocc *src = a, *dst = b;
    for (int sh = 0; sh < 64; sh += 8) {
        if ((((all_or ^ all_and) >> sh) & 0xFF) == 0) continue;       /* digit equal everywhere */
        memset(cnt, 0, sizeof(cnt));
        for (int64_t i = 0; i < n; i++) cnt[(src[i].key >> sh) & 0xFF]++;
        int64_t o = 0;
        for (int d = 0; d < 256; d++) { int64_t t = cnt[d]; cnt[d] = o; o += t; }
        for (int64_t i = 0; i < n; i++) dst[cnt[(src[i].key >> sh) & 0xFF]++] = src[i];
        kocc* t = src; src = dst; dst = t;
    }
    if (src != a) memcpy(a, src, sizeof(kocc) * (size_t)n);
    free(b);
    return 0;
}

int64_t pgo_dbg_range(const uint8_t* buf, int64_t n, int k, int rc0, int64_t ns, int ns_never, int64_t chunk,
                      uint64_t lo, uint64_t hi, uint64_t** keys_out, uint16_t** masks_out) {
    init_tables();
    if (k < 1) k = 1;
    if (k > 27) k = 27;
    range_ctx c = {lo, hi, NULL, 0, 0};
    int64_t nb = 0, nr = 0;
    dbg_pass(buf, n, k, rc0, ns, ns_never, chunk, range_window, &c, &nb, &nr);
    c.cap = c.n;
    c.v = (kocc*)malloc(sizeof(kocc) * (size_t)(c.cap ? c.cap : 1));
    if (!c.v) return -1;
    c.n = 0;
    dbg_pass(buf, n, k, rc0, ns, ns_never, chunk, range_window, &c, &nb, &nr);
    if (c.n != c.cap || radix_sort_kocc(c.v, c.n) != 0) { free(c.v); return -1; }
    int64_t m = 0;
    for (int64_t i = 0; i < c.n; i++) {               /* OR per key, in key order */
        if (m && c.v[m - 1].key == c.v[i].key) c.v[m - 1].mask |= c.v[i].mask;
        else c.v[m++] = c.v[i];
    }
    uint64_t* K = (uint64_t*)malloc(8 * (size_t)(m ? m : 1));
    uint16_t* M = (uint16_t*)malloc(2 * (size_t)(m ? m : 1));
    if (!K || !M) { free(K); free(M); free(c.v); return -1; }
    for (int64_t i = 0; i < m; i++) { K[i] = c.v[i].key; M[i] = c.v[i].mask; }
    free(c.v);
    *keys_out = K; *masks_out = M;
    return m;
}
void pgo_free_buf(void* p) { free(p); }

/* rdbg_edge_weight :1446-1518 for one walk */
typedef struct {
    const oakht* rdbg; edge_map* m; int64_t walk;
    int have0; uint64_t n0, v0;
} edge_walk;

static void edge_window(void* ctx, uint64_t idx, uint64_t key, uint8_t hd, uint8_t nt) {
    (void)idx;
    edge_walk* w = (edge_walk*)ctx;
    if (key == SENTINEL) return;                                   /* :1461-1462 */
    if (!oak_has_key(w->rdbg, key)) return;                        /* :1465 */
    uint64_t v = ((uint64_t)LASTC[hd] << EDGE_OFFBIT) | (uint64_t)LASTC[nt];
    if (!w->have0) { w->have0 = 1; w->n0 = key; w->v0 = v; return; }
    em_count(w->m, w->n0, w->v0, key, v, w->walk);
    w->n0 = key; w->v0 = v;
}

static void reverse_order(edge_map* m) {
    for (int64_t i = 0, j = m->n_order - 1; i < j; i++, j--) {
        int64_t t = m->order[i]; m->order[i] = m->order[j]; m->order[j] = t;
    }
}

int pgo_edges(pgo_result* r, const uint8_t* buf, int64_t n, int rc1,
              int64_t ns, int ns_never, int64_t chunk) {
    init_tables();
    if (!r || !r->has_rdbg) return -1;
    if (r->has_edges) em_free(&r->edges);
    em_init(&r->edges); r->has_edges = 1;
    uint8_t* rv = NULL; int64_t rvcap = 0;
    int64_t N = 0, offset = 0, walk = 0;
    for (;;) {                                              /* seq2graph :1876-1890 */
        int64_t chk = 0, ptr = 0; int done = 1;
        rec_iter it; it_init(&it, buf, n, offset);
        while (next_record(&it)) {                          /* :1813-1825 */
            edge_walk w = {&r->rdbg, &r->edges, walk++, 0, 0, 0};
            walk_windows(it.seq, it.seq_len, r->k, edge_window, &w);
            if (rc1) {
                edge_walk w2 = {&r->rdbg, &r->edges, walk++, 0, 0, 0};
                walk_windows(reverse_seq(it.seq, it.seq_len, &rv, &rvcap), it.seq_len, r->k,
                             edge_window, &w2);
            }
            N += it.seq_len;
            if (ns_hit(N, ns, ns_never)) break;
            chk += it.seq_len;
            if (chk > chunk) { done = -1; ptr = it.r_ptr; break; }
        }
        it_free(&it);
        if (done == -1) {
            offset = ptr;
            /* dump(jit=True) pops items LIFO (dict2array :229) and load_on_disk
             * re-inserts them in that order: the Dict order reverses. */
            reverse_order(&r->edges);
        } else {
            break;
        }
    }
    free(rv);
    return 0;
}

/* ------------------------------------------------------------ labels */
typedef struct { int64_t* key; int64_t* val; int64_t* id; uint8_t* used; int64_t cap; } label_map;

static uint64_t lab_hash(int64_t a, int64_t b) { return mix64((uint64_t)a * 0x9e3779b97f4a7c15ULL ^ mix64((uint64_t)b)); }
static void lm_build(label_map* L, const int64_t* k, const int64_t* v, const int64_t* id, int64_t n) {
    L->cap = 16; while (L->cap < 2 * n + 16) L->cap *= 2;
    L->key = (int64_t*)malloc(8 * (size_t)L->cap); L->val = (int64_t*)malloc(8 * (size_t)L->cap);
    L->id = (int64_t*)malloc(8 * (size_t)L->cap); L->used = (uint8_t*)calloc((size_t)L->cap, 1);
    for (int64_t i = 0; i < n; i++) {
        uint64_t h = lab_hash(k[i], v[i]) & (uint64_t)(L->cap - 1);
        while (L->used[h] && !(L->key[h] == k[i] && L->val[h] == v[i])) h = (h + 1) & (uint64_t)(L->cap - 1);
        L->used[h] = 1; L->key[h] = k[i]; L->val[h] = v[i]; L->id[h] = id[i];   /* later wins */
    }
}
static int lm_get(const label_map* L, int64_t a, int64_t b, int64_t* out) {
    uint64_t h = lab_hash(a, b) & (uint64_t)(L->cap - 1);
    while (L->used[h]) {
        if (L->key[h] == a && L->val[h] == b) { *out = L->id[h]; return 1; }
        h = (h + 1) & (uint64_t)(L->cap - 1);
    }
    return 0;
}
static void lm_free(label_map* L) { free(L->key); free(L->val); free(L->id); free(L->used); }

typedef struct {
    const label_map* L; int k;
    int64_t* starts; int64_t* labels; int64_t n, cap;
} path_walk;

static void path_push(path_walk* p, int64_t s, int64_t l) {
    if (p->n == p->cap) {
        p->cap = p->cap ? p->cap * 2 : 64;
        p->starts = (int64_t*)realloc(p->starts, 8 * (size_t)p->cap);
        p->labels = (int64_t*)realloc(p->labels, 8 * (size_t)p->cap);
    }
    p->starts[p->n] = s; p->labels[p->n] = l; p->n++;
}
/* seq2path_jit_ :1535-1560 */
static void path_window(void* ctx, uint64_t idx, uint64_t key, uint8_t hd, uint8_t nt) {
    path_walk* p = (path_walk*)ctx;
    int64_t hv = ((int64_t)LASTC[hd] << OFFBIT) | (int64_t)LASTC[nt];
    int64_t label;
    if (!lm_get(p->L, (int64_t)key, hv, &label)) return;
    if (p->starts[p->n - 1] < (int64_t)idx) {
        int64_t pos = (int64_t)idx + p->k;
        if (p->labels[p->n - 1] != label) path_push(p, pos, label);
        else p->starts[p->n - 1] = pos;
    }
}

static void add_row(pgo_result* r, int64_t hst, int64_t hlen, int64_t s, int64_t e, int64_t strand, int64_t lab) {
    if (r->n_rows == r->cap_rows) {
        r->cap_rows = r->cap_rows ? r->cap_rows * 2 : 1024;
        r->rows = (row_rec*)realloc(r->rows, sizeof(row_rec) * (size_t)r->cap_rows);
    }
    r->rows[r->n_rows++] = (row_rec){hst, hlen, s, e, strand, lab};
}

int pgo_rows(pgo_result* r, const uint8_t* buf, int64_t n, int rc1,
             int64_t ns, int ns_never,
             const int64_t* lab_key, const int64_t* lab_val, const int64_t* lab_id,
             int64_t n_labels) {
    init_tables();
    if (!r) return -1;
    r->n_rows = 0;
    label_map L; lm_build(&L, lab_key, lab_val, lab_id, n_labels);
    uint8_t* rv = NULL; int64_t rvcap = 0;
    path_walk p = {&L, r->k, NULL, NULL, 0, 0};
    int64_t N = 0;
    /* seqs2path_jit_ :1833 passes `isfasta` (True) into seqio_jit_'s offset slot */
    rec_iter it; it_init(&it, buf, n, 1);
    while (next_record(&it)) {
        int64_t lseq = it.seq_len;
        p.n = 0; path_push(&p, 0, -1);
        walk_windows(it.seq, lseq, r->k, path_window, &p);
        for (int64_t i = 1; i < p.n; i++)            /* int32 output array :1533, :1569-1571 */
            add_row(r, it.r_qid_st, it.r_qid_len, (int32_t)p.starts[i - 1], (int32_t)p.starts[i], 1,
                    (int32_t)p.labels[i]);
        if (rc1) {
            p.n = 0; path_push(&p, 0, -1);
            walk_windows(reverse_seq(it.seq, lseq, &rv, &rvcap), lseq, r->k, path_window, &p);
            for (int64_t i = 1; i < p.n; i++) {       /* :1842-1844 */
                int32_t st = (int32_t)p.starts[i - 1], ed = (int32_t)p.starts[i];
                add_row(r, it.r_qid_st, it.r_qid_len, (int32_t)(lseq - ed), (int32_t)(lseq - st), -1,
                        (int32_t)p.labels[i]);
            }
        }
        N += lseq;
        if (ns_hit(N, ns, ns_never)) break;
    }
    it_free(&it);
    free(p.starts); free(p.labels); free(rv);
    lm_free(&L);
    return 0;
}

/* ------------------------------------------------------------ accessors */
int64_t pgo_n_dbg(const pgo_result* r) { return r->dbg.size; }
int64_t pgo_n_rdbg(const pgo_result* r) { return r->rdbg.size; }
int64_t pgo_n_edges(const pgo_result* r) { return r->has_edges ? r->edges.n_order : 0; }
int64_t pgo_n_rows(const pgo_result* r) { return r->n_rows; }
int64_t pgo_n_bases(const pgo_result* r) { return r->n_bases; }
int64_t pgo_n_records(const pgo_result* r) { return r->n_records; }
double pgo_seconds_dbg(const pgo_result* r) { return r->t_dbg; }
double pgo_seconds_rdbg(const pgo_result* r) { return r->t_rdbg; }

void pgo_get_dbg(const pgo_result* r, uint64_t* keys, uint16_t* masks) {   /* iteritems :623-631 */
    int64_t o = 0;
    for (int64_t i = 0; i < r->dbg.cap; i++)
        if (r->dbg.counts[i]) { keys[o] = r->dbg.keys[i]; masks[o] = r->dbg.vals[i]; o++; }
}
void pgo_get_dbg_counts(const pgo_result* r, uint8_t* counts) {         /* counts, same order */
    int64_t o = 0;
    for (int64_t i = 0; i < r->dbg.cap; i++)
        if (r->dbg.counts[i]) counts[o++] = r->dbg.counts[i];
}
int64_t pgo_dbg_capacity(const pgo_result* r) { return r->dbg.cap; }   /* dump parameters[0] (:253) */
void pgo_get_rdbg(const pgo_result* r, uint64_t* keys) {
    int64_t o = 0;
    for (int64_t i = 0; i < r->rdbg.cap; i++)
        if (r->rdbg.counts[i]) keys[o++] = r->rdbg.keys[i];
}
void pgo_get_edges(const pgo_result* r, uint64_t* t, int64_t* counts) {
    for (int64_t i = 0; i < r->edges.n_order; i++) {
        const edge_rec* e = &r->edges.e[r->edges.order[i]];
        t[4 * i] = e->n0; t[4 * i + 1] = e->v0; t[4 * i + 2] = e->n1; t[4 * i + 3] = e->v1;
        counts[i] = e->count;
    }
}
void pgo_get_rows(const pgo_result* r, int64_t* out) {
    for (int64_t i = 0; i < r->n_rows; i++) {
        const row_rec* w = &r->rows[i];
        out[6 * i] = w->hst; out[6 * i + 1] = w->hlen; out[6 * i + 2] = w->start;
        out[6 * i + 3] = w->end; out[6 * i + 4] = w->strand; out[6 * i + 5] = w->label;
    }
}
void pgo_set_rdbg(pgo_result* r, const uint64_t* keys, int64_t n) {
    if (r->has_rdbg) oak_free(&r->rdbg);
    oak_init(&r->rdbg, 1 << 20); r->has_rdbg = 1;            /* init_dict, then __setitem__ per key */
    for (int64_t i = 0; i < n; i++) oak_push(&r->rdbg, keys[i], 0);
}

void pgo_free(pgo_result* r) {
    if (!r) return;
    if (r->has_dbg) oak_free(&r->dbg);
    if (r->has_rdbg) oak_free(&r->rdbg);
    if (r->has_edges) em_free(&r->edges);
    free(r->rows);
    free(r);
}
