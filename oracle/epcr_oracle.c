/*
 * epcr_oracle.c -- scalar C restatement of the merpcr search path.
 * TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the checker; never linked into the product.
 *
 * Restates, with single-chunk (-T 1) semantics, src/merpcr/core/engine.py of
 * FOI-Bioinformatics/merpcr:
 *   scan            _process_thread  engine.py:453-505
 *   verify + pair   _match_sts       engine.py:507-597
 *   compare         _compare_seqs    engine.py:599-642
 *   output order    hits.sort(key=pos1) over discovery order, engine.py:434
 * Parity pinning: checked against the Python oracle (oracle/epcr_oracle.py),
 * which is itself checked against the reference's golden outputs
 * (tests/test_oracle_golden.py, tests/test_c_oracle.py).
 *
 * Input bytes are compared after ASCII upper-casing; bytes >= 0x80 are opaque
 * (literal equality only), exactly as the device encoding defines them.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { int32_t W, M, N, X, I; } oparams;
typedef struct { uint64_t pos1, pos2; uint32_t seq, rec; } ohit;

typedef struct {
    uint32_t n_rec;
    const uint32_t* key;
    const uint32_t* hash_off;
    const uint64_t* pcr_size;
    const uint8_t* p1;
    const uint64_t* p1_off;
    const uint8_t* p2;
    const uint64_t* p2_off;
    /* key -> bucket of record indices (insertion order) */
    uint64_t cap;
    uint32_t* slot_key;
    int64_t* slot_head; /* first record of the bucket, -1 empty */
    int64_t* next_rec;  /* next record with the same key */
} otable;

static uint8_t up(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }

static int code2(uint8_t c) {
    switch (c) {
        case 'A': return 0; case 'C': return 1; case 'G': return 2;
        case 'T': case 'U': return 3;
        default: return -1;
    }
}

static int iupac(uint8_t c) {
    switch (c) {
        case 'A': return 1; case 'C': return 2; case 'G': return 4; case 'T': case 'U': return 8;
        case 'R': return 5; case 'Y': return 10; case 'M': return 3; case 'K': return 12;
        case 'S': return 6; case 'W': return 9; case 'B': return 14; case 'D': return 13;
        case 'H': return 11; case 'V': return 7; case 'N': return 15;
        default: return 0;
    }
}

/* engine.py:599-642 */
static int compare(const uint8_t* g, const uint8_t* p, uint32_t L, int plus, const oparams* prm) {
    int mm = 0;
    for (uint32_t i = 0; i < L; ++i) {
        const uint8_t a = up(g[i]), b = up(p[i]);
        int ok;
        if (prm->I && iupac(a) && iupac(b)) ok = (iupac(a) & iupac(b)) != 0;
        else ok = a == b;
        if (!ok) {
            const int prot = plus ? ((int64_t)i >= (int64_t)L - prm->X) : ((int64_t)i < prm->X);
            if (prot) return 0;
            if (++mm > prm->N) return 0;
        }
    }
    return 1;
}

typedef struct { ohit* v; uint64_t n, cap; } hitvec;

static int push(hitvec* h, uint64_t p1, uint64_t p2, uint32_t seq, uint32_t rec) {
    if (h->n == h->cap) {
        uint64_t nc = h->cap ? h->cap * 2 : 1024;
        ohit* nv = (ohit*)realloc(h->v, nc * sizeof(ohit));
        if (!nv) return -1;
        h->v = nv;
        h->cap = nc;
    }
    h->v[h->n].pos1 = p1;
    h->v[h->n].pos2 = p2;
    h->v[h->n].seq = seq;
    h->v[h->n].rec = rec;
    h->n++;
    return 0;
}

static uint64_t slot_of(uint32_t key, uint64_t cap) {
    return (uint64_t)(((uint64_t)key * 0x9E3779B97F4A7C15ull) >> 17) & (cap - 1);
}

static int64_t bucket(const otable* t, uint32_t key) {
    uint64_t s = slot_of(key, t->cap);
    while (t->slot_head[s] >= 0) {
        if (t->slot_key[s] == key) return t->slot_head[s];
        s = (s + 1) & (t->cap - 1);
    }
    return -1;
}

/* engine.py:507-597 for record r at amplicon start k */
static int match_at(const otable* t, const oparams* prm, const uint8_t* s, uint64_t n, uint64_t k,
                    uint32_t r, uint32_t seq, hitvec* out) {
    const uint64_t l1 = t->p1_off[r + 1] - t->p1_off[r];
    const uint64_t l2 = t->p2_off[r + 1] - t->p2_off[r];
    if (k + l1 > n || !compare(s + k, t->p1 + t->p1_off[r], (uint32_t)l1, 1, prm)) return 0;
    const uint64_t avail = n - (k + l1);
    if (avail < l2) return 0;
    uint64_t e = t->pcr_size[r];
    int64_t hi;
    if (e > avail + l1) {
        e = avail + l1;
        hi = 0;
    } else {
        hi = (int64_t)(n - k - e) < prm->M ? (int64_t)(n - k - e) : prm->M;
    }
    int64_t lo = (int64_t)e - (int64_t)l1 - (int64_t)l2;
    if (lo > prm->M) lo = prm->M;
    if (lo < 0) lo = 0;
    /* try order 0, -1, +1, -2, +2, ... (engine.py:542-593) */
    for (int64_t i = 0; i <= prm->M; ++i) {
        for (int side = 0; side < 2; ++side) {
            int64_t d;
            if (i == 0) {
                if (side) continue;
                d = 0;
            } else {
                d = side ? i : -i;
                if (d < 0 && i > lo) continue;
                if (d > 0 && i > hi) continue;
            }
            const int64_t p2 = (int64_t)k + (int64_t)e - (int64_t)l2 + d;
            if (d <= 0 && (int64_t)(k + l1) > p2) continue;
            if (p2 + (int64_t)l2 > (int64_t)n) continue;
            if (compare(s + p2, t->p2 + t->p2_off[r], (uint32_t)l2, 0, prm))
                if (push(out, k, (uint64_t)p2 + l2 - 1, seq, r)) return -1;
        }
    }
    return 0;
}

/* engine.py:453-505 restricted to amplicon starts k in [klo, khi) */
static int scan_range(const otable* t, const oparams* prm, const uint8_t* s, uint64_t n, uint32_t seq,
                      uint64_t klo, uint64_t khi, uint32_t max_off, hitvec* out) {
    const int W = prm->W;
    if (n <= (uint64_t)W) return 0;
    const uint64_t mask = (W == 16) ? 0xFFFFFFFFull : ((1ull << (2 * W)) - 1);
    uint64_t pend = khi + max_off;
    if (pend > n - W + 1) pend = n - W + 1;
    if (klo >= pend) return 0;
    uint64_t h = 0;
    int64_t last_bad = -1;
    for (uint64_t j = klo; j < pend + W - 1; ++j) {
        const int c = code2(up(s[j]));
        if (c < 0) {
            last_bad = (int64_t)j;
            h = (h << 2) & mask;
        } else {
            h = ((h << 2) | (uint64_t)c) & mask;
        }
        if (j + 1 < klo + W) continue;
        const uint64_t pos = j + 1 - W;
        if (last_bad >= (int64_t)pos) continue;
        for (int64_t r = bucket(t, (uint32_t)h); r >= 0; r = t->next_rec[r]) {
            const uint32_t off = t->hash_off[r];
            if (pos < off) continue;
            const uint64_t k = pos - off;
            if (k < klo || k >= khi) continue;
            const uint64_t l1 = t->p1_off[r + 1] - t->p1_off[r];
            if (k + l1 > n) continue;
            if (match_at(t, prm, s, n, k, (uint32_t)r, seq, out)) return -1;
        }
    }
    return 0;
}

typedef struct { uint64_t k; uint32_t off, rec; uint64_t idx; } skey;

static const otable* g_sort_table;

static int cmp_hit(const void* a, const void* b) {
    const skey* x = (const skey*)a;
    const skey* y = (const skey*)b;
    if (x->k != y->k) return x->k < y->k ? -1 : 1;
    /* stable on discovery order (engine.py:434 is a stable sort by pos1) */
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

typedef struct {
    const otable* t;
    const oparams* prm;
    const uint8_t* s;
    uint64_t n, klo, khi;
    uint32_t seq, max_off;
    hitvec out;
    int rc;
} job;

static void* run_job(void* arg) {
    job* j = (job*)arg;
    j->rc = scan_range(j->t, j->prm, j->s, j->n, j->seq, j->klo, j->khi, j->max_off, &j->out);
    if (!j->rc && j->out.n > 1) {
        skey* ks = (skey*)malloc(j->out.n * sizeof(skey));
        ohit* tmp = (ohit*)malloc(j->out.n * sizeof(ohit));
        if (!ks || !tmp) {
            free(ks);
            free(tmp);
            j->rc = -1;
            return NULL;
        }
        for (uint64_t i = 0; i < j->out.n; ++i) {
            ks[i].k = j->out.v[i].pos1;
            ks[i].idx = i;
        }
        qsort(ks, j->out.n, sizeof(skey), cmp_hit);
        for (uint64_t i = 0; i < j->out.n; ++i) tmp[i] = j->out.v[ks[i].idx];
        memcpy(j->out.v, tmp, j->out.n * sizeof(ohit));
        free(ks);
        free(tmp);
    }
    return NULL;
}

/* Whole search.  Sequence s is split into `nthreads` contiguous ranges of amplicon
 * start k; each range is scanned and sorted on its own, and the concatenation is
 * the reference's order.  Returns the hit count (>= 0) or -1; *out is malloc'd. */
int64_t oracle_search(const oparams* prm, uint32_t n_seq, const uint8_t* const* seqs, const uint64_t* lens,
                      uint32_t n_rec, const uint32_t* key, const uint32_t* hash_off, const uint64_t* pcr_size,
                      const uint8_t* p1, const uint64_t* p1_off, const uint8_t* p2, const uint64_t* p2_off,
                      int nthreads, ohit** out) {
    otable t;
    memset(&t, 0, sizeof(t));
    t.n_rec = n_rec;
    t.key = key;
    t.hash_off = hash_off;
    t.pcr_size = pcr_size;
    t.p1 = p1;
    t.p1_off = p1_off;
    t.p2 = p2;
    t.p2_off = p2_off;
    t.cap = 64;
    while (t.cap < 2ull * n_rec + 2) t.cap <<= 1;
    t.slot_key = (uint32_t*)calloc(t.cap, sizeof(uint32_t));
    t.slot_head = (int64_t*)malloc(t.cap * sizeof(int64_t));
    t.next_rec = (int64_t*)malloc((n_rec + 1) * sizeof(int64_t));
    int64_t* tail = (int64_t*)malloc(t.cap * sizeof(int64_t));
    if (!t.slot_key || !t.slot_head || !t.next_rec || !tail) return -1;
    for (uint64_t i = 0; i < t.cap; ++i) t.slot_head[i] = -1;
    uint32_t max_off = 0;
    for (uint32_t r = 0; r < n_rec; ++r) {
        t.next_rec[r] = -1;
        if (hash_off[r] > max_off) max_off = hash_off[r];
        uint64_t s = slot_of(key[r], t.cap);
        while (t.slot_head[s] >= 0 && t.slot_key[s] != key[r]) s = (s + 1) & (t.cap - 1);
        if (t.slot_head[s] < 0) {
            t.slot_key[s] = key[r];
            t.slot_head[s] = r;
        } else {
            t.next_rec[tail[s]] = r;
        }
        tail[s] = r;
    }
    free(tail);
    if (nthreads < 1) nthreads = 1;
    hitvec all = {0, 0, 0};
    int rc = 0;
    job* jobs = (job*)calloc((size_t)nthreads, sizeof(job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    for (uint32_t q = 0; q < n_seq && !rc; ++q) {
        const uint64_t n = lens[q];
        for (int i = 0; i < nthreads; ++i) {
            jobs[i].t = &t;
            jobs[i].prm = prm;
            jobs[i].s = seqs[q];
            jobs[i].n = n;
            jobs[i].seq = q;
            jobs[i].max_off = max_off;
            jobs[i].klo = n * (uint64_t)i / (uint64_t)nthreads;
            jobs[i].khi = n * (uint64_t)(i + 1) / (uint64_t)nthreads;
            jobs[i].out.n = 0;
            jobs[i].rc = 0;
        }
        if (nthreads == 1) run_job(&jobs[0]);
        else {
            for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, run_job, &jobs[i]);
            for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
        }
        for (int i = 0; i < nthreads && !rc; ++i) {
            if (jobs[i].rc) rc = -1;
            for (uint64_t h = 0; h < jobs[i].out.n && !rc; ++h) {
                ohit* x = &jobs[i].out.v[h];
                if (push(&all, x->pos1, x->pos2, x->seq, x->rec)) rc = -1;
            }
        }
    }
    for (int i = 0; i < nthreads; ++i) free(jobs[i].out.v);
    free(jobs);
    free(th);
    free(t.slot_key);
    free(t.slot_head);
    free(t.next_rec);
    (void)g_sort_table;
    if (rc) {
        free(all.v);
        return -1;
    }
    *out = all.v;
    return (int64_t)all.n;
}

void oracle_free(void* p) { free(p); }
