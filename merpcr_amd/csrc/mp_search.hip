// The hot path: seed scan -> primer-1 verify -> amplicon pair-check -> hits.
//
// Replaces, with T=1 semantics, MerPCR._process_thread (engine.py:453-505),
// _match_sts (engine.py:507-597) and _compare_seqs (engine.py:599-642), all in
// src/merpcr/core/engine.py of the reference.
//
// Kernel structure (one 256-thread workgroup = one tile of kTile window
// positions of one sequence; each wave owns 1024 consecutive positions):
//   1. seed stage: 64 consecutive window positions per wave step, one per lane.
//      Each lane pulls its W-mer from the 2-bit plane and its ambiguity bits from
//      ginv (L1-broadcast loads), tests the presence filter and, on a hit, probes
//      the open-addressed table for its bucket.
//   2. compaction: lanes holding a bucket append (pos, bucket) to a per-wave LDS
//      queue with a ballot + popcount prefix, so verification runs with all 64
//      lanes busy whatever the seed density.
//   3. drain (queue >= 64 entries): a wave prefix over bucket sizes expands the
//      queue into (pos, record) candidates, 64 per pass; each lane verifies
//      primer 1 with a bit-sliced 2-bit compare (32 bases per step, exception
//      positions resolved through the run index), then pair-checks primer 2 over
//      the amplicon +- margin window and emits 128-bit order keys.
#include <algorithm>

#include "mp_internal.h"

namespace mp {

struct ScanArgs {
    const uint64_t* g2;
    const uint64_t* gexc;
    const uint64_t* ginv;
    const uint64_t* xr_start;
    const uint8_t* xr_char;
    uint64_t n_xr;
    const uint64_t* seq_base;
    const uint64_t* seq_len;
    const SeqSpan* spans;
    uint32_t n_spans;
    const uint32_t* filt;
    uint32_t filt_log2;
    int filt_direct;
    const uint64_t* slots;
    uint32_t slot_log2;
    const uint32_t* boff;
    const uint32_t* blist;
    const DevRec* recs;
    const uint32_t* rank;
    const uint64_t* planes;
    const uint8_t* pchars;
    int W, M, N, X, I;
    uint64_t g_lo, g_hi;
    uint64_t* hit_hi;
    uint64_t* hit_lo;
    unsigned long long* counters;
    uint64_t cap;
};

__device__ __forceinline__ uint8_t exc_char(const ScanArgs& a, uint64_t j) {
    uint64_t lo = 0, hi = a.n_xr;  // last run with start <= j
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a.xr_start[mid] <= j) lo = mid;
        else hi = mid;
    }
    return a.xr_char[lo];
}

// _compare_seqs (engine.py:599-642) of the L genome bases at global gpos against
// one primer: protected positions are i >= L-X on the '+' strand (plus == true)
// and i < X on the '-' strand; any protected mismatch or more than N fails.
__device__ bool primer_ok(const ScanArgs& a, uint64_t gpos, uint32_t L, uint32_t pl, uint32_t ch,
                          bool plus) {
    int mm = 0;
    for (uint32_t c = 0; c < L; c += 32) {
        const int len = (int)min(32u, L - c);
        const uint64_t G = ext2(a.g2, gpos + c);
        const uint64_t* P = a.planes + (uint64_t)(pl + (c >> 5)) * 4;
        const uint64_t lo = G & kEven, hi = (G >> 1) & kEven;
        const uint64_t nlo = lo ^ kEven, nhi = hi ^ kEven;
        const uint64_t match = (nhi & nlo & P[0]) | (nhi & lo & P[1]) | (hi & nlo & P[2]) | (hi & lo & P[3]);
        const uint64_t inside = sp_lt(len);
        uint64_t mmv = ~match & inside;
        uint32_t ex = (uint32_t)(ext1(a.gexc, gpos + c) >> 32);
        if (len < 32) ex &= ~(0xFFFFFFFFu >> len);
        while (ex) {
            const int i = __clz(ex);
            ex &= ~(0x80000000u >> i);
            const bool ok = char_match(exc_char(a, gpos + c + (uint32_t)i), a.pchars[ch + c + (uint32_t)i], a.I);
            const uint64_t bit = 1ull << (62 - 2 * i);
            mmv = ok ? (mmv & ~bit) : (mmv | bit);
        }
        uint64_t prot;
        if (plus) {
            const int64_t a0 = (int64_t)L - a.X - (int64_t)c;  // first protected local position
            prot = inside & ~sp_lt((int)max<int64_t>(min<int64_t>(a0, 32), 0));
        } else {
            const int64_t b0 = (int64_t)a.X - (int64_t)c;  // protected local positions < b0
            prot = sp_lt((int)max<int64_t>(min<int64_t>(b0, len), 0));
        }
        if (mmv & prot) return false;
        mm += __popcll(mmv);
        if (mm > a.N) return false;
    }
    return true;
}

__device__ __forceinline__ void emit(const ScanArgs& a, uint64_t gk, uint32_t rank, uint32_t tr) {
    const unsigned long long idx = atomicAdd(&a.counters[0], 1ull);
    if (idx < a.cap) {
        a.hit_hi[idx] = gk;
        a.hit_lo[idx] = ((uint64_t)rank << 32) | tr;
    }
}

// _match_sts (engine.py:507-597) for record `rec` seeded at window position pos.
__device__ void process_candidate(const ScanArgs& a, uint64_t sbase, uint32_t n, uint32_t pos, uint32_t rec,
                                  uint32_t& ncand) {
    const DevRec r = a.recs[rec];
    if (pos < r.hash_off) return;
    const uint32_t k = pos - r.hash_off;
    if ((uint64_t)k + r.l1 > n) return;
    const uint64_t gk = sbase + k;
    if (gk < a.g_lo || gk >= a.g_hi) return;
    ++ncand;
    if (!primer_ok(a, gk, r.l1, r.p1_pl, r.p1_ch, true)) return;
    const uint32_t avail = n - k - r.l1;
    if (avail < r.l2) return;
    uint32_t e;
    int hi;
    if (r.size > n - k) {
        e = n - k;
        hi = 0;
    } else {
        e = r.size;
        hi = (int)min<uint32_t>((uint32_t)a.M, n - k - e);
    }
    const int lo = (int)max<int64_t>(0, min<int64_t>(a.M, (int64_t)e - r.l1 - r.l2));
    const uint32_t rk = a.rank[rec];
    for (int d = -lo; d <= hi; ++d) {
        const int64_t p2 = (int64_t)k + e - r.l2 + d;
        if (d <= 0 && (int64_t)k + r.l1 > p2) continue;
        if (p2 + r.l2 > (int64_t)n) continue;
        if (primer_ok(a, sbase + (uint64_t)p2, r.l2, r.p2_pl, r.p2_ch, false)) emit(a, gk, rk, try_rank(d));
    }
}

__device__ __forceinline__ bool lookup(const ScanArgs& a, uint32_t h, uint32_t& bs, uint32_t& bc) {
    const uint32_t mask = (1u << a.slot_log2) - 1;
    uint32_t s = table_slot(h, a.slot_log2);
    for (;;) {
        const uint64_t v = a.slots[s];
        if (v == kEmptySlot) return false;
        if ((uint32_t)(v >> 32) == h) {
            const uint32_t b = (uint32_t)v;
            bs = a.boff[b];
            bc = a.boff[b + 1] - bs;
            return true;
        }
        s = (s + 1) & mask;
    }
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
    }
    return v;
}

__global__ __launch_bounds__(kBlock) void scan_kernel(ScanArgs a) {
    __shared__ uint32_t q_pos[kWaves][128];
    __shared__ uint32_t q_bs[kWaves][128];
    __shared__ uint32_t q_bc[kWaves][128];
    __shared__ uint32_t q_pre[kWaves][128];
    __shared__ uint32_t s_span;

    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    if (threadIdx.x == 0) {
        uint32_t lo = 0, hi = a.n_spans;  // last span with tile0 <= blockIdx.x
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (a.spans[mid].tile0 <= blockIdx.x) lo = mid;
            else hi = mid;
        }
        s_span = lo;
    }
    __syncthreads();
    const SeqSpan sp = a.spans[s_span];
    const uint64_t sbase = a.seq_base[sp.seq];
    const uint32_t n = (uint32_t)a.seq_len[sp.seq];
    const uint32_t tile_begin = sp.p_lo + (uint32_t)(blockIdx.x - sp.tile0) * kTile;
    const uint32_t wb = tile_begin + (uint32_t)w * (64 * kStepsPerWave);
    const uint32_t we = min(wb + 64 * kStepsPerWave, sp.p_hi);
    const int W = a.W;
    uint32_t* qp = q_pos[w];
    uint32_t* qs = q_bs[w];
    uint32_t* qc = q_bc[w];
    uint32_t* qr = q_pre[w];
    uint32_t qn = 0;
    uint32_t ncand = 0;

    auto drain = [&]() {
        const uint32_t c0 = lane < (int)qn ? qc[lane] : 0u;
        const uint32_t c1 = lane + 64 < (int)qn ? qc[lane + 64] : 0u;
        const uint32_t s0 = wave_incl_scan(c0, lane);
        const uint32_t t0 = __shfl(s0, 63, 64);
        const uint32_t s1 = wave_incl_scan(c1, lane) + t0;
        const uint32_t total = __shfl(s1, 63, 64);
        if (lane < (int)qn) qr[lane] = s0 - c0;
        if (lane + 64 < (int)qn) qr[lane + 64] = s1 - c1;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        for (uint32_t b = 0; b < total; b += 64) {
            const uint32_t c = b + (uint32_t)lane;
            if (c < total) {
                uint32_t lo = 0, hi = qn;
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (qr[mid] <= c) lo = mid;
                    else hi = mid;
                }
                const uint32_t rec = a.blist[qs[lo] + (c - qr[lo])];
                process_candidate(a, sbase, n, qp[lo], rec, ncand);
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        qn = 0;
    };

    for (uint32_t p0 = wb; p0 < we; p0 += 64) {
        const uint32_t pos = p0 + (uint32_t)lane;
        uint32_t bs = 0, bc = 0;
        if (pos < we) {
            const uint64_t j = sbase + pos;
            if ((ext1(a.ginv, j) >> (64 - W)) == 0) {
                const uint32_t h = (uint32_t)(ext2(a.g2, j) >> (64 - 2 * W));
                const uint32_t fi = a.filt_direct ? h : filter_index(h, a.filt_log2);
                if ((a.filt[fi >> 5] >> (fi & 31)) & 1u) lookup(a, h, bs, bc);
            }
        }
        const bool have = bc > 0;
        const uint64_t m = __ballot(have);
        if (have) {
            const uint32_t slot = qn + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            qp[slot] = pos;
            qs[slot] = bs;
            qc[slot] = bc;
        }
        qn += (uint32_t)__popcll(m);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (qn >= 64) drain();
    }
    if (qn) drain();
    // candidate statistics, one atomic per wave
    uint32_t tot = ncand;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
    if (lane == 0 && tot) atomicAdd(&a.counters[1], (unsigned long long)tot);
}

__global__ void decode_kernel(const uint64_t* __restrict__ hi, const uint64_t* __restrict__ lo, uint64_t n,
                              const uint64_t* __restrict__ seq_base, const uint64_t* __restrict__ seq_len,
                              uint32_t n_seq, const uint32_t* __restrict__ inv_rank,
                              const DevRec* __restrict__ recs, mp_hit* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t gk = hi[i];
    const uint64_t l = lo[i];
    uint32_t a = 0, b = n_seq;  // last sequence with base <= gk
    while (b - a > 1) {
        const uint32_t mid = (a + b) >> 1;
        if (seq_base[mid] <= gk) a = mid;
        else b = mid;
    }
    const uint64_t k = gk - seq_base[a];
    const uint32_t rec = inv_rank[l >> 32];
    const int32_t d = try_offset((uint32_t)l);
    const uint64_t len = seq_len[a];
    const uint64_t size = recs[rec].size;
    const uint64_t e = size > len - k ? len - k : size;
    mp_hit h;
    h.pos1 = k;
    h.pos2 = (uint64_t)((int64_t)(k + e) - 1 + d);
    h.seq = a;
    h.rec = rec;
    out[i] = h;
}

static void free_search(Search* s) {
    if (!s) return;
    hipFree(s->keys); hipFree(s->tmp_hi); hipFree(s->tmp_lo); hipFree(s->out); hipFree(s->sort_tmp);
    hipFree(s->counters); hipFree(s->spans);
    if (s->ev0) hipEventDestroy(s->ev0);
    if (s->ev1) hipEventDestroy(s->ev1);
    delete s;
}

static int alloc_hits(Search* s, uint64_t cap) {
    hipFree(s->keys); hipFree(s->tmp_hi); hipFree(s->tmp_lo); hipFree(s->out);
    s->keys = s->tmp_hi = s->tmp_lo = nullptr;
    s->out = nullptr;
    s->cap = 0;
    MP_HIP_CHECK(hipMalloc(&s->keys, cap * 16));
    MP_HIP_CHECK(hipMalloc(&s->tmp_hi, cap * 8));
    MP_HIP_CHECK(hipMalloc(&s->tmp_lo, cap * 8));
    MP_HIP_CHECK(hipMalloc(&s->out, cap * sizeof(mp_hit)));
    s->cap = cap;
    return MP_OK;
}

}  // namespace mp

using namespace mp;

MP_EXPORT int mp_search_create(void* table, void* genome, void** out) {
    if (!table || !genome || !out) return fail(MP_E_ARG, "mp_search_create: null pointer");
    *out = nullptr;
    Table* t = (Table*)table;
    Genome* g = (Genome*)genome;
    if (t->device != g->device) return fail(MP_E_ARG, "mp_search_create: table and genome on different devices");
    Search* s = new Search();
    s->table = t;
    s->genome = g;
    int rc = MP_OK;
    do {
        if (hipSetDevice(g->device) != hipSuccess) { rc = fail(MP_E_HIP, "hipSetDevice failed"); break; }
        if (hipMalloc(&s->counters, 64) != hipSuccess) { rc = fail(MP_E_NOMEM, "counter allocation failed"); break; }
        if (hipEventCreate(&s->ev0) != hipSuccess || hipEventCreate(&s->ev1) != hipSuccess) {
            rc = fail(MP_E_HIP, "event creation failed");
            break;
        }
        rc = alloc_hits(s, 1 << 16);
    } while (0);
    if (rc) {
        free_search(s);
        return rc;
    }
    *out = s;
    return MP_OK;
}

MP_EXPORT int mp_search_run(void* search, const mp_range* range, void* stream, uint64_t* n_hits) {
    Search* s = (Search*)search;
    if (!s) return fail(MP_E_ARG, "mp_search_run: null search");
    Table* t = s->table;
    Genome* g = s->genome;
    if (!g->sealed) return fail(MP_E_STATE, "mp_search_run: genome not sealed (call mp_genome_seal)");
    hipStream_t st = (hipStream_t)stream;
    MP_HIP_CHECK(hipSetDevice(g->device));
    mp_range r{0, g->n_seq, 0, 0};
    if (range) r = *range;
    if (r.seq_begin > r.seq_end || r.seq_end > g->n_seq)
        return fail(MP_E_ARG, "mp_search_run: bad sequence range");
    const uint32_t W = (uint32_t)t->prm.wordsize;

    // owned (seq, k) range in global coordinates
    const uint64_t g_lo = (r.seq_begin < g->n_seq) ? g->base[r.seq_begin] + r.k_begin : g->total;
    const uint64_t g_hi = (r.seq_end < g->n_seq) ? g->base[r.seq_end] + r.k_end : g->total;

    // window positions to scan: k in the owned range, extended by max hash offset
    std::vector<SeqSpan> spans;
    uint64_t tiles = 0, windows = 0;
    const uint32_t last = std::min<uint32_t>(r.seq_end, g->n_seq ? g->n_seq - 1 : 0);
    for (uint32_t q = r.seq_begin; q <= last && q < g->n_seq; ++q) {
        const uint64_t n = g->len[q];
        if (n <= W) continue;  // engine.py:458: no window in a sequence of length <= W
        uint64_t klo = (q == r.seq_begin) ? r.k_begin : 0;
        uint64_t khi = (q == r.seq_end) ? r.k_end : n;
        if (q > r.seq_end || (q == r.seq_end && r.k_end == 0)) continue;
        khi = std::min<uint64_t>(khi, n);
        if (klo >= khi) continue;
        const uint64_t plo = klo;
        const uint64_t phi = std::min<uint64_t>(khi + t->max_hash_off, n - W + 1);
        if (plo >= phi) continue;
        SeqSpan sp;
        sp.tile0 = tiles;
        sp.seq = q;
        sp.p_lo = (uint32_t)plo;
        sp.p_hi = (uint32_t)phi;
        sp.pad = 0;
        spans.push_back(sp);
        tiles += (phi - plo + kTile - 1) / kTile;
        windows += phi - plo;
    }
    s->n_windows = windows;
    s->n_candidates = 0;
    s->n_hits = 0;
    s->scan_ms = 0.f;
    if (n_hits) *n_hits = 0;
    if (!tiles) return MP_OK;
    if (spans.size() > s->spans_cap) {
        hipFree(s->spans);
        s->spans = nullptr;
        s->spans_cap = 0;
        MP_HIP_CHECK(hipMalloc(&s->spans, spans.size() * sizeof(SeqSpan)));
        s->spans_cap = spans.size();
    }
    MP_HIP_CHECK(hipMemcpyAsync(s->spans, spans.data(), spans.size() * sizeof(SeqSpan), hipMemcpyHostToDevice, st));

    ScanArgs a;
    a.g2 = g->g2; a.gexc = g->gexc; a.ginv = g->ginv;
    a.xr_start = g->xr_start; a.xr_char = g->xr_char; a.n_xr = g->n_xr;
    a.seq_base = g->d_base; a.seq_len = g->d_len;
    a.spans = s->spans; a.n_spans = (uint32_t)spans.size();
    a.filt = t->filt; a.filt_log2 = t->filt_log2; a.filt_direct = t->filt_direct;
    a.slots = t->slots; a.slot_log2 = t->slot_log2;
    a.boff = t->boff; a.blist = t->blist; a.recs = t->recs; a.rank = t->rank;
    a.planes = t->planes; a.pchars = t->pchars;
    a.W = t->prm.wordsize; a.M = t->prm.margin; a.N = t->prm.mismatches;
    a.X = t->prm.three_prime_match; a.I = t->prm.iupac_mode;
    a.g_lo = g_lo; a.g_hi = g_hi;

    unsigned long long cnt[2] = {0, 0};
    for (int attempt = 0; attempt < 2; ++attempt) {
        a.hit_hi = s->keys;
        a.hit_lo = s->keys + s->cap;
        a.counters = s->counters;
        a.cap = s->cap;
        MP_HIP_CHECK(hipMemsetAsync(s->counters, 0, 16, st));
        MP_HIP_CHECK(hipEventRecord(s->ev0, st));
        hipLaunchKernelGGL(scan_kernel, dim3((uint32_t)tiles), dim3(kBlock), 0, st, a);
        MP_HIP_CHECK(hipGetLastError());
        MP_HIP_CHECK(hipEventRecord(s->ev1, st));
        MP_HIP_CHECK(hipMemcpyAsync(cnt, s->counters, 16, hipMemcpyDeviceToHost, st));
        MP_HIP_CHECK(hipStreamSynchronize(st));
        if (cnt[0] <= s->cap) break;
        int rc = alloc_hits(s, cnt[0] + cnt[0] / 4 + 1024);
        if (rc) return rc;
    }
    if (cnt[0] > s->cap) return fail(MP_E_STATE, "mp_search_run: hit buffer overflow after growth");
    MP_HIP_CHECK(hipEventElapsedTime(&s->scan_ms, s->ev0, s->ev1));
    s->n_candidates = cnt[1];
    const uint64_t nh = cnt[0];
    int rc = sort_hits(s, nh, st);
    if (rc) return rc;
    if (nh) {
        const uint32_t blocks = (uint32_t)((nh + 255) / 256);
        hipLaunchKernelGGL(decode_kernel, dim3(blocks), dim3(256), 0, st, s->keys, s->keys + s->cap, nh,
                           g->d_base, g->d_len, g->n_seq, t->inv_rank, t->recs, s->out);
        MP_HIP_CHECK(hipGetLastError());
    }
    MP_HIP_CHECK(hipStreamSynchronize(st));
    s->n_hits = nh;
    if (n_hits) *n_hits = nh;
    return MP_OK;
}

MP_EXPORT int mp_search_fetch(void* search, mp_hit* out, uint64_t cap, void* stream) {
    Search* s = (Search*)search;
    if (!s || (s->n_hits && !out)) return fail(MP_E_ARG, "mp_search_fetch: null pointer");
    if (cap < s->n_hits) return fail(MP_E_CAP, "mp_search_fetch: output buffer too small");
    if (!s->n_hits) return MP_OK;
    MP_HIP_CHECK(hipSetDevice(s->genome->device));
    MP_HIP_CHECK(hipMemcpyAsync(out, s->out, s->n_hits * sizeof(mp_hit), hipMemcpyDeviceToHost,
                                (hipStream_t)stream));
    MP_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
    return MP_OK;
}

MP_EXPORT int mp_search_fetch_device(void* search, mp_hit* dev_out, uint64_t cap, void* stream) {
    Search* s = (Search*)search;
    if (!s || (s->n_hits && !dev_out)) return fail(MP_E_ARG, "mp_search_fetch_device: null pointer");
    if (cap < s->n_hits) return fail(MP_E_CAP, "mp_search_fetch_device: output buffer too small");
    if (!s->n_hits) return MP_OK;
    MP_HIP_CHECK(hipSetDevice(s->genome->device));
    MP_HIP_CHECK(hipMemcpyAsync(dev_out, s->out, s->n_hits * sizeof(mp_hit), hipMemcpyDeviceToDevice,
                                (hipStream_t)stream));
    return MP_OK;
}

MP_EXPORT int mp_search_device_hits(void* search, const mp_hit** dev_hits) {
    Search* s = (Search*)search;
    if (!s || !dev_hits) return fail(MP_E_ARG, "mp_search_device_hits: null pointer");
    *dev_hits = s->out;
    return MP_OK;
}

MP_EXPORT int mp_search_last_stats(void* search, float* scan_ms, uint64_t* n_windows, uint64_t* n_candidates) {
    Search* s = (Search*)search;
    if (!s) return fail(MP_E_ARG, "mp_search_last_stats: null search");
    if (scan_ms) *scan_ms = s->scan_ms;
    if (n_windows) *n_windows = s->n_windows;
    if (n_candidates) *n_candidates = s->n_candidates;
    return MP_OK;
}

MP_EXPORT void mp_search_destroy(void* search) { free_search((Search*)search); }
