// Device hit order, the common case: a bucket sort on the device hit count, fused
// with decode (no rocPRIM here, so the first search loads a small code object; the
// rocPRIM fallbacks live in mp_sort.hip).
//
// The reference's output order (the stable sort on pos1 at src/merpcr/core/engine.py:434
// applied to discovery order) is the lexicographic order (sequence, k, hash_offset,
// record, try rank) -- SURVEY 8a-8 -- packed here into one 64-bit key.
#include <algorithm>

#include "mp_internal.h"

namespace mp {

static unsigned bits_for(uint64_t v) {
    unsigned b = 1;
    while (b < 64 && (v >> b)) ++b;
    return b;
}

// ---------------------------------------------------------------- device-count bucket sort
// The common case (the order key fits 64 bits) sorts without the host knowing the hit
// count: pair_kernel counts every key's bucket as it writes it, so the sort follows it on
// the stream with no host round trip.  Keys are bucketed by their top bits (global k:
// hits spread over the genome), counted, scattered, and each bucket is ranked in LDS by
// one workgroup that writes the decoded mp_hit records straight to the output.  A bucket
// larger than kSortCap (hits piled on a few positions, e.g. a dense repeat) sets
// h_out[kSortOverflow]; the host then sorts with rocPRIM instead.
constexpr uint32_t kSortCap = 2048;
constexpr uint32_t kRankCap = 256;  // buckets over this are "crowded" (bitonic, one workgroup each)
constexpr unsigned kMaxBucketBits = 16;

// Exclusive scan of the bucket counts by one 1024-thread workgroup (bucket_offsets_block,
// mp_internal.h).  With h_out it is also the run's finish (finish_fold): pair_kernel, the
// last producer of the counters, is complete, so they go to the device-mapped host words the
// host polls, the hit-region counts to rcount for the scatter, and every counter is zeroed
// for the next run (the sort after it reports an overflow straight to h_out[kSortOverflow]).
__global__ __launch_bounds__(1024) void bucket_offsets(const uint32_t* __restrict__ cnt, uint32_t nb,
                                                       uint32_t* __restrict__ off, uint32_t* __restrict__ cursor,
                                                       unsigned long long* __restrict__ counters, uint32_t n_words,
                                                       unsigned long long* __restrict__ h_out,
                                                       unsigned long long* __restrict__ rcount,
                                                       uint32_t* __restrict__ crowded) {
    __shared__ uint4 s_v4[kOffTile / 4];
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_crowd;
    if (threadIdx.x == 0) s_crowd = 0;
    if (h_out) finish_fold(counters, n_words, h_out, rcount);
    __syncthreads();
    // the crowded buckets (kRankCap < keys <= kSortCap) for crowded_sort_decode
    bucket_offsets_block(cnt, nb, off, cursor, s_v4, s_w, crowded, &s_crowd, kRankCap, kSortCap);
    __syncthreads();
    if (threadIdx.x == 0) crowded[0] = s_crowd;  // the previous run's sort is complete (stream order)
}

// A bucket the device order cannot hold: flagged in the host word (the device counters are
// already zeroed for the next run).
__device__ __forceinline__ void flag_overflow(unsigned long long* h_out) {
    __hip_atomic_store(&h_out[kSortOverflow], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The keys of every hit-list region (its first min(rcount[x], cap_r) slots) into bucket order.
__global__ void bucket_scatter(const uint64_t* __restrict__ keys, const unsigned long long* __restrict__ rcount,
                               uint64_t cap_r, unsigned shift, uint32_t* __restrict__ cursor, uint64_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint32_t x = 0; x < (uint32_t)kHitRegions; ++x)
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u), n = rcount[x] < cap_r ? rcount[x] : cap_r;
         base < n; base += stride) {
        const uint64_t i = base + (uint64_t)lane;
        const bool on = i < n;
        const uint64_t key = on ? keys[x * cap_r + i] : 0ull;
        const uint32_t b = on ? (uint32_t)(key >> shift) : 0xFFFFFFFFu;
        uint32_t head, len;
        bucket_runs(b, on, lane, head, len);
        uint32_t pos = 0;
        if (on && head == (uint32_t)lane) pos = atomicAdd(&cursor[b], len);
        pos = (uint32_t)__shfl((int)pos, (int)head, 64) + ((uint32_t)lane - head);
        if (on) out[pos] = key;
    }
}

// The last sequence whose base is <= gk, found by the whole wave (every lane active, gk
// wave-uniform): a 64-ary search, one parallel load per level -- one level for up to 64
// sequences (c3-c5: 24), two up to 4,096.
__device__ inline uint32_t wave_seq_find(const uint64_t* __restrict__ seq_base, uint32_t n_seq, uint64_t gk,
                                         uint32_t lane) {
    uint32_t lo = 0, n = n_seq;  // the answer lies in [lo, lo + n); seq_base[lo] <= gk (seq_base[0] = 0)
    while (n > 64) {
        const uint32_t step = (n + 63) / 64;
        const uint32_t idx = lo + lane * step;
        const bool le = lane * step < n && seq_base[idx] <= gk;
        const uint32_t c = (uint32_t)__popcll(__ballot(le));  // >= 1: lane 0 holds seq_base[lo]
        lo += (c - 1) * step;
        n = min(step, n - (c - 1) * step);
    }
    const bool le = lane < n && seq_base[lo + lane] <= gk;
    return lo + (uint32_t)__popcll(__ballot(le)) - 1u;
}

// The sequences [lo, hi] that the global positions of bucket b's keys can fall in (keys of
// bucket b are [b << shift, (b << shift) | (2^shift - 1)], positions are key >> low_bits):
// the per-hit search is then over that range, usually one sequence, instead of a binary
// search over seq_base with five dependent loads per hit (c4's order stage: 1.6M hits).
struct SeqRange {
    uint32_t lo, hi;
};
__device__ inline SeqRange bucket_seqs(uint32_t b, unsigned shift, unsigned low_bits,
                                       const uint64_t* __restrict__ seq_base, uint32_t n_seq, uint32_t lane) {
    const uint64_t k0 = (uint64_t)b << shift, k1 = k0 | ((1ull << shift) - 1ull);
    return SeqRange{wave_seq_find(seq_base, n_seq, k0 >> low_bits, lane), wave_seq_find(seq_base, n_seq, k1 >> low_bits, lane)};
}

// The decoded record of one key, written at its sorted slot (as decode_kernel does); its
// sequence is searched within sr (bucket_seqs).
__device__ inline void decode_hit(uint64_t key, uint64_t slot, unsigned try_bits, unsigned low_bits,
                                  const uint64_t* __restrict__ seq_base, const uint64_t* __restrict__ seq_len,
                                  SeqRange sr, const uint2* __restrict__ rank_rec,
                                  mp_hit* __restrict__ out) {
    const uint64_t gk = key >> low_bits;
    const uint32_t rank = (uint32_t)((key & ((1ull << low_bits) - 1ull)) >> try_bits);
    const uint32_t tr = (uint32_t)(key & ((1ull << try_bits) - 1ull));
    uint32_t a = sr.lo, b = sr.hi + 1u;  // last sequence with base <= gk
    while (b - a > 1) {
        const uint32_t mid = (a + b) >> 1;
        if (seq_base[mid] <= gk) a = mid;
        else b = mid;
    }
    const uint64_t k = gk - seq_base[a];
    const uint2 rr = rank_rec[rank];  // {record, size}: one load, not inv_rank then the record
    const uint32_t rec = rr.x;
    const uint64_t len = seq_len[a];
    const uint64_t size = rr.y;
    const uint64_t e = size > len - k ? len - k : size;
    mp_hit h;
    h.pos1 = k;
    h.pos2 = (uint64_t)((int64_t)(k + e) - 1 + try_offset(tr));
    h.seq = a;
    h.rec = rec;
    out[slot] = h;
}

// kBucketsPerBlock buckets per 256-thread workgroup.  A bucket of at most 64 keys (the common
// case: ~32 per bucket at capacity) is ranked by its own wave, counting the smaller keys
// (unique: one hit per (k, record, try)) over shuffles.  The workgroup then takes the larger
// ones up to 256 keys one after another, ranking by counting through LDS.  Buckets over 256
// (c4: IUPAC primers over N runs pile up to 2,048 hits on a position) go to the crowded list
// for crowded_sort_decode, one 1024-thread workgroup each: a 256-thread workgroup sorting
// them one after another (bitonic, 66 barrier stages for 2,048 keys) made the longest
// workgroup of this kernel the order stage's critical path.  (One workgroup per bucket left
// c4's 65,536 workgroups of ~24 keys dispatch-bound: 94 us.)
constexpr uint32_t kBucketsPerBlock = 4;
__global__ __launch_bounds__(256) void bucket_sort_decode(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ off,
                                                          uint32_t nb, unsigned shift, unsigned try_bits, unsigned low_bits,
                                                          const uint64_t* __restrict__ seq_base,
                                                          const uint64_t* __restrict__ seq_len, uint32_t n_seq,
                                                          const uint2* __restrict__ rank_rec,
                                                          mp_hit* __restrict__ out, unsigned long long* __restrict__ h_out,
                                                          uint32_t* __restrict__ crowded) {
    __shared__ uint64_t s_k[kRankCap];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t b0 = blockIdx.x * kBucketsPerBlock;
    {
        const bool in = b0 + wave < nb;  // nb < kBucketsPerBlock under a forced sort_bucket_bits
        const uint32_t start = in ? off[b0 + wave] : 0u, m = in ? off[b0 + wave + 1] - start : 0u;
        if (m > kSortCap && lane == 0) flag_overflow(h_out);
        if (m > 0 && m <= 64) {  // wave-uniform; no barrier inside
            const uint64_t key = lane < m ? keys[start + lane] : ~0ull;
            uint32_t r = 0;
            for (uint32_t j = 0; j < m; ++j) {
                const uint64_t kj = __shfl(key, (int)j, 64);
                r += kj < key || (kj == key && j < lane);  // ties: stable
            }
            const SeqRange sr = bucket_seqs(b0 + wave, shift, low_bits, seq_base, n_seq, lane);
            if (lane < m) decode_hit(key, start + r, try_bits, low_bits, seq_base, seq_len, sr, rank_rec, out);
        }
        if (!__syncthreads_or(m > 64 && m <= kRankCap)) return;  // every wave reaches this barrier
    }
    for (uint32_t q = 0; q < kBucketsPerBlock && b0 + q < nb; ++q) {  // block-uniform loop
        const uint32_t start = off[b0 + q], m = off[b0 + q + 1] - start;
        if (m <= 64 || m > kRankCap) continue;  // done by its wave above / crowded_sort_decode
        for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) s_k[i] = keys[start + i];
        const SeqRange sr = bucket_seqs(b0 + q, shift, low_bits, seq_base, n_seq, lane);  // every lane of every wave
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
            const uint64_t key = s_k[i];
            uint32_t r = 0;
            for (uint32_t j = 0; j < m; ++j) r += s_k[j] < key || (s_k[j] == key && j < i);  // ties: stable
            decode_hit(key, start + r, try_bits, low_bits, seq_base, seq_len, sr, rank_rec, out);
        }
        __syncthreads();  // s_k is refilled by the next bucket
    }
}

// One in-wave bitonic compare-exchange stage (j <= 32) on a lane's two keys: e0 at index
// i0 = base + lane, e1 at i0 + 64; partners by shuffle, direction from bit k of the index.
__device__ __forceinline__ uint64_t cx_lane(uint64_t e, uint32_t i, uint32_t j, uint32_t k) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)e, (int)j, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(e >> 32), (int)j, 64);
    const uint64_t o = ((uint64_t)hi << 32) | lo;
    const bool up = (i & k) == 0, lower = (i & j) == 0;
    return (lower == up) ? (e < o ? e : o) : (e > o ? e : o);
}

// The crowded buckets (kRankCap < keys <= kSortCap) of a mode-1 run, one per 1024-thread
// workgroup (persistent over the list): bitonic sort of the bucket padded to a power of two.
// Wave w holds keys [128 w, 128 w + 128) in registers, two per lane (i and i + 64): every
// stage with j <= 64 is a register compare or a shuffle, and only the stages with j >= 128
// (10 of the 66 for 2,048 keys) go through LDS with a barrier each.  (All 66 through LDS,
// one barrier each: c4's crowded buckets took 109 us.)
// One crowded bucket b (kRankCap < keys <= kSortCap) sorted and decoded by the whole
// 1024-thread workgroup (s_k: kSortCap keys of LDS).
__device__ __forceinline__ void crowded_bucket(uint32_t b, uint64_t* s_k, const uint64_t* __restrict__ keys,
                                               const uint32_t* __restrict__ off, unsigned shift, unsigned try_bits,
                                               unsigned low_bits, const uint64_t* __restrict__ seq_base,
                                               const uint64_t* __restrict__ seq_len, uint32_t n_seq,
                                               const uint2* __restrict__ rank_rec, mp_hit* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u, base = (threadIdx.x >> 6) * 128u;
    const uint32_t i0 = base + lane, i1 = i0 + 64u;
    const uint32_t start = off[b], m = off[b + 1] - start;
    uint32_t P = 2 * kRankCap;
    while (P < m) P <<= 1;
    const bool on = base < P;  // wave-uniform: this wave holds keys of the padded bucket
    uint64_t e0 = i0 < m ? keys[start + i0] : ~0ull, e1 = i1 < m ? keys[start + i1] : ~0ull;
    for (uint32_t k = 2; k <= P; k <<= 1) {
        if (k > 128u) {  // stages j >= 128 across waves, through LDS
            if (on) {
                s_k[i0] = e0;
                s_k[i1] = e1;
            }
            __syncthreads();
            for (uint32_t j = k >> 1; j >= 128u; j >>= 1) {
                for (uint32_t t = threadIdx.x; t < P / 2; t += blockDim.x) {
                    const uint32_t i = ((t & ~(j - 1)) << 1) | (t & (j - 1));  // the pair's lower index
                    const uint32_t ij = i | j;
                    const uint64_t x = s_k[i], y = s_k[ij];
                    if ((x > y) == ((i & k) == 0)) {
                        s_k[i] = y;
                        s_k[ij] = x;
                    }
                }
                __syncthreads();
            }
            if (on) {
                e0 = s_k[i0];
                e1 = s_k[i1];
            }
            __syncthreads();  // every wave has read before the next k writes
        }
        if (on) {
            if (k >= 128u) {  // j = 64: the lane's own two keys (i0 is the lower index)
                const bool up = (i0 & k) == 0;
                const uint64_t lo = e0 < e1 ? e0 : e1, hi = e0 < e1 ? e1 : e0;
                e0 = up ? lo : hi;
                e1 = up ? hi : lo;
            }
            for (uint32_t j = (k >> 1) < 32u ? (k >> 1) : 32u; j > 0; j >>= 1) {
                e0 = cx_lane(e0, i0, j, k);
                e1 = cx_lane(e1, i1, j, k);
            }
        }
    }
    if (on) {
        const SeqRange sr = bucket_seqs(b, shift, low_bits, seq_base, n_seq, lane);
        if (i0 < m) decode_hit(e0, start + i0, try_bits, low_bits, seq_base, seq_len, sr, rank_rec, out);
        if (i1 < m) decode_hit(e1, start + i1, try_bits, low_bits, seq_base, seq_len, sr, rank_rec, out);
    }
}

__global__ __launch_bounds__(1024) void crowded_sort_decode(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ off,
                                                            unsigned shift, unsigned try_bits, unsigned low_bits,
                                                            const uint64_t* __restrict__ seq_base,
                                                            const uint64_t* __restrict__ seq_len, uint32_t n_seq,
                                                            const uint2* __restrict__ rank_rec,
                                                            mp_hit* __restrict__ out, const uint32_t* __restrict__ crowded) {
    __shared__ uint64_t s_k[kSortCap];
    static_assert(kSortCap == 2 * 1024, "two keys per thread of the 1024-thread workgroup");
    const uint32_t n = crowded[0];
    for (uint32_t c = blockIdx.x; c < n; c += gridDim.x)  // block-uniform
        crowded_bucket(crowded[1 + c], s_k, keys, off, shift, try_bits, low_bits, seq_base, seq_len, n_seq, rank_rec, out);
}

// Order mode 0: pair_kernel left every bucket's keys in its slot (bucket b at b * slot_cap,
// in arrival order) and, from its last block, the bucket offsets.  One wave per bucket ranks
// the bucket's keys -- up to 64 by shuffles, up to slot_cap by counting through the wave's
// LDS -- and writes the decoded records at off[b] + rank.  No scatter pass, no block barrier.
// A bucket over slot_cap (its keys did not all fit) sets h_out[kSortOverflow]; the host
// then orders the run in mode 1 from the linear keys.
constexpr uint32_t kSlotWaves = 4;
__global__ __launch_bounds__(64 * kSlotWaves) void sort_decode_slots(
    const uint64_t* __restrict__ slots, uint32_t slot_cap, const uint32_t* __restrict__ off, uint32_t nb,
    unsigned shift, unsigned try_bits, unsigned low_bits, const uint64_t* __restrict__ seq_base, const uint64_t* __restrict__ seq_len,
    uint32_t n_seq, const uint2* __restrict__ rank_rec, mp_hit* __restrict__ out,
    unsigned long long* __restrict__ h_out) {
    __shared__ uint64_t s_k[kSlotWaves][kSlotCap];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t b = blockIdx.x * kSlotWaves + wave;
    if (b >= nb) return;  // wave-uniform, and no block barrier follows
    const uint32_t start = off[b], m = off[b + 1] - start;
    if (m == 0) return;
    if (m > slot_cap) {
        if (lane == 0) flag_overflow(h_out);
        return;
    }
    const uint64_t* src = slots + (uint64_t)b * slot_cap;
    const SeqRange sr = bucket_seqs(b, shift, low_bits, seq_base, n_seq, lane);
    if (m <= 64) {
        const uint64_t key = lane < m ? src[lane] : ~0ull;
        uint32_t r = 0;
        for (uint32_t j = 0; j < m; ++j) {
            const uint64_t kj = __shfl(key, (int)j, 64);
            r += kj < key || (kj == key && j < lane);  // ties: stable (keys are unique anyway)
        }
        if (lane < m) decode_hit(key, start + r, try_bits, low_bits, seq_base, seq_len, sr, rank_rec, out);
        return;
    }
    uint64_t* k = s_k[wave];
    for (uint32_t i = lane; i < m; i += 64) k[i] = src[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (uint32_t i = lane; i < m; i += 64) {
        const uint64_t key = k[i];
        uint32_t r = 0;
        for (uint32_t j = 0; j < m; ++j) r += k[j] < key || (k[j] == key && j < i);
        decode_hit(key, start + r, try_bits, low_bits, seq_base, seq_len, sr, rank_rec, out);
    }
}

bool sort_hits_device_ok(const Search* s) {
    const unsigned hi_bits = bits_for(s->genome->total);
    const unsigned try_bits = bits_for(2ull * (uint64_t)std::max(s->table->prm.margin, 0));
    return hi_bits + s->table->rank_bits + try_bits <= 64 && (s->opt.sort == MP_SORT_AUTO || s->opt.sort == MP_SORT_SCATTER);
}

int alloc_sort_buckets(Search* s) {
    // counts, nb + 1 offsets, cursors, then the hit-region counts (16-B aligned)
    // + the crowded list: its count and up to 2^kMaxBucketBits bucket indices
    if (!s->bucket) MP_HIP_CHECK(hipMalloc(&s->bucket, (3ull << kMaxBucketBits) * 4 + 16 + kHitRegions * 8 +
                                                           4 * ((1ull << kMaxBucketBits) + 1)));
    return MP_OK;
}

SortPlan sort_plan(const Search* s) {
    SortPlan P;
    const unsigned hi_bits = bits_for(s->genome->total);
    P.try_bits = bits_for(2ull * (uint64_t)std::max(s->table->prm.margin, 0));
    P.low_bits = s->table->rank_bits + P.try_bits;
    const unsigned key_bits = hi_bits + P.low_bits;
    // ~32 hits per bucket at the buffer's capacity (the count is not known on the host)
    unsigned bb = bits_for(s->cap / 32);
    bb = std::min(std::max(bb, 6u), kMaxBucketBits);
    if (s->opt.sort_bucket_bits > 0) bb = std::min((unsigned)s->opt.sort_bucket_bits, kMaxBucketBits);
    bb = std::min(bb, key_bits);
    P.shift = key_bits - bb;
    P.nb = 1u << bb;
    P.slot_cap = kSlotCap;
    return P;
}

uint32_t* sort_bucket_counts(Search* s) { return s->bucket; }
uint32_t* sort_bucket_offsets(Search* s) { return s->bucket + (1u << kMaxBucketBits); }
uint32_t* sort_bucket_cursors(Search* s) { return s->bucket + 2 * (1u << kMaxBucketBits) + 1; }
unsigned long long* sort_region_counts(Search* s) {
    return reinterpret_cast<unsigned long long*>(s->bucket + 3 * (1u << kMaxBucketBits) + 4);
}
uint32_t* sort_crowded(Search* s) { return s->bucket + 3 * (1u << kMaxBucketBits) + 4 + 2 * kHitRegions; }

int alloc_sort_slots(Search* s, const SortPlan& P) {
    const size_t need = (size_t)P.nb * P.slot_cap * sizeof(uint64_t);
    if (need <= s->slots_bytes) return MP_OK;
    hipFree(s->slots);
    s->slots = nullptr;
    s->slots_bytes = 0;
    MP_HIP_CHECK(hipMalloc(&s->slots, need));
    s->slots_bytes = need;
    return MP_OK;
}

int sort_hits_device(Search* s, hipStream_t st, int mode, bool finish) {
    const SortPlan P = sort_plan(s);
    const int arc = alloc_sort_buckets(s);
    if (arc) return arc;
    uint32_t* off = sort_bucket_offsets(s);
    uint32_t* cursor = sort_bucket_cursors(s);
    const Genome* g = s->genome;
    // A separate launch, not pair_kernel's last block: publishing the counts inside the pair
    // kernel needs an agent-scope release per block (buffer_wbl2 of the XCD's L2, several
    // us each across the persistent grid), measured +65 us on a 1/8 c3 step.
    hipLaunchKernelGGL(bucket_offsets, dim3(1), dim3(1024), 0, st, sort_bucket_counts(s), P.nb, off, cursor,
                       s->counters, (uint32_t)(counter_bytes() / 8), finish ? s->d_hcnt : nullptr, sort_region_counts(s),
                       sort_crowded(s));
    MP_HIP_CHECK(hipGetLastError());
    if (mode == 0) {
        hipLaunchKernelGGL(sort_decode_slots, dim3((P.nb + kSlotWaves - 1) / kSlotWaves), dim3(64 * kSlotWaves), 0, st,
                           s->slots, P.slot_cap, off, P.nb, P.shift, P.try_bits, P.low_bits, g->d_base, g->d_len, g->n_seq,
                           s->table->rank_rec, s->out, s->d_hcnt);
        MP_HIP_CHECK(hipGetLastError());
        return MP_OK;
    }
    const uint32_t grid = (uint32_t)std::min<uint64_t>((s->cap + 255) / 256, 2048);
    hipLaunchKernelGGL(bucket_scatter, dim3(grid), dim3(256), 0, st, s->tmp_lo, sort_region_counts(s),
                       s->cap / kHitRegions, P.shift, cursor, s->tmp_hi);
    MP_HIP_CHECK(hipGetLastError());
    // crowded buckets: MP_CROWD_GRID workgroups (tuning; default one per CU)
    static const uint32_t crowd_grid = [] {
        const char* e = std::getenv("MP_CROWD_GRID");
        return e ? (uint32_t)std::max(1, std::atoi(e)) : 0u;
    }();
    const uint32_t cg = crowd_grid ? crowd_grid : (uint32_t)s->n_cu;
    hipLaunchKernelGGL(bucket_sort_decode, dim3((P.nb + kBucketsPerBlock - 1) / kBucketsPerBlock), dim3(256), 0, st,
                       s->tmp_hi, off, P.nb, P.shift, P.try_bits, P.low_bits,
                       g->d_base, g->d_len, g->n_seq, s->table->rank_rec, s->out, s->d_hcnt, sort_crowded(s));
    MP_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(crowded_sort_decode, dim3(cg), dim3(1024), 0, st, s->tmp_hi, off, P.shift, P.try_bits,
                       P.low_bits, g->d_base, g->d_len, g->n_seq, s->table->rank_rec, s->out,
                       sort_crowded(s));
    MP_HIP_CHECK(hipGetLastError());
    return MP_OK;
}

}  // namespace mp
