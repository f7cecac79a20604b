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
// Buckets of more than kRankCap keys are "crowded" (crowded_sort_decode): up to kWaveSortCap
// keys a wave sorts in its registers (wave_bitonic), larger ones the whole workgroup (bitonic
// through LDS).
constexpr uint32_t kRankCap = 256;
constexpr uint32_t kWaveSortCap = 1024;
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

// One in-wave bitonic compare-exchange stage (j <= 32) on a lane's two keys: e0 at index
// i0 = base + lane, e1 at i0 + 64; partners by shuffle, direction from bit k of the index.
__device__ __forceinline__ uint64_t cx_lane(uint64_t e, uint32_t i, uint32_t j, uint32_t k) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)e, (int)j, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(e >> 32), (int)j, 64);
    const uint64_t o = ((uint64_t)hi << 32) | lo;
    const bool up = (i & k) == 0, lower = (i & j) == 0;
    return (lower == up) ? (e < o ? e : o) : (e > o ? e : o);
}

// The value lane ^ J holds (J < 64, a compile-time constant), without the LDS crossbar where a
// VALU permute does it: DPP quad permutes for J = 1, 2; a half-row mirror then a reversed quad
// (lane ^ 7 ^ 3) for J = 4; a row rotate by 8 for J = 8; the swizzle unit for J = 16;
// v_permlane32_swap for J = 32 (lanes 32-63 of the first operand swap with lanes 0-31 of the
// second: with both = v, the first result holds v[lane - 32] in the upper half and the second
// v[lane + 32] in the lower).
template <uint32_t J>
__device__ __forceinline__ uint32_t xor_lane(uint32_t v, uint32_t lane) {
    if constexpr (J == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    else if constexpr (J == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    else if constexpr (J == 4) {
        const int m = __builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
        return (uint32_t)__builtin_amdgcn_update_dpp(0, m, 0x1B, 0xF, 0xF, false);      // quad_perm [3,2,1,0]
    } else if constexpr (J == 8) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    else if constexpr (J == 16) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (16 << 10) | 0x1F);  // xor 16
    else {
        static_assert(J == 32, "lane partner within the wave");
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return lane < 32u ? (uint32_t)r[1] : (uint32_t)r[0];
    }
}

// Bitonic sort (ascending) of the 64 * kR keys one wave holds, kR per lane: element
// i = 64 r + lane is register r of the lane.  Stages with j >= 64 pair two registers of the
// same lane (their direction, bit k >= 128 of i, is the register's); stages with j < 64 pair
// lanes (xor_lane).  No LDS array, no barrier.  Templates over (k, j) unroll every stage, so
// register indices and permute patterns are constants.  (A run-time (k, j) loop over one
// specialised stage per j, 5x less code, took c4's crowded buckets from 54 to 86 us.)
template <int kR, uint32_t K, uint32_t J>
__device__ __forceinline__ void bitonic_stage(uint64_t (&e)[kR], uint32_t lane) {
    if constexpr (J >= 64u) {
        constexpr uint32_t jr = J / 64u;
#pragma unroll
        for (uint32_t r = 0; r < (uint32_t)kR; ++r) {
            if ((r & jr) == 0u) {
                const bool up = ((r * 64u) & K) == 0u;
                const uint64_t x = e[r], y = e[r | jr];
                const uint64_t lo = x < y ? x : y, hi = x < y ? y : x;
                e[r] = up ? lo : hi;
                e[r | jr] = up ? hi : lo;
            }
        }
    } else {
        const bool lower = (lane & J) == 0u;
#pragma unroll
        for (uint32_t r = 0; r < (uint32_t)kR; ++r) {
            const uint64_t o = ((uint64_t)xor_lane<J>((uint32_t)(e[r] >> 32), lane) << 32) | xor_lane<J>((uint32_t)e[r], lane);
            const bool up = ((r * 64u + lane) & K) == 0u;
            e[r] = (lower == up) ? (e[r] < o ? e[r] : o) : (e[r] > o ? e[r] : o);
        }
    }
    if constexpr (J > 1u) bitonic_stage<kR, K, J / 2u>(e, lane);
}

template <int kR, uint32_t K = 2>
__device__ __forceinline__ void wave_bitonic(uint64_t (&e)[kR], uint32_t lane) {
    bitonic_stage<kR, K, K / 2u>(e, lane);
    if constexpr (K < 64u * (uint32_t)kR) wave_bitonic<kR, 2u * K>(e, lane);
}

// One bucket of 64 < m <= 64 kR keys, sorted and decoded by its wave.
template <int kR>
__device__ __forceinline__ void wave_sort_decode(const uint64_t* __restrict__ keys, uint32_t start, uint32_t m,
                                                 uint32_t lane, unsigned try_bits, unsigned low_bits,
                                                 const uint64_t* __restrict__ seq_base, const uint64_t* __restrict__ seq_len,
                                                 SeqRange sr, const uint2* __restrict__ rank_rec, mp_hit* __restrict__ out) {
    uint64_t e[kR];
#pragma unroll
    for (uint32_t r = 0; r < (uint32_t)kR; ++r) e[r] = r * 64u + lane < m ? keys[start + r * 64u + lane] : ~0ull;
    wave_bitonic<kR>(e, lane);
#pragma unroll
    for (uint32_t r = 0; r < (uint32_t)kR; ++r)
        if (r * 64u + lane < m) decode_hit(e[r], start + r * 64u + lane, try_bits, low_bits, seq_base, seq_len, sr, rank_rec, out);
}

// One wave per bucket, kBucketsPerBlock waves per workgroup, no barrier.  A bucket of at most
// 64 keys (the common case: ~32 per bucket at capacity) is ranked by counting the smaller keys
// (unique: one hit per (k, record, try)) over shuffles; up to kRankCap keys by a register
// bitonic sort of 256 slots (wave_bitonic).  Larger buckets are on the crowded list for
// crowded_sort_decode, which keeps the 512- and 1,024-slot register sorts (and their VGPRs)
// out of this kernel's occupancy.  c4 (1.6M hits, ~100 tries of one (k, record) on each of 12k
// positions): 5.6k buckets of 65-256 keys and 1.6k of 257-849.  Round 4 ranked the 65-256 ones
// by counting through LDS (256-thread workgroup per bucket in turn) and sorted the rest with
// 1024-thread bitonic sorts through LDS: 62 + 66 us.  (One workgroup per bucket left c4's
// 65,536 workgroups of ~24 keys dispatch-bound: 94 us.)
constexpr uint32_t kBucketsPerBlock = 4;
__global__ __launch_bounds__(64 * kBucketsPerBlock) void bucket_sort_decode(
    const uint64_t* __restrict__ keys, const uint32_t* __restrict__ off, uint32_t nb, unsigned shift, unsigned try_bits,
    unsigned low_bits, const uint64_t* __restrict__ seq_base, const uint64_t* __restrict__ seq_len, uint32_t n_seq,
    const uint2* __restrict__ rank_rec, mp_hit* __restrict__ out, unsigned long long* __restrict__ h_out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t b = blockIdx.x * kBucketsPerBlock + (threadIdx.x >> 6);
    if (b >= nb) return;  // wave-uniform; no barrier in this kernel
    const uint32_t start = off[b], m = off[b + 1] - start;
    if (m > kSortCap && lane == 0) flag_overflow(h_out);
    if (m == 0 || m > kRankCap) return;  // crowded: crowded_sort_decode
    const SeqRange sr = bucket_seqs(b, shift, low_bits, seq_base, n_seq, lane);
    if (m <= 64) {
        const uint64_t key = lane < m ? keys[start + lane] : ~0ull;
        uint32_t r = 0;
        for (uint32_t j = 0; j < m; ++j) {
            const uint64_t kj = __shfl(key, (int)j, 64);
            r += kj < key || (kj == key && j < lane);  // ties: stable
        }
        if (lane < m) decode_hit(key, start + r, try_bits, low_bits, seq_base, seq_len, sr, rank_rec, out);
    } else {
        static_assert(kRankCap == 256, "4 keys per lane");
        wave_sort_decode<4>(keys, start, m, lane, try_bits, low_bits, seq_base, seq_len, sr, rank_rec, out);
    }
}

// The crowded buckets (kRankCap < keys <= kSortCap) of a mode-1 run.  Up to kWaveSortCap keys:
// one wave each (wave_sort_decode, 512 or 1,024 register slots).  Larger ones: one 1024-thread
// workgroup each (persistent over the list), bitonic sort of the bucket padded to a power of two.
// Wave w holds keys [128 w, 128 w + 128) in registers, two per lane (i and i + 64): every
// stage with j <= 64 is a register compare or a shuffle, and only the stages with j >= 128
// (10 of the 66 for 2,048 keys) go through LDS with a barrier each.  (All 66 through LDS,
// one barrier each: c4's crowded buckets took 109 us.)
// One crowded bucket b (kWaveSortCap < keys <= kSortCap) sorted and decoded by the whole
// 1024-thread workgroup (s_k: kSortCap keys of LDS).
__device__ __forceinline__ void crowded_bucket(uint32_t b, uint64_t* s_k, const uint64_t* __restrict__ keys,
                                               const uint32_t* __restrict__ off, unsigned shift, unsigned try_bits,
                                               unsigned low_bits, const uint64_t* __restrict__ seq_base,
                                               const uint64_t* __restrict__ seq_len, uint32_t n_seq,
                                               const uint2* __restrict__ rank_rec, mp_hit* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u, base = (threadIdx.x >> 6) * 128u;
    const uint32_t i0 = base + lane, i1 = i0 + 64u;
    const uint32_t start = off[b], m = off[b + 1] - start;
    uint32_t P = kWaveSortCap;
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
    // up to kWaveSortCap keys: one wave per bucket, registers only (no barrier in this loop)
    // list items go round-robin over the workgroups first (item c to workgroup c mod grid), so
    // that a short list spreads over every CU (c4: 1.6k items, 256 workgroups of 16 waves;
    // consecutive items per workgroup had filled 102 CUs with 16 sorts each)
    const uint32_t lane = threadIdx.x & 63u, waves = gridDim.x * (blockDim.x / 64u);
    for (uint32_t c = (threadIdx.x >> 6) * gridDim.x + blockIdx.x; c < n; c += waves) {  // wave-uniform
        const uint32_t b = crowded[1 + c], start = off[b], m = off[b + 1] - start;
        if (m > kWaveSortCap) continue;
        const SeqRange sr = bucket_seqs(b, shift, low_bits, seq_base, n_seq, lane);
        if (m <= 512u) wave_sort_decode<8>(keys, start, m, lane, try_bits, low_bits, seq_base, seq_len, sr, rank_rec, out);
        else wave_sort_decode<16>(keys, start, m, lane, try_bits, low_bits, seq_base, seq_len, sr, rank_rec, out);
    }
    static_assert(kWaveSortCap == 1024 && 2 * kRankCap == 512, "8 and 16 keys per lane");
    // larger: the whole workgroup per bucket
    for (uint32_t c = blockIdx.x; c < n; c += gridDim.x) {  // block-uniform
        const uint32_t b = crowded[1 + c];
        if (off[b + 1] - off[b] > kWaveSortCap)
            crowded_bucket(b, s_k, keys, off, shift, try_bits, low_bits, seq_base, seq_len, n_seq, rank_rec, out);
    }
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
    // crowded buckets: mp_search_options.crowd_grid workgroups (tuning; default one per CU)
    const uint32_t cg = s->opt.crowd_grid ? (uint32_t)s->opt.crowd_grid : (uint32_t)s->n_cu;
    hipLaunchKernelGGL(bucket_sort_decode, dim3((P.nb + kBucketsPerBlock - 1) / kBucketsPerBlock), dim3(256), 0, st,
                       s->tmp_hi, off, P.nb, P.shift, P.try_bits, P.low_bits,
                       g->d_base, g->d_len, g->n_seq, s->table->rank_rec, s->out, s->d_hcnt);
    MP_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(crowded_sort_decode, dim3(cg), dim3(1024), 0, st, s->tmp_hi, off, P.shift, P.try_bits,
                       P.low_bits, g->d_base, g->d_len, g->n_seq, s->table->rank_rec, s->out,
                       sort_crowded(s));
    MP_HIP_CHECK(hipGetLastError());
    return MP_OK;
}

}  // namespace mp
