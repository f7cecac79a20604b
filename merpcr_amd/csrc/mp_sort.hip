// Device sorts (rocPRIM radix sort; kept in its own translation unit because of
// its compile time).
//
// sort_hits puts the raw hits of a run into the reference's output order: the
// stable sort on pos1 at src/merpcr/core/engine.py:434 applied to discovery
// order is the lexicographic order (sequence, k, hash_offset, record, try rank)
// -- SURVEY 8a-8.  Hits carry it as a 128-bit key (hi = global k coordinate,
// lo = rank(record) << 32 | try rank) and two stable LSD passes order them.
#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>

#include "mp_internal.h"

namespace mp {

static unsigned bits_for(uint64_t v) {
    unsigned b = 1;
    while (b < 64 && (v >> b)) ++b;
    return b;
}

static int ensure_tmp(void** p, size_t* have, size_t need) {
    if (need <= *have) return MP_OK;
    hipFree(*p);
    *p = nullptr;
    *have = 0;
    MP_HIP_CHECK(hipMalloc(p, need));
    *have = need;
    return MP_OK;
}

// Slot j of hit-list region x (j < rcount[x], kHitBase) -> its place in the compacted list
// (regions in order); -1 past the region's count.
__device__ __forceinline__ int64_t compact_index(const unsigned long long* __restrict__ rcount, uint64_t cap_r,
                                                 uint64_t slot) {
    const uint32_t x = (uint32_t)(slot / cap_r);
    const uint64_t j = slot - (uint64_t)x * cap_r;
    uint64_t pre = 0;
    for (uint32_t y = 0; y < x; ++y) pre += rcount[y];
    return j < rcount[x] ? (int64_t)(pre + j) : -1;
}

// (k, record rank, try rank) of every hit in one 64-bit key, most significant first, into
// the compacted list.
__global__ void pack_keys(const uint64_t* __restrict__ hi, const uint64_t* __restrict__ lo,
                          const unsigned long long* __restrict__ rcount, uint64_t cap_r, unsigned try_bits,
                          unsigned low_bits, uint64_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cap_r * kHitRegions) return;
    const int64_t c = compact_index(rcount, cap_r, i);
    if (c < 0) return;
    const uint64_t l = lo[i];
    out[c] = (hi[i] << low_bits) | ((l >> 32) << try_bits) | (l & 0xFFFFFFFFull);
}

// The regions' (hi, lo) pairs into the compacted list.
__global__ void compact_hits(const uint64_t* __restrict__ hi, const uint64_t* __restrict__ lo,
                             const unsigned long long* __restrict__ rcount, uint64_t cap_r,
                             uint64_t* __restrict__ ohi, uint64_t* __restrict__ olo) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cap_r * kHitRegions) return;
    const int64_t c = compact_index(rcount, cap_r, i);
    if (c < 0) return;
    ohi[c] = hi[i];
    olo[c] = lo[i];
}

__global__ void unpack_keys(const uint64_t* __restrict__ key, uint64_t n, unsigned try_bits, unsigned low_bits,
                            uint64_t* __restrict__ hi, uint64_t* __restrict__ lo) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = key[i];
    hi[i] = k >> low_bits;
    lo[i] = (((k & ((1ull << low_bits) - 1ull)) >> try_bits) << 32) | (k & ((1ull << try_bits) - 1ull));
}


int sort_hits(Search* s, uint64_t n, hipStream_t st, const uint64_t** hi_out, const uint64_t** lo_out) {
    uint64_t* hi = s->keys;
    uint64_t* lo = s->keys + s->cap;
    *hi_out = hi;
    *lo_out = lo;
    if (n == 0) return MP_OK;
    // the hits sit in kHitRegions regions of cap_r slots (pair_kernel); every pass below
    // works on the compacted list of n
    const uint64_t cap_r = s->cap / kHitRegions;
    const unsigned long long* rcount = sort_region_counts(s);
    const unsigned cblocks = (unsigned)((s->cap + 255) / 256);
    const unsigned lo_bits = 32 + s->table->rank_bits;
    const unsigned hi_bits = bits_for(s->genome->total);
    // try ranks are <= 2M (engine.py:540-560: d in [-M, M])
    const unsigned try_bits = bits_for(2ull * (uint64_t)std::max(s->table->prm.margin, 0));
    const unsigned low_bits = s->table->rank_bits + try_bits;
    if (hi_bits + low_bits <= 64 && s->opt.sort != MP_SORT_RADIX128) {
        // the whole order key fits 64 bits: one keys-only radix sort
        const unsigned blocks = (unsigned)((n + 255) / 256);
        hipLaunchKernelGGL(pack_keys, dim3(cblocks), dim3(256), 0, st, hi, lo, rcount, cap_r, try_bits, low_bits, s->tmp_lo);
        MP_HIP_CHECK(hipGetLastError());
        size_t need = 0;
        MP_HIP_CHECK(rocprim::radix_sort_keys(nullptr, need, s->tmp_lo, s->tmp_hi, (size_t)n, 0, hi_bits + low_bits, st));
        int rc = ensure_tmp(&s->sort_tmp, &s->sort_tmp_bytes, need);
        if (rc) return rc;
        size_t b = s->sort_tmp_bytes;
        MP_HIP_CHECK(rocprim::radix_sort_keys(s->sort_tmp, b, s->tmp_lo, s->tmp_hi, (size_t)n, 0, hi_bits + low_bits, st));
        hipLaunchKernelGGL(unpack_keys, dim3(blocks), dim3(256), 0, st, s->tmp_hi, n, try_bits, low_bits, hi, lo);
        MP_HIP_CHECK(hipGetLastError());
        return MP_OK;
    }
    hipLaunchKernelGGL(compact_hits, dim3(cblocks), dim3(256), 0, st, hi, lo, rcount, cap_r, s->tmp_hi, s->tmp_lo);
    MP_HIP_CHECK(hipGetLastError());
    size_t need1 = 0, need2 = 0;
    MP_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, need1, s->tmp_lo, lo, s->tmp_hi, hi, (size_t)n,
                                           0, lo_bits, st));
    MP_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, need2, hi, s->tmp_hi, lo, s->tmp_lo, (size_t)n,
                                           0, hi_bits, st));
    int rc = ensure_tmp(&s->sort_tmp, &s->sort_tmp_bytes, std::max(need1, need2));
    if (rc) return rc;
    size_t b1 = s->sort_tmp_bytes, b2 = s->sort_tmp_bytes;
    // pass 1: by lo (record rank, try rank), carrying hi
    MP_HIP_CHECK(rocprim::radix_sort_pairs(s->sort_tmp, b1, s->tmp_lo, lo, s->tmp_hi, hi, (size_t)n,
                                           0, lo_bits, st));
    // pass 2: stable by hi (global k), carrying lo; the result in (tmp_hi, tmp_lo)
    MP_HIP_CHECK(rocprim::radix_sort_pairs(s->sort_tmp, b2, hi, s->tmp_hi, lo, s->tmp_lo, (size_t)n,
                                           0, hi_bits, st));
    *hi_out = s->tmp_hi;
    *lo_out = s->tmp_lo;
    return MP_OK;
}

// Exception runs may be appended out of order by separate puts: order them by start.
int sort_runs(Genome* g, hipStream_t st) {
    const uint64_t n = g->n_xr;
    if (n < 2) return MP_OK;
    uint64_t* ks = nullptr;
    uint8_t* vs = nullptr;
    void* tmp = nullptr;
    size_t tb = 0;
    int rc = MP_OK;
    do {
        if (hipMalloc(&ks, n * 8) != hipSuccess || hipMalloc(&vs, n) != hipSuccess) {
            rc = fail(MP_E_NOMEM, "sort_runs: allocation failed");
            break;
        }
        const unsigned kb = bits_for(g->total);
        if (rocprim::radix_sort_pairs(nullptr, tb, g->xr_start, ks, g->xr_char, vs, (size_t)n, 0, kb, st) !=
                hipSuccess ||
            hipMalloc(&tmp, tb) != hipSuccess ||
            rocprim::radix_sort_pairs(tmp, tb, g->xr_start, ks, g->xr_char, vs, (size_t)n, 0, kb, st) !=
                hipSuccess ||
            hipMemcpyAsync(g->xr_start, ks, n * 8, hipMemcpyDeviceToDevice, st) != hipSuccess ||
            hipMemcpyAsync(g->xr_char, vs, n, hipMemcpyDeviceToDevice, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {
            rc = fail(MP_E_HIP, "sort_runs: device sort failed");
        }
    } while (0);
    hipFree(ks);
    hipFree(vs);
    hipFree(tmp);
    return rc;
}

}  // namespace mp
