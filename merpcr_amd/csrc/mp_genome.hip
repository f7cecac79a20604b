// Genome residency: pack filtered sequence bytes into the HBM planes.
//
// Stands in for the sequence strings that MerPCR.search walks per record
// (src/merpcr/core/engine.py:373-411, upper-cased at engine.py:455) after
// FASTALoader's character filter (src/merpcr/io/fasta.py:60).  One thread packs
// one 64-base group: two 2-bit words, one ginv word and one gexc word, and lists
// the heads of exception runs (maximal same-character stretches of non-ACGT
// bases inside its put) for the sparse character index.
#include <algorithm>

#include "mp_internal.h"

namespace mp {

__device__ __forceinline__ uint8_t dev_upcase(uint8_t c) {
    return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c;
}

// code in bits 0-1, exc in bit 2, inv in bit 3
__device__ __forceinline__ uint32_t classify(uint8_t u) {
    switch (u) {
        case 'A': return 0u;
        case 'C': return 1u;
        case 'G': return 2u;
        case 'T': return 3u;
        case 'U': return 3u | 4u;
        default: return 4u | 8u;
    }
}

__global__ __launch_bounds__(256) void pack_kernel(const uint8_t* __restrict__ src, uint64_t nbytes,
                                                   uint64_t gstart, uint64_t* __restrict__ g2,
                                                   uint64_t* __restrict__ gexc,
                                                   uint64_t* __restrict__ ginv,
                                                   uint64_t* __restrict__ xr_start,
                                                   uint8_t* __restrict__ xr_char,
                                                   unsigned long long* __restrict__ xr_count,
                                                   uint64_t xr_cap, uint64_t xr_base,
                                                   unsigned long long* __restrict__ u_count) {
    const uint64_t grp = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i0 = grp * 64;
    const bool active = i0 < nbytes;
    uint64_t w0 = 0, w1 = 0, exc = ~0ull, inv = ~0ull;
    uint32_t heads = 0;
    uint64_t headmask = 0;  // bit 63-i set at run heads
    if (active) {
        const uint32_t cnt = (uint32_t)min<uint64_t>(64, nbytes - i0);
        uint8_t prev = 0;
        bool prev_exc = false;
        if (i0 > 0) {
            prev = dev_upcase(src[i0 - 1]);
            prev_exc = (classify(prev) & 4u) != 0;
        }
        uint8_t buf[64];
        if (cnt == 64) {
            const uint4* s4 = reinterpret_cast<const uint4*>(src + i0);
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const uint4 x = s4[v];
                *reinterpret_cast<uint4*>(buf + 16 * v) = x;
            }
        } else {
            for (uint32_t i = 0; i < 64; ++i) buf[i] = i < cnt ? src[i0 + i] : 0;
        }
        exc = 0;
        inv = 0;
#pragma unroll 8
        for (uint32_t i = 0; i < 64; ++i) {
            const uint8_t u = dev_upcase(buf[i]);
            const uint32_t c = classify(u);
            const bool pad = i >= cnt;
            const uint64_t code = pad ? 0ull : (uint64_t)(c & 3u);
            if (i < 32) w0 |= code << (62 - 2 * i);
            else w1 |= code << (62 - 2 * (i - 32));
            const bool e = pad || (c & 4u);
            const bool v = pad || (c & 8u);
            exc |= (uint64_t)e << (63 - i);
            inv |= (uint64_t)v << (63 - i);
            const bool head = !pad && (c & 4u) && (!prev_exc || prev != u);
            headmask |= (uint64_t)head << (63 - i);
            prev = u;
            prev_exc = !pad && (c & 4u);
        }
        heads = __popcll(headmask);
        const uint32_t nu = (uint32_t)__popcll(exc & ~inv & (cnt == 64 ? ~0ull : ~(~0ull >> cnt)));
        if (nu) atomicAdd(u_count, (unsigned long long)nu);
        const uint64_t gw = (gstart + i0) >> 5;
        g2[gw] = w0;
        g2[gw + 1] = w1;
        gexc[(gstart + i0) >> 6] = exc;
        ginv[(gstart + i0) >> 6] = inv;
    }
    // wave-aggregated reservation of run-index entries
    const uint64_t ball = __ballot(heads > 0);
    uint32_t incl = heads;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    unsigned long long wbase = 0;
    if (ball) {
        if (lane == 0) wbase = atomicAdd(xr_count, (unsigned long long)total);
        wbase = __shfl(wbase, 0, 64);
    }
    if (heads) {
        uint64_t out = xr_base + wbase + (incl - heads);
        uint64_t m = headmask;
        while (m) {
            const int i = __clzll(m);  // position of the top set bit = base index
            m &= ~(1ull << (63 - i));
            if (out < xr_cap) {
                xr_start[out] = gstart + i0 + (uint64_t)i;
                xr_char[out] = dev_upcase(src[i0 + i]);
            }
            ++out;
        }
    }
}

// dir[b] = index of the last exception run starting at or before b << kDirShift.
__global__ void run_dir_kernel(const uint64_t* __restrict__ xr_start, uint64_t n_xr, uint32_t* __restrict__ dir,
                               uint64_t n_dir) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n_dir) return;
    const uint64_t j = b << kDirShift;
    uint64_t lo = 0, hi = n_xr;
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (xr_start[mid] <= j) lo = mid;
        else hi = mid;
    }
    dir[b] = (uint32_t)lo;
}

static void free_genome(Genome* g) {
    if (!g) return;
    hipFree(g->xr_dir); hipFree(g->d_ucount);
    hipFree(g->g2); hipFree(g->gexc); hipFree(g->ginv); hipFree(g->d_base); hipFree(g->d_len);
    hipFree(g->xr_start); hipFree(g->xr_char); hipFree(g->d_counter); hipFree(g->staging);
    delete g;
}

static int grow_runs(Genome* g, uint64_t need) {
    if (need <= g->xr_cap) return MP_OK;
    uint64_t cap = std::max<uint64_t>(need + need / 2, 1 << 16);
    uint64_t* ns = nullptr;
    uint8_t* nc = nullptr;
    MP_HIP_CHECK(hipMalloc(&ns, cap * sizeof(uint64_t)));
    MP_HIP_CHECK(hipMalloc(&nc, cap));
    if (g->n_xr) {
        MP_HIP_CHECK(hipMemcpy(ns, g->xr_start, g->n_xr * sizeof(uint64_t), hipMemcpyDeviceToDevice));
        MP_HIP_CHECK(hipMemcpy(nc, g->xr_char, g->n_xr, hipMemcpyDeviceToDevice));
    }
    hipFree(g->xr_start);
    hipFree(g->xr_char);
    g->dev_bytes += (cap - g->xr_cap) * 9;
    g->xr_start = ns;
    g->xr_char = nc;
    g->xr_cap = cap;
    return MP_OK;
}

static int put_device_bytes(Genome* g, uint32_t seq, uint64_t offset, const uint8_t* dsrc,
                            uint64_t nbytes, hipStream_t st) {
    if (seq >= g->n_seq) return fail(MP_E_ARG, "mp_genome_put: sequence index out of range");
    if (offset % 64) return fail(MP_E_ARG, "mp_genome_put: offset must be a multiple of 64");
    if (offset + nbytes > g->len[seq]) return fail(MP_E_ARG, "mp_genome_put: write past sequence end");
    if (offset + nbytes < g->len[seq] && nbytes % 64)
        return fail(MP_E_ARG, "mp_genome_put: non-final chunk must be a multiple of 64 bytes");
    if (!nbytes) return MP_OK;
    g->sealed = false;
    const uint64_t groups = (nbytes + 63) / 64;
    const uint32_t blocks = (uint32_t)((groups + 255) / 256);
    // first pass: pack + count runs; grow the run index and redo on overflow
    for (int attempt = 0; attempt < 2; ++attempt) {
        MP_HIP_CHECK(hipMemsetAsync(g->d_counter, 0, sizeof(unsigned long long), st));
        hipLaunchKernelGGL(pack_kernel, dim3(blocks), dim3(256), 0, st, dsrc, nbytes,
                           g->base[seq] + offset, g->g2, g->gexc, g->ginv, g->xr_start, g->xr_char,
                           g->d_counter, g->xr_cap, g->n_xr, g->d_ucount);
        MP_HIP_CHECK(hipGetLastError());
        unsigned long long cnt = 0;
        MP_HIP_CHECK(hipMemcpyAsync(&cnt, g->d_counter, sizeof(cnt), hipMemcpyDeviceToHost, st));
        MP_HIP_CHECK(hipStreamSynchronize(st));
        if (g->n_xr + cnt <= g->xr_cap) {
            g->n_xr += cnt;
            return MP_OK;
        }
        int rc = grow_runs(g, g->n_xr + cnt);
        if (rc) return rc;
    }
    return fail(MP_E_STATE, "mp_genome_put: run index did not fit after growth");
}

}  // namespace mp

using namespace mp;

// Host layout of a sequence set: each sequence padded to a multiple of 64 bases.
static int layout(Genome* g, uint32_t n_seq, const uint64_t* seq_len) {
    for (uint32_t s = 0; s < n_seq; ++s)
        if (seq_len[s] >= 0xFFFFFFFFull) return fail(MP_E_ARG, "sequence longer than 2^32-2 bases is not supported");
    g->n_seq = n_seq;
    g->len.assign(seq_len, seq_len + n_seq);
    g->base.resize(n_seq);
    uint64_t off = 0;
    for (uint32_t s = 0; s < n_seq; ++s) {
        g->base[s] = off;
        off += round_up(g->len[s], 64);
    }
    g->total = off;
    return MP_OK;
}

// Device planes for the current layout (reused when they fit), padding and
// unwritten bases marked ambiguous, run index emptied.
static int place(Genome* g) {
    const uint64_t off = g->total;
    const uint64_t w2 = off / 32 + 4, w1 = off / 64 + 4;
    if (off > g->plane_cap || !g->g2) {
        hipFree(g->g2); hipFree(g->gexc); hipFree(g->ginv);
        g->g2 = g->gexc = g->ginv = nullptr;
        g->plane_cap = 0;
        if (hipMalloc(&g->g2, w2 * 8) != hipSuccess || hipMalloc(&g->gexc, w1 * 8) != hipSuccess ||
            hipMalloc(&g->ginv, w1 * 8) != hipSuccess)
            return fail(MP_E_NOMEM, "mp_genome: device allocation failed");
        g->plane_cap = off;
    }
    if (g->n_seq > g->seq_cap || !g->d_base) {
        hipFree(g->d_base); hipFree(g->d_len);
        g->d_base = g->d_len = nullptr;
        g->seq_cap = 0;
        const uint64_t n = std::max<uint64_t>(g->n_seq, 1);
        if (hipMalloc(&g->d_base, n * 8) != hipSuccess || hipMalloc(&g->d_len, n * 8) != hipSuccess)
            return fail(MP_E_NOMEM, "mp_genome: device allocation failed");
        g->seq_cap = (uint32_t)n;
    }
    if (!g->d_counter && (hipMalloc(&g->d_counter, 64) != hipSuccess || hipMalloc(&g->d_ucount, 64) != hipSuccess))
        return fail(MP_E_NOMEM, "mp_genome: device allocation failed");
    g->dev_bytes = (g->plane_cap / 32 + 4) * 8 + 2 * (g->plane_cap / 64 + 4) * 8 + g->xr_cap * 9;
    if (hipMemset(g->d_ucount, 0, 64) != hipSuccess || hipMemset(g->g2, 0, w2 * 8) != hipSuccess ||
        hipMemset(g->gexc, 0xFF, w1 * 8) != hipSuccess || hipMemset(g->ginv, 0xFF, w1 * 8) != hipSuccess)
        return fail(MP_E_HIP, "mp_genome: memset failed");
    if (g->n_seq && (hipMemcpy(g->d_base, g->base.data(), g->n_seq * 8, hipMemcpyHostToDevice) != hipSuccess ||
                     hipMemcpy(g->d_len, g->len.data(), g->n_seq * 8, hipMemcpyHostToDevice) != hipSuccess))
        return fail(MP_E_HIP, "mp_genome: upload failed");
    g->n_xr = 0;
    g->has_u = false;
    g->sealed = false;
    return grow_runs(g, 1 << 16);
}

MP_EXPORT int mp_genome_create(int32_t device, uint32_t n_seq, const uint64_t* seq_len, void** out) {
    if (!out || (n_seq && !seq_len)) return fail(MP_E_ARG, "mp_genome_create: null pointer");
    *out = nullptr;
    Genome* g = new Genome();
    g->device = device;
    int rc = layout(g, n_seq, seq_len);
    if (!rc && hipSetDevice(device) != hipSuccess) rc = fail(MP_E_HIP, "hipSetDevice failed");
    if (!rc) rc = place(g);
    if (rc) {
        free_genome(g);
        return rc;
    }
    *out = g;
    return MP_OK;
}

MP_EXPORT int mp_genome_reset(void* genome, uint32_t n_seq, const uint64_t* seq_len) {
    Genome* g = (Genome*)genome;
    if (!g || (n_seq && !seq_len)) return fail(MP_E_ARG, "mp_genome_reset: null pointer");
    MP_HIP_CHECK(hipSetDevice(g->device));
    int rc = layout(g, n_seq, seq_len);
    if (!rc) rc = place(g);
    return rc;
}

MP_EXPORT int mp_genome_put_device(void* genome, uint32_t seq, uint64_t offset, const uint8_t* dev_bytes,
                                   uint64_t nbytes, void* stream) {
    Genome* g = (Genome*)genome;
    if (!g || (nbytes && !dev_bytes)) return fail(MP_E_ARG, "mp_genome_put_device: null pointer");
    MP_HIP_CHECK(hipSetDevice(g->device));
    return put_device_bytes(g, seq, offset, dev_bytes, nbytes, (hipStream_t)stream);
}

MP_EXPORT int mp_genome_put(void* genome, uint32_t seq, uint64_t offset, const uint8_t* host_bytes,
                            uint64_t nbytes, void* stream) {
    Genome* g = (Genome*)genome;
    if (!g || (nbytes && !host_bytes)) return fail(MP_E_ARG, "mp_genome_put: null pointer");
    MP_HIP_CHECK(hipSetDevice(g->device));
    hipStream_t st = (hipStream_t)stream;
    const uint64_t piece = 256ull << 20;  // staging granularity (multiple of 64)
    if (!g->staging) {
        g->staging_cap = piece;
        MP_HIP_CHECK(hipMalloc(&g->staging, g->staging_cap));
    }
    for (uint64_t done = 0; done < nbytes || (nbytes == 0 && done == 0); done += piece) {
        if (nbytes == 0) break;
        const uint64_t n = std::min(piece, nbytes - done);
        MP_HIP_CHECK(hipMemcpyAsync(g->staging, host_bytes + done, n, hipMemcpyHostToDevice, st));
        int rc = put_device_bytes(g, seq, offset + done, g->staging, n, st);
        if (rc) return rc;
    }
    return MP_OK;
}

MP_EXPORT int mp_genome_seal(void* genome, void* stream) {
    Genome* g = (Genome*)genome;
    if (!g) return fail(MP_E_ARG, "mp_genome_seal: null genome");
    MP_HIP_CHECK(hipSetDevice(g->device));
    hipStream_t st = (hipStream_t)stream;
    int rc = sort_runs(g, st);
    if (rc) return rc;
    if (g->n_xr >> 32) return fail(MP_E_ARG, "more than 2^32 exception runs");
    hipFree(g->xr_dir);
    g->xr_dir = nullptr;
    g->n_dir = (g->total >> kDirShift) + 2;
    MP_HIP_CHECK(hipMalloc(&g->xr_dir, g->n_dir * sizeof(uint32_t)));
    hipLaunchKernelGGL(run_dir_kernel, dim3((uint32_t)((g->n_dir + 255) / 256)), dim3(256), 0, st, g->xr_start,
                       g->n_xr, g->xr_dir, g->n_dir);
    MP_HIP_CHECK(hipGetLastError());
    unsigned long long nu = 0;
    MP_HIP_CHECK(hipMemcpyAsync(&nu, g->d_ucount, sizeof(nu), hipMemcpyDeviceToHost, st));
    MP_HIP_CHECK(hipStreamSynchronize(st));
    g->has_u = nu != 0;
    g->sealed = true;
    return MP_OK;
}

MP_EXPORT int mp_genome_stats(void* genome, uint64_t* total_bases, uint64_t* n_exc_runs, uint64_t* dev_bytes) {
    Genome* g = (Genome*)genome;
    if (!g) return fail(MP_E_ARG, "mp_genome_stats: null genome");
    if (total_bases) {
        uint64_t t = 0;
        for (auto l : g->len) t += l;
        *total_bases = t;
    }
    if (n_exc_runs) *n_exc_runs = g->n_xr;
    if (dev_bytes) *dev_bytes = g->dev_bytes;
    return MP_OK;
}

MP_EXPORT void mp_genome_destroy(void* genome) { free_genome((Genome*)genome); }
