// Genome residency: pack filtered sequence bytes into the HBM planes.
//
// Stands in for the sequence strings that MerPCR.search walks per record
// (src/merpcr/core/engine.py:373-411, upper-cased at engine.py:455) after
// FASTALoader's character filter (src/merpcr/io/fasta.py:60).  pack_kernel turns each
// 64-base group into two 2-bit words, one ginv, one gexc and one gwild word, and lists the
// heads of exception runs (maximal same-character stretches of non-ACGT bases inside
// its put) for the sparse character index.
#include <algorithm>

#include "mp_internal.h"

namespace mp {

// ---------------------------------------------------------------- byte classification
// Four bytes at a time (SWAR).  Per byte b, u = upper-case(b) (a-z only, as str.upper() on
// the ASCII letters; engine.py:455):
//   2-bit code  A=0 C=1 G=2 T=U=3 (bits 2-3 xor bits 1-2 of the byte, case-blind), 0 for
//               every other byte (an exception base reads as 'A' in the 2-bit plane)
//   inv         u is not one of A/C/G/T/U: every W-mer through it is unseeded (engine.py:464-503)
//   exc         u is not exactly A/C/G/T: the primer compare looks the character up
// Bit 7 of each byte of the masks below carries the per-byte result.

// 0x80 in each byte of v that is zero (exact: no carry crosses a byte)
__device__ __forceinline__ uint32_t zbytes(uint32_t v) {
    return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v) & 0x80808080u;
}
// per-byte flags (bit 7 of each byte, byte 0 = first base) -> 4 bits, first base on top
__device__ __forceinline__ uint32_t nib4(uint32_t m) {
    const uint32_t t = m >> 7;
    return ((t & 1u) << 3) | ((t >> 6) & 4u) | ((t >> 15) & 2u) | ((t >> 24) & 1u);
}
struct Cls4 {
    uint32_t code8;  // the 4 bases' 2-bit codes, first base on top
    uint32_t exc, inv;  // per-byte flags (bit 7)
    uint32_t wild;   // per-byte flag: 'N' (either case), which every IUPAC primer base matches
    uint32_t up;     // upper-cased bytes
};
__device__ __forceinline__ Cls4 classify4(uint32_t w) {
    const uint32_t l = w | 0x20202020u;  // case-blind compare against the lower-case letters
    const uint32_t acgt = zbytes(l ^ 0x61616161u) | zbytes(l ^ 0x63636363u) | zbytes(l ^ 0x67676767u) |
                          zbytes(l ^ 0x74747474u);
    const uint32_t acgtu = acgt | zbytes(l ^ 0x75757575u);
    uint32_t c = ((w >> 2) ^ (w >> 1)) & 0x03030303u;
    c &= (acgtu >> 7) * 3u;
    Cls4 r;
    r.code8 = ((c & 3u) << 6) | (((c >> 8) & 3u) << 4) | (((c >> 16) & 3u) << 2) | (c >> 24);
    r.exc = ~acgt & 0x80808080u;
    r.inv = ~acgtu & 0x80808080u;
    r.wild = zbytes(l ^ 0x6E6E6E6Eu);
    const uint32_t t = w & 0x7F7F7F7Fu;  // a-z: t >= 0x61, t <= 0x7A and the byte is ASCII
    const uint32_t lower = (t + 0x1F1F1F1Fu) & (0xFAFAFAFAu - t) & ~w & 0x80808080u;
    r.up = w - (lower >> 2);
    return r;
}
__device__ __forceinline__ uint32_t byte_of(uint4 v, uint32_t i) {  // byte i of 16, no register indexing
    const uint32_t w = i < 8 ? (i < 4 ? v.x : v.y) : (i < 12 ? v.z : v.w);
    return (w >> (8u * (i & 3u))) & 0xFFu;
}

// Filtered sequence bytes -> the planes.  A wave packs a 4 KiB tile per iteration: four
// 1 KiB pieces, each one coalesced 16-B load per lane, all four issued before any is used.
// A lane classifies its 16 bytes (classify4); four neighbouring lanes make one 64-base group:
// its two g2 words and its gexc / ginv words come together by shuffles and are stored by the
// group's first lanes (contiguous in memory across the wave).  Heads of exception runs
// (maximal stretches of one non-ACGT character inside this put) are listed for the sparse
// character index with one wave-aggregated reservation per piece.  Bytes past nbytes are
// padding (ambiguous, never a run head).  (The previous form, one thread per 64 bytes
// through a 64-byte private array, ran at ~160 GB/s.)
constexpr uint32_t kPackTile = 4096;
constexpr uint32_t kPackPiece = 1024;
__global__ __launch_bounds__(256) void pack_kernel(const uint8_t* __restrict__ src, uint64_t nbytes,
                                                   uint64_t gstart, uint64_t* __restrict__ g2,
                                                   uint64_t* __restrict__ gexc,
                                                   uint64_t* __restrict__ ginv,
                                                   uint64_t* __restrict__ gwild,
                                                   uint64_t* __restrict__ xr_start,
                                                   uint8_t* __restrict__ xr_char,
                                                   unsigned long long* __restrict__ xr_count,
                                                   uint64_t xr_cap, uint64_t xr_base,
                                                   unsigned long long* __restrict__ u_count) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t q = lane & 3u;
    const uint64_t n_tiles = (nbytes + kPackTile - 1) / kPackTile;
    const uint64_t wave0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t n_waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const bool vec_ok = (reinterpret_cast<uintptr_t>(src) & 15u) == 0;
    uint32_t n_u = 0;
    for (uint64_t tile = wave0; tile < n_tiles; tile += n_waves) {  // wave-uniform
        const uint64_t t0 = tile * kPackTile;
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t o = t0 + (uint64_t)k * kPackPiece + (uint64_t)lane * 16u;
            if (vec_ok && o + 16 <= nbytes) {
                v[k] = *reinterpret_cast<const uint4*>(src + o);
            } else {  // the put's ragged end (or an unaligned source): bytes, 0 past the end
                uint32_t b[16];
#pragma unroll
                for (int j = 0; j < 16; ++j) b[j] = o + (uint64_t)j < nbytes ? src[o + j] : 0u;
                v[k] = make_uint4(b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24, b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24,
                                  b[8] | b[9] << 8 | b[10] << 16 | b[11] << 24,
                                  b[12] | b[13] << 8 | b[14] << 16 | b[15] << 24);
            }
        }
        // the byte before the tile (run heads continue across tiles, not across puts)
        uint32_t prev_up = 0, prev_exc = 0;
        if (t0 > 0) {
            const Cls4 c = classify4((uint32_t)src[t0 - 1]);
            prev_up = c.up & 0xFFu;
            prev_exc = c.exc & 0x80u;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t o = t0 + (uint64_t)k * kPackPiece + (uint64_t)lane * 16u;  // this lane's first byte
            const Cls4 c0 = classify4(v[k].x), c1 = classify4(v[k].y), c2 = classify4(v[k].z), c3 = classify4(v[k].w);
            const uint64_t left = o < nbytes ? nbytes - o : 0;
            const uint32_t valid16 = left >= 16 ? 0xFFFFu : (0xFFFFu << (16u - (uint32_t)left)) & 0xFFFFu;
            const uint32_t code32 = (c0.code8 << 24) | (c1.code8 << 16) | (c2.code8 << 8) | c3.code8;
            uint32_t exc16 = (nib4(c0.exc) << 12) | (nib4(c1.exc) << 8) | (nib4(c2.exc) << 4) | nib4(c3.exc);
            uint32_t inv16 = (nib4(c0.inv) << 12) | (nib4(c1.inv) << 8) | (nib4(c2.inv) << 4) | nib4(c3.inv);
            exc16 |= ~valid16 & 0xFFFFu;  // padding: ambiguous
            inv16 |= ~valid16 & 0xFFFFu;
            const uint32_t wild16 =
                ((nib4(c0.wild) << 12) | (nib4(c1.wild) << 8) | (nib4(c2.wild) << 4) | nib4(c3.wild)) & valid16;
            n_u += (uint32_t)__popc(exc16 & ~inv16 & valid16);
            // run heads: an exception byte whose predecessor (in this put) is not the same
            // exception character
            const uint32_t pu_l = (uint32_t)__shfl_up((int)(c3.up >> 24), 1, 64);
            const uint32_t pe_l = (uint32_t)__shfl_up((int)(c3.exc >> 24), 1, 64);
            const uint32_t pu0 = lane ? pu_l : prev_up, pe0 = lane ? pe_l : prev_exc;
            const uint32_t h0 = c0.exc & ~(((c0.exc << 8) | pe0) & zbytes(c0.up ^ ((c0.up << 8) | pu0)));
            const uint32_t h1 = c1.exc & ~(((c1.exc << 8) | (c0.exc >> 24)) & zbytes(c1.up ^ ((c1.up << 8) | (c0.up >> 24))));
            const uint32_t h2 = c2.exc & ~(((c2.exc << 8) | (c1.exc >> 24)) & zbytes(c2.up ^ ((c2.up << 8) | (c1.up >> 24))));
            const uint32_t h3 = c3.exc & ~(((c3.exc << 8) | (c2.exc >> 24)) & zbytes(c3.up ^ ((c3.up << 8) | (c2.up >> 24))));
            const uint32_t head16 = ((nib4(h0) << 12) | (nib4(h1) << 8) | (nib4(h2) << 4) | nib4(h3)) & valid16;
            // the next piece's lane 0 continues from this piece's last byte (lane 63)
            prev_up = (uint32_t)__shfl((int)(c3.up >> 24), 63, 64);
            prev_exc = (uint32_t)__shfl((int)(c3.exc >> 24), 63, 64);
            // one 64-base group per 4 lanes: g2 words from lanes q = 0, 2; flag words from q = 0
            const uint32_t code_n = (uint32_t)__shfl_down((int)code32, 1, 64);
            const uint32_t e1 = (uint32_t)__shfl_down((int)exc16, 1, 64), e2 = (uint32_t)__shfl_down((int)exc16, 2, 64),
                           e3 = (uint32_t)__shfl_down((int)exc16, 3, 64);
            const uint32_t i1 = (uint32_t)__shfl_down((int)inv16, 1, 64), i2 = (uint32_t)__shfl_down((int)inv16, 2, 64),
                           i3 = (uint32_t)__shfl_down((int)inv16, 3, 64);
            const uint32_t n1 = (uint32_t)__shfl_down((int)wild16, 1, 64), n2 = (uint32_t)__shfl_down((int)wild16, 2, 64),
                           n3 = (uint32_t)__shfl_down((int)wild16, 3, 64);
            const uint64_t grp0 = o - (uint64_t)q * 16u;  // the group's first byte in the put
            if (grp0 < nbytes) {
                const uint64_t gb = gstart + grp0;
                if ((q & 1u) == 0) g2[(gb >> 5) + (q >> 1)] = ((uint64_t)code32 << 32) | code_n;
                if (q == 0) {
                    gexc[gb >> 6] = ((uint64_t)exc16 << 48) | ((uint64_t)e1 << 32) | ((uint64_t)e2 << 16) | e3;
                    ginv[gb >> 6] = ((uint64_t)inv16 << 48) | ((uint64_t)i1 << 32) | ((uint64_t)i2 << 16) | i3;
                    gwild[gb >> 6] = ((uint64_t)wild16 << 48) | ((uint64_t)n1 << 32) | ((uint64_t)n2 << 16) | n3;
                }
            }
            // wave-aggregated reservation of run-index entries (rare: N runs, IUPAC bases)
            if (__any(head16 != 0u)) {
                const uint32_t nh = (uint32_t)__popc(head16);
                uint32_t incl = nh;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t y = (uint32_t)__shfl_up((int)incl, d, 64);
                    if ((int)lane >= d) incl += y;
                }
                const uint32_t total = (uint32_t)__shfl((int)incl, 63, 64);
                unsigned long long wbase = 0;
                if (lane == 0) wbase = atomicAdd(xr_count, (unsigned long long)total);
                wbase = (unsigned long long)__shfl((long long)wbase, 0, 64);
                uint64_t out = xr_base + wbase + (incl - nh);
                uint32_t m = head16;
                const uint4 up = make_uint4(c0.up, c1.up, c2.up, c3.up);
                while (m) {
                    const uint32_t i = (uint32_t)__clz(m) - 16u;  // byte index, first base = bit 15
                    m &= ~(0x8000u >> i);
                    if (out < xr_cap) {
                        xr_start[out] = gstart + o + i;
                        xr_char[out] = (uint8_t)byte_of(up, i);
                    }
                    ++out;
                }
            }
        }
    }
    // U bases seen (RNA input): one atomic per wave
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) n_u += (uint32_t)__shfl_xor((int)n_u, d, 64);
    if (lane == 0 && n_u) atomicAdd(u_count, (unsigned long long)n_u);
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
    hipFree(g->g2); hipFree(g->gexc); hipFree(g->ginv); hipFree(g->gwild); hipFree(g->gpair); hipFree(g->d_base); hipFree(g->d_len);
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
    const uint64_t tiles = (nbytes + kPackTile - 1) / kPackTile;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((tiles + 3) / 4, 8192);  // 4 waves per block
    // first pass: pack + count runs; grow the run index and redo on overflow
    for (int attempt = 0; attempt < 2; ++attempt) {
        MP_HIP_CHECK(hipMemsetAsync(g->d_counter, 0, sizeof(unsigned long long), st));
        hipLaunchKernelGGL(pack_kernel, dim3(blocks), dim3(256), 0, st, dsrc, nbytes,
                           g->base[seq] + offset, g->g2, g->gexc, g->ginv, g->gwild, g->xr_start, g->xr_char,
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
        hipFree(g->g2); hipFree(g->gexc); hipFree(g->ginv); hipFree(g->gwild); hipFree(g->gpair);
        g->g2 = g->gexc = g->ginv = g->gwild = g->gpair = nullptr;
        g->plane_cap = 0;
        if (hipMalloc(&g->g2, w2 * 8) != hipSuccess || hipMalloc(&g->gexc, w1 * 8) != hipSuccess ||
            hipMalloc(&g->ginv, w1 * 8) != hipSuccess || hipMalloc(&g->gwild, w1 * 8) != hipSuccess ||
            hipMalloc(&g->gpair, w1 * 32) != hipSuccess)
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
    g->dev_bytes = (g->plane_cap / 32 + 4) * 8 + 3 * (g->plane_cap / 64 + 4) * 8 + (g->plane_cap / 64 + 4) * 32 +
                   g->xr_cap * 9;
    if (hipMemset(g->d_ucount, 0, 64) != hipSuccess || hipMemset(g->g2, 0, w2 * 8) != hipSuccess ||
        hipMemset(g->gexc, 0xFF, w1 * 8) != hipSuccess || hipMemset(g->ginv, 0xFF, w1 * 8) != hipSuccess ||
        hipMemset(g->gwild, 0, w1 * 8) != hipSuccess)
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
    if (g->n_pending) return fail(MP_E_STATE, "mp_genome_reset: a search run over this genome is enqueued");
    MP_HIP_CHECK(hipSetDevice(g->device));
    int rc = layout(g, n_seq, seq_len);
    if (!rc) rc = place(g);
    return rc;
}

MP_EXPORT int mp_genome_put_device(void* genome, uint32_t seq, uint64_t offset, const uint8_t* dev_bytes,
                                   uint64_t nbytes, void* stream) {
    Genome* g = (Genome*)genome;
    if (!g || (nbytes && !dev_bytes)) return fail(MP_E_ARG, "mp_genome_put_device: null pointer");
    if (g->n_pending) return fail(MP_E_STATE, "mp_genome_put_device: a search run over this genome is enqueued");
    MP_HIP_CHECK(hipSetDevice(g->device));
    return put_device_bytes(g, seq, offset, dev_bytes, nbytes, (hipStream_t)stream);
}

MP_EXPORT int mp_genome_put(void* genome, uint32_t seq, uint64_t offset, const uint8_t* host_bytes,
                            uint64_t nbytes, void* stream) {
    Genome* g = (Genome*)genome;
    if (!g || (nbytes && !host_bytes)) return fail(MP_E_ARG, "mp_genome_put: null pointer");
    if (g->n_pending) return fail(MP_E_STATE, "mp_genome_put: a search run over this genome is enqueued");
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

// Genome::gpair from the planes: block b = {g2[2b], g2[2b + 1], gexc[b], gwild[b]}
__global__ void interleave_pair_kernel(const uint64_t* __restrict__ g2, const uint64_t* __restrict__ gexc,
                                       const uint64_t* __restrict__ gwild, uint64_t* __restrict__ out, uint64_t nb) {
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * blockDim.x) {
        reinterpret_cast<ulonglong2*>(out)[2 * b] = make_ulonglong2(g2[2 * b], g2[2 * b + 1]);
        reinterpret_cast<ulonglong2*>(out)[2 * b + 1] = make_ulonglong2(gexc[b], gwild[b]);
    }
}

MP_EXPORT int mp_genome_seal(void* genome, void* stream) {
    Genome* g = (Genome*)genome;
    if (!g) return fail(MP_E_ARG, "mp_genome_seal: null genome");
    if (g->n_pending) return fail(MP_E_STATE, "mp_genome_seal: a search run over this genome is enqueued");
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
    {
        const uint64_t nb = g->total / 64 + 2;  // every block a stretch read can reach (g2 holds total / 32 + 4 words)
        hipLaunchKernelGGL(interleave_pair_kernel, dim3((uint32_t)std::min<uint64_t>((nb + 255) / 256, 8192)), dim3(256), 0, st,
                           g->g2, g->gexc, g->gwild, g->gpair, nb);
        MP_HIP_CHECK(hipGetLastError());
    }
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

MP_EXPORT int mp_genome_download(void* genome, uint64_t* g2, uint64_t* gexc, uint64_t* ginv, uint64_t* gwild,
                                 uint64_t* xr_start, uint8_t* xr_char) {
    Genome* g = (Genome*)genome;
    if (!g) return fail(MP_E_ARG, "mp_genome_download: null genome");
    if (!g->sealed) return fail(MP_E_STATE, "mp_genome_download: genome not sealed");
    MP_HIP_CHECK(hipSetDevice(g->device));
    if (g2) MP_HIP_CHECK(hipMemcpy(g2, g->g2, g->total / 32 * 8, hipMemcpyDeviceToHost));
    if (gexc) MP_HIP_CHECK(hipMemcpy(gexc, g->gexc, g->total / 64 * 8, hipMemcpyDeviceToHost));
    if (ginv) MP_HIP_CHECK(hipMemcpy(ginv, g->ginv, g->total / 64 * 8, hipMemcpyDeviceToHost));
    if (gwild) MP_HIP_CHECK(hipMemcpy(gwild, g->gwild, g->total / 64 * 8, hipMemcpyDeviceToHost));
    if (xr_start && g->n_xr) MP_HIP_CHECK(hipMemcpy(xr_start, g->xr_start, g->n_xr * 8, hipMemcpyDeviceToHost));
    if (xr_char && g->n_xr) MP_HIP_CHECK(hipMemcpy(xr_char, g->xr_char, g->n_xr, hipMemcpyDeviceToHost));
    return MP_OK;
}

MP_EXPORT void mp_genome_destroy(void* genome) { free_genome((Genome*)genome); }
