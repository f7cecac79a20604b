// Device FASTA ingestion of ASCII files (the device form of FASTALoader.load_file,
// src/merpcr/io/fasta.py:18-71).
//
// The host reader (mp_fasta.hip) spends ~0.35 s of 16 threads on a 3 GB file; here the raw
// bytes go to HBM as they are (pread into pinned staging by several host threads, async
// copies), and the reference's rules run on the device:
//   * a line is a header when its first non-whitespace character is '>' (line.strip() then
//     startswith('>'), fasta.py:47-51; universal newlines end a line at "\n", "\r" and
//     "\r\n"; str.strip()'s ASCII whitespace is \t \n \v \f \r \x1c-\x1f and space);
//   * every other byte is kept iff it is one of the 32 letters c with c.upper() in
//     "ACGTBDHKMNRSVWXY" (fasta.py:60) -- whitespace, line ends, digits and the rest are
//     never kept, so filtering whole lines equals strip-then-filter;
//   * a record's sequence is the kept bytes between its header line's end and the next
//     header ('>'); bytes before the first header line's end belong to no record.
// The kept bytes of all records are compacted (per-64-KiB-tile counts, one scan, one
// ordered write) into one contiguous device buffer, record after record, which is exactly
// what mp_genome_put_device packs.  Any byte >= 0x80 (Unicode whitespace and U+017F need
// Python's rules) or more than kMaxHeaders header lines leave the file to the host reader
// (*ascii = 0).
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mp_internal.h"

namespace mp {

constexpr uint32_t kFaTile = 65536;          // bytes per compaction tile (one 1024-thread block)
constexpr uint32_t kFaPerThread = 64;        // bytes per thread of a tile
// Header lines the device path takes.  Its per-record cost is a pread of each header line on
// the host and two 1024-thread blocks of fa_points_kernel per record (each rescans a tile), so
// a file of many short records (reads, ESTs) is the host reader's: it has no per-record pass.
constexpr uint32_t kMaxHeaders = 1u << 16;
static_assert(kFaTile == 1024 * kFaPerThread, "one tile per 1024-thread block");

// Keep set of fasta.py:60 over ASCII: the letters A B C D G H K M N R S T V W X Y, either case.
constexpr uint32_t kKeepLetters = (1u << 0) | (1u << 1) | (1u << 2) | (1u << 3) | (1u << 6) | (1u << 7) | (1u << 10) |
                                  (1u << 12) | (1u << 13) | (1u << 17) | (1u << 18) | (1u << 19) | (1u << 21) |
                                  (1u << 22) | (1u << 23) | (1u << 24);
__host__ __device__ __forceinline__ bool fa_keep(uint32_t x) {
    const uint32_t i = (x | 0x20u) - 0x61u;  // 'A'-'Z' and 'a'-'z' to 0..25; nothing else lands there
    return i < 26u && ((kKeepLetters >> i) & 1u);
}
// str.strip() whitespace that does not end a line (\t \v \f \x1c-\x1f space)
__host__ __device__ __forceinline__ bool fa_blank(uint32_t x) {
    return x == 0x20u || x == 0x09u || x == 0x0Bu || x == 0x0Cu || (x >= 0x1Cu && x <= 0x1Fu);
}
__host__ __device__ __forceinline__ bool fa_eol(uint32_t x) { return x == 0x0Au || x == 0x0Du; }

struct FastaDev {
    int device = 0;
    uint8_t* raw = nullptr;       // the file (freed after the compaction)
    uint8_t* bases = nullptr;     // kept bytes of every record, record after record
    uint64_t total = 0;
    std::vector<std::string> deflines;
    std::vector<uint64_t> off, len;  // per record, into bases
};

static void free_fasta_dev(FastaDev* f) {
    if (!f) return;
    (void)hipSetDevice(f->device);
    (void)hipFree(f->raw);
    (void)hipFree(f->bases);
    delete f;
}

// Pass 1: any non-ASCII byte, and the header lines ('>' after only blanks since the line's
// start).  A '>' inside a sequence line is just a dropped byte.
__global__ void fa_scan_kernel(const uint8_t* __restrict__ raw, uint64_t n, uint32_t* __restrict__ flags,
                               uint64_t* __restrict__ hdr) {
    uint32_t hi = 0;
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; i < n;
         i += (uint64_t)gridDim.x * blockDim.x * 16) {
        uint8_t b[16];
        if (i + 16 <= n) {
            const uint4 v = *reinterpret_cast<const uint4*>(raw + i);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 16; ++k) b[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
        } else {
            for (int k = 0; k < 16; ++k) b[k] = i + k < n ? raw[i + k] : 0;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            hi |= b[k] & 0x80u;
            if (b[k] == '>') {
                uint64_t j = i + k;
                while (j > 0 && fa_blank(raw[j - 1])) --j;
                if (j == 0 || fa_eol(raw[j - 1])) {
                    const uint32_t at = atomicAdd(&flags[1], 1u);
                    if (at < kMaxHeaders) hdr[at] = i + k;
                }
            }
        }
    }
    if (__any(hi != 0) && (threadIdx.x & 63) == 0) atomicOr(&flags[0], 1u);
}

// Kept-byte mask of bytes [b0, b0 + 64) (bit j = byte b0 + j), outside the excluded spans
// [slo[s], shi[s]) (sorted, disjoint: everything up to the first header line's end, then
// every header line from its '>' to its end).
__device__ __forceinline__ uint64_t fa_mask(const uint8_t* __restrict__ raw, uint64_t n, uint64_t b0,
                                            const uint64_t* __restrict__ slo, const uint64_t* __restrict__ shi,
                                            uint32_t nspan) {
    uint64_t m = 0;
    if (b0 >= n) return 0;
    if (b0 + 64 <= n) {
        const uint4* p = reinterpret_cast<const uint4*>(raw + b0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 v = p[q];
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    m |= (uint64_t)fa_keep((w[c] >> (8 * k)) & 0xFFu) << (16 * q + 4 * c + k);
        }
    } else {
        for (uint32_t k = 0; b0 + k < n; ++k) m |= (uint64_t)fa_keep(raw[b0 + k]) << k;
    }
    // the first span ending after b0 (binary search), then every span starting before b0 + 64
    uint32_t lo = 0, hi = nspan;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (shi[mid] <= b0) lo = mid + 1;
        else hi = mid;
    }
    for (uint32_t s = lo; s < nspan && slo[s] < b0 + 64; ++s) {
        const uint64_t a = slo[s] > b0 ? slo[s] - b0 : 0, e = shi[s] - b0 < 64 ? shi[s] - b0 : 64;
        if (e > a) m &= ~(((e - a) >= 64 ? ~0ull : ((1ull << (e - a)) - 1ull)) << a);
    }
    return m;
}

// Block-wide exclusive prefix of one count per thread (1024 threads); the total in *tot.
__device__ __forceinline__ uint32_t fa_block_prefix(uint32_t c, uint32_t* s_w, uint32_t* tot) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
        if ((int)lane >= o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint32_t pre = 0, t = 0;
    for (uint32_t k = 0; k < 16; ++k) {
        pre += k < w ? s_w[k] : 0u;
        t += s_w[k];
    }
    __syncthreads();
    *tot = t;
    return pre + x - c;
}

// Pass 2: kept bytes per tile.
__global__ __launch_bounds__(1024) void fa_count_kernel(const uint8_t* __restrict__ raw, uint64_t n,
                                                        const uint64_t* __restrict__ slo, const uint64_t* __restrict__ shi,
                                                        uint32_t nspan, uint32_t* __restrict__ cnt) {
    __shared__ uint32_t s_w[16];
    const uint64_t b0 = (uint64_t)blockIdx.x * kFaTile + (uint64_t)threadIdx.x * kFaPerThread;
    const uint32_t c = (uint32_t)__popcll(fa_mask(raw, n, b0, slo, shi, nspan));
    uint32_t tot;
    (void)fa_block_prefix(c, s_w, &tot);
    if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
}

// Pass 3 (one workgroup): tile offsets off[t] = kept bytes of the tiles before t (64-bit),
// off[nt] = the total.
__global__ __launch_bounds__(1024) void fa_offsets_kernel(const uint32_t* __restrict__ cnt, uint32_t nt,
                                                          uint64_t* __restrict__ off) {
    __shared__ uint64_t s_w[16];
    __shared__ uint64_t s_carry;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < nt; base += 1024) {
        const uint32_t i = base + threadIdx.x;
        const uint64_t c = i < nt ? cnt[i] : 0u;
        uint64_t x = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = (uint64_t)__shfl_up((long long)x, o, 64);
            if ((int)lane >= o) x += y;
        }
        if (lane == 63) s_w[w] = x;
        __syncthreads();
        uint64_t pre = s_carry, t = 0;
        for (uint32_t k = 0; k < 16; ++k) {
            pre += k < w ? s_w[k] : 0u;
            t += s_w[k];
        }
        if (i < nt) off[i] = pre + x - c;
        __syncthreads();
        if (threadIdx.x == 0) s_carry += t;
        __syncthreads();
    }
    if (threadIdx.x == 0) off[nt] = s_carry;
}

// Pass 4: every tile's kept bytes, in order, at its offset.
__global__ __launch_bounds__(1024) void fa_compact_kernel(const uint8_t* __restrict__ raw, uint64_t n,
                                                          const uint64_t* __restrict__ slo, const uint64_t* __restrict__ shi,
                                                          uint32_t nspan, const uint64_t* __restrict__ off,
                                                          uint8_t* __restrict__ out) {
    __shared__ uint32_t s_w[16];
    const uint64_t b0 = (uint64_t)blockIdx.x * kFaTile + (uint64_t)threadIdx.x * kFaPerThread;
    uint64_t m = fa_mask(raw, n, b0, slo, shi, nspan);
    uint32_t tot;
    const uint32_t pre = fa_block_prefix((uint32_t)__popcll(m), s_w, &tot);
    uint8_t* dst = out + off[blockIdx.x] + pre;
    while (m) {
        const uint32_t j = (uint32_t)__builtin_ctzll(m);
        m &= m - 1;
        *dst++ = raw[b0 + j];
    }
}

// Pass 5: kept bytes before each point p (one workgroup per point: its tile's offset plus
// the kept bytes of [tile start, p)).
__global__ __launch_bounds__(1024) void fa_points_kernel(const uint8_t* __restrict__ raw, uint64_t n,
                                                         const uint64_t* __restrict__ slo, const uint64_t* __restrict__ shi,
                                                         uint32_t nspan, const uint64_t* __restrict__ off,
                                                         const uint64_t* __restrict__ pts, uint64_t* __restrict__ pre_out) {
    __shared__ uint32_t s_w[16];
    const uint64_t p = pts[blockIdx.x];
    const uint64_t t = p / kFaTile;
    const uint64_t b0 = t * kFaTile + (uint64_t)threadIdx.x * kFaPerThread;
    uint64_t m = fa_mask(raw, n, b0, slo, shi, nspan);
    if (b0 >= p) m = 0;
    else if (p - b0 < 64) m &= (1ull << (p - b0)) - 1ull;
    uint32_t tot;
    (void)fa_block_prefix((uint32_t)__popcll(m), s_w, &tot);
    const uint64_t nt = (n + kFaTile - 1) / kFaTile;  // p == n on a tile boundary: off[nt] is the total
    if (threadIdx.x == 0) pre_out[blockIdx.x] = off[t < nt ? t : nt] + tot;
}

// The file into device memory: pread by several host threads into pinned staging pieces,
// each copied asynchronously on the thread's own stream (double-buffered).
static int upload_file(int fd, uint64_t size, uint8_t* dev, int device) {
    const uint64_t piece = 16ull << 20;
    const uint64_t np = (size + piece - 1) / piece;
    const uint32_t T = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(np, std::min(8u, std::max(1u, std::thread::hardware_concurrency()))));
    std::vector<int> rc(T, MP_OK);
    std::vector<std::string> msg(T);
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            auto bad = [&](const std::string& m) {
                rc[t] = MP_E_IO;
                msg[t] = m;
            };
            if (hipSetDevice(device) != hipSuccess) return bad("hipSetDevice failed");
            hipStream_t st = nullptr;
            uint8_t* pin[2] = {nullptr, nullptr};
            hipEvent_t ev[2] = {nullptr, nullptr};
            if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess ||
                hipHostMalloc((void**)&pin[0], piece, hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc((void**)&pin[1], piece, hipHostMallocDefault) != hipSuccess ||
                hipEventCreateWithFlags(&ev[0], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&ev[1], hipEventDisableTiming) != hipSuccess) {
                bad("pinned staging allocation failed");
            } else {
                uint32_t it = 0;
                for (uint64_t c = t; c < np && !rc[t]; c += T, ++it) {
                    const int s = (int)(it & 1u);
                    if (it >= 2 && hipEventSynchronize(ev[s]) != hipSuccess) { bad("staging copy failed"); break; }
                    const uint64_t o = c * piece, want = std::min(piece, size - o);
                    uint64_t got = 0;
                    while (got < want) {
                        const ssize_t r = pread(fd, pin[s] + got, want - got, (off_t)(o + got));
                        if (r <= 0) break;
                        got += (uint64_t)r;
                    }
                    if (got != want) { bad("read failed"); break; }
                    if (hipMemcpyAsync(dev + o, pin[s], want, hipMemcpyHostToDevice, st) != hipSuccess ||
                        hipEventRecord(ev[s], st) != hipSuccess) {
                        bad("host-to-device copy failed");
                        break;
                    }
                }
                if (hipStreamSynchronize(st) != hipSuccess && !rc[t]) bad("host-to-device copy failed");
            }
            for (int s = 0; s < 2; ++s) {
                if (ev[s]) (void)hipEventDestroy(ev[s]);
                if (pin[s]) (void)hipHostFree(pin[s]);
            }
            if (st) (void)hipStreamDestroy(st);
        });
    for (auto& x : th) x.join();
    for (uint32_t t = 0; t < T; ++t)
        if (rc[t]) return fail(rc[t], "mp_fasta_load_device: " + msg[t]);
    return MP_OK;
}

// The header line starting at '>' (file position p): its end (the line break or EOF) and the
// stripped text (str.strip(): the '>' is its first character, trailing whitespace removed).
static int header_line(int fd, uint64_t size, uint64_t p, uint64_t* end, std::string* text) {
    std::string s;
    char buf[4096];
    uint64_t q = p;
    for (;;) {
        if (q >= size) break;
        const ssize_t r = pread(fd, buf, (size_t)std::min<uint64_t>(sizeof(buf), size - q), (off_t)q);
        if (r <= 0) return fail(MP_E_IO, "mp_fasta_load_device: read failed");
        const char* e = (const char*)std::memchr(buf, '\n', (size_t)r);
        const char* e2 = (const char*)std::memchr(buf, '\r', (size_t)r);
        if (!e || (e2 && e2 < e)) e = e2;
        const size_t take = e ? (size_t)(e - buf) : (size_t)r;
        s.append(buf, take);
        q += take;
        if (e) break;
    }
    *end = q;
    size_t k = s.size();
    while (k > 0 && (fa_blank((uint8_t)s[k - 1]) || fa_eol((uint8_t)s[k - 1]))) --k;
    s.resize(k);
    *text = std::move(s);
    return MP_OK;
}

static int load_device(const char* path, int device, hipStream_t st, FastaDev* f, int32_t* ascii) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return fail(MP_E_IO, std::string("mp_fasta_load_device: cannot open ") + path);
    struct Closer {
        int fd;
        ~Closer() { close(fd); }
    } closer{fd};
    struct stat sb;
    if (fstat(fd, &sb) != 0) return fail(MP_E_IO, "mp_fasta_load_device: stat failed");
    const uint64_t n = (uint64_t)sb.st_size;
    MP_HIP_CHECK(hipSetDevice(device));
    if (!n) {
        *ascii = 1;
        return MP_OK;
    }
    MP_HIP_CHECK(hipMalloc(&f->raw, n + 64));
    int rc = upload_file(fd, n, f->raw, device);
    if (rc) return rc;
    // pass 1
    uint32_t* flags = nullptr;
    uint64_t* hdr = nullptr;
    MP_HIP_CHECK(hipMalloc(&flags, 2 * sizeof(uint32_t)));
    struct Freer {
        void* p[6] = {};
        ~Freer() {
            for (void* q : p) (void)hipFree(q);
        }
    } fr;
    fr.p[0] = flags;
    MP_HIP_CHECK(hipMalloc(&hdr, (size_t)kMaxHeaders * sizeof(uint64_t)));
    fr.p[1] = hdr;
    MP_HIP_CHECK(hipMemsetAsync(flags, 0, 2 * sizeof(uint32_t), st));
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 16 * 256 - 1) / (16 * 256), 8192);
    hipLaunchKernelGGL(fa_scan_kernel, dim3(grid), dim3(256), 0, st, f->raw, n, flags, hdr);
    MP_HIP_CHECK(hipGetLastError());
    uint32_t hf[2];
    MP_HIP_CHECK(hipMemcpyAsync(hf, flags, sizeof(hf), hipMemcpyDeviceToHost, st));
    MP_HIP_CHECK(hipStreamSynchronize(st));
    if (hf[0] || hf[1] > kMaxHeaders) {  // the host reader's file
        *ascii = 0;
        return MP_OK;
    }
    *ascii = 1;
    const uint32_t nh = hf[1];
    if (!nh) return MP_OK;  // no header line: no record (fasta.py:64-66)
    std::vector<uint64_t> pos(nh);
    MP_HIP_CHECK(hipMemcpyAsync(pos.data(), hdr, nh * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    MP_HIP_CHECK(hipStreamSynchronize(st));
    std::sort(pos.begin(), pos.end());
    std::vector<uint64_t> lend(nh), slo(nh), shi(nh), pts(2 * (size_t)nh);
    f->deflines.resize(nh);
    for (uint32_t k = 0; k < nh; ++k) {
        rc = header_line(fd, n, pos[k], &lend[k], &f->deflines[k]);
        if (rc) return rc;
        slo[k] = k ? pos[k] : 0;  // everything before the first header line's end belongs to no record
        shi[k] = lend[k];
        pts[2 * (size_t)k] = lend[k];
        pts[2 * (size_t)k + 1] = k + 1 < nh ? pos[k + 1] : n;
    }
    uint64_t *d_slo = nullptr, *d_shi = nullptr, *d_pts = nullptr, *d_pre = nullptr, *d_off = nullptr;
    uint32_t* d_cnt = nullptr;
    const uint32_t nt = (uint32_t)((n + kFaTile - 1) / kFaTile);
    MP_HIP_CHECK(hipMalloc(&d_slo, nh * 2 * sizeof(uint64_t)));
    fr.p[2] = d_slo;
    d_shi = d_slo + nh;
    MP_HIP_CHECK(hipMalloc(&d_pts, nh * 4 * sizeof(uint64_t)));
    fr.p[3] = d_pts;
    d_pre = d_pts + 2 * (size_t)nh;
    MP_HIP_CHECK(hipMalloc(&d_cnt, nt * sizeof(uint32_t)));
    fr.p[4] = d_cnt;
    MP_HIP_CHECK(hipMalloc(&d_off, (nt + 1) * sizeof(uint64_t)));
    fr.p[5] = d_off;
    MP_HIP_CHECK(hipMemcpyAsync(d_slo, slo.data(), nh * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    MP_HIP_CHECK(hipMemcpyAsync(d_shi, shi.data(), nh * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    MP_HIP_CHECK(hipMemcpyAsync(d_pts, pts.data(), 2 * (size_t)nh * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(fa_count_kernel, dim3(nt), dim3(1024), 0, st, f->raw, n, d_slo, d_shi, nh, d_cnt);
    MP_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(fa_offsets_kernel, dim3(1), dim3(1024), 0, st, d_cnt, nt, d_off);
    MP_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(fa_points_kernel, dim3(2 * nh), dim3(1024), 0, st, f->raw, n, d_slo, d_shi, nh, d_off, d_pts, d_pre);
    MP_HIP_CHECK(hipGetLastError());
    std::vector<uint64_t> pre(2 * (size_t)nh);
    uint64_t total = 0;
    MP_HIP_CHECK(hipMemcpyAsync(&total, d_off + nt, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    MP_HIP_CHECK(hipMemcpyAsync(pre.data(), d_pre, 2 * (size_t)nh * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    MP_HIP_CHECK(hipStreamSynchronize(st));
    f->total = total;
    MP_HIP_CHECK(hipMalloc(&f->bases, total + 64));
    hipLaunchKernelGGL(fa_compact_kernel, dim3(nt), dim3(1024), 0, st, f->raw, n, d_slo, d_shi, nh, d_off, f->bases);
    MP_HIP_CHECK(hipGetLastError());
    MP_HIP_CHECK(hipStreamSynchronize(st));
    f->off.resize(nh);
    f->len.resize(nh);
    for (uint32_t k = 0; k < nh; ++k) {
        f->off[k] = pre[2 * (size_t)k];
        f->len[k] = pre[2 * (size_t)k + 1] - pre[2 * (size_t)k];
    }
    (void)hipFree(f->raw);
    f->raw = nullptr;
    return MP_OK;
}

}  // namespace mp

using namespace mp;

MP_EXPORT int mp_fasta_load_device(const char* path, int32_t device, void* stream, void** out, int32_t* ascii) {
    if (!path || !out || !ascii) return fail(MP_E_ARG, "mp_fasta_load_device: null pointer");
    *out = nullptr;
    *ascii = 0;
    FastaDev* f = new FastaDev();
    f->device = device;
    const int rc = load_device(path, device, (hipStream_t)stream, f, ascii);
    if (rc || !*ascii) {
        free_fasta_dev(f);
        return rc;
    }
    *out = f;
    return MP_OK;
}

MP_EXPORT int mp_fasta_device_info(void* fasta, uint64_t* n_records, uint64_t* total_bases, const uint8_t** dev_bases) {
    FastaDev* f = (FastaDev*)fasta;
    if (!f) return fail(MP_E_ARG, "mp_fasta_device_info: null handle");
    if (n_records) *n_records = f->deflines.size();
    if (total_bases) *total_bases = f->total;
    if (dev_bases) *dev_bases = f->bases;
    return MP_OK;
}

MP_EXPORT int mp_fasta_device_record(void* fasta, uint64_t i, const uint8_t** defline, uint64_t* defline_len,
                                     uint64_t* offset, uint64_t* length) {
    FastaDev* f = (FastaDev*)fasta;
    if (!f || i >= f->deflines.size()) return fail(MP_E_ARG, "mp_fasta_device_record: bad handle or index");
    if (defline) *defline = (const uint8_t*)f->deflines[i].data();
    if (defline_len) *defline_len = f->deflines[i].size();
    if (offset) *offset = f->off[i];
    if (length) *length = f->len[i];
    return MP_OK;
}

MP_EXPORT int mp_fasta_device_read(void* fasta, uint64_t offset, uint64_t n, uint8_t* host_dst) {
    FastaDev* f = (FastaDev*)fasta;
    if (!f || (n && !host_dst) || offset > f->total || n > f->total - offset)
        return fail(MP_E_ARG, "mp_fasta_device_read: bad handle or range");
    if (!n) return MP_OK;
    MP_HIP_CHECK(hipSetDevice(f->device));
    MP_HIP_CHECK(hipMemcpy(host_dst, f->bases + offset, n, hipMemcpyDeviceToHost));
    return MP_OK;
}

MP_EXPORT void mp_fasta_device_destroy(void* fasta) { free_fasta_dev((FastaDev*)fasta); }
