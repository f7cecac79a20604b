// Native FASTA reader: replaces FASTALoader.load_file (src/merpcr/io/fasta.py:18-71).
//
// Host code only.  Reproduces the reference's text-mode read exactly:
//   * the file is decoded as strict UTF-8 (Python's default text encoding here); an
//     invalid sequence is an error, as the reference's UnicodeDecodeError;
//   * universal newlines: "\n", "\r\n" and a lone "\r" end a line;
//   * each line is str.strip()ped with Python's whitespace set (ASCII \t\n\v\f\r, the
//     \x1c-\x1f separators, space, and the Unicode spaces U+0085 U+00A0 U+1680
//     U+2000-200A U+2028 U+2029 U+202F U+205F U+3000) -- leading whitespace decides
//     whether a line is a header, both ends shape the defline;
//   * blank lines are skipped; a stripped line starting with '>' starts a record whose
//     defline is the stripped line; other lines keep exactly the characters c with
//     c.upper() in "ACGTBDHKMNRSVWXY": the 32 ASCII letters of either case plus U+017F
//     (long s, upper 'S'), kept as its UTF-8 bytes; lines before the first header are
//     dropped; empty records are kept.
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "mp_internal.h"
#include "mp_text.h"

namespace mp {

// Growable byte buffer without the zero-fill of std::vector::resize.
struct Bytes {
    uint8_t* p = nullptr;
    size_t n = 0, cap = 0;
    Bytes() = default;
    Bytes(const Bytes&) = delete;
    Bytes(Bytes&& o) noexcept : p(o.p), n(o.n), cap(o.cap) { o.p = nullptr; o.n = o.cap = 0; }
    ~Bytes() { std::free(p); }
    uint8_t* grow(size_t extra) {
        if (n + extra > cap) {
            size_t c = cap ? cap : 4096;
            while (c < n + extra) c *= 2;
            uint8_t* q = (uint8_t*)std::realloc(p, c);
            if (!q) throw std::bad_alloc();
            p = q;
            cap = c;
        }
        return p + n;
    }
};

struct FastaRec {
    std::string defline;
    Bytes seq;
};

struct Fasta {
    std::vector<FastaRec> recs;
    uint64_t total = 0;
};

static const uint8_t* keep_table() {
    static uint8_t t[256];
    static bool init = false;
    if (!init) {
        std::memset(t, 0, sizeof(t));
        for (const char* p = "ABCDGHKMNRSTVWXY"; *p; ++p) {
            t[(uint8_t)*p] = 1;
            t[(uint8_t)(*p + 32)] = 1;
        }
        init = true;
    }
    return t;
}

// Append the kept characters of sequence text [s, e) (no line ends inside).
static void filter_into(Bytes& out, const uint8_t* s, const uint8_t* e, bool ascii) {
    const uint8_t* keep = keep_table();
    uint8_t* const o0 = out.grow((size_t)(e - s));
    uint8_t* o = o0;
    if (ascii) {
        for (const uint8_t* p = s; p < e; ++p) {
            *o = *p;
            o += keep[*p];
        }
    } else {
        for (const uint8_t* p = s; p < e;) {
            if (*p < 0x80) {
                *o = *p;
                o += keep[*p];
                ++p;
            } else if (p[0] == 0xC5 && p + 1 < e && p[1] == 0xBF) {  // U+017F
                *o++ = 0xC5;
                *o++ = 0xBF;
                p += 2;
            } else {
                uint32_t cp;
                p += utf8_next(p, e, &cp);  // validated already
            }
        }
    }
    out.n += (size_t)(o - o0);
}

// Trailing str.strip() of a defline held in `h`.
static void rstrip_py(std::string& h) {
    const uint8_t* b = (const uint8_t*)h.data();
    const uint8_t* t = b + h.size();
    while (t > b) {
        uint32_t cp;
        const int k = utf8_prev(b, t, &cp);
        if (!k || !py_space(cp)) break;
        t -= k;
    }
    h.resize((size_t)(t - b));
}

static size_t find_eol(const uint8_t* d, size_t i, size_t lim, bool has_cr) {
    if (!has_cr) {  // LF-only text: glibc's vectorised memchr
        const void* q = std::memchr(d + i, '\n', lim - i);
        return q ? (size_t)((const uint8_t*)q - d) : lim;
    }
    while (i < lim && d[i] != '\n' && d[i] != '\r') ++i;
    return i;
}

}  // namespace mp

using namespace mp;

// Streaming state machine over the file: no line is ever buffered whole, so a
// single-line chromosome costs one pass.  Only an incomplete trailing UTF-8 code point
// (< 4 bytes) is carried between reads.
static int load_into(FILE* fp, const char* path, size_t chunk, Fasta* f) {
    enum { kLineStart, kSeq, kHead } st = kLineStart;
    FastaRec* cur = nullptr;
    std::string head;
    std::vector<uint8_t> buf(chunk + 4);
    size_t carry = 0;
    uint64_t consumed = 0;  // file offset of buf[0]
    bool eof = false, skip_lf = false;
    while (!eof) {
        const size_t got = std::fread(buf.data() + carry, 1, chunk, fp);
        if (got < chunk) {
            if (std::ferror(fp)) return fail(MP_E_IO, std::string("read error: ") + path);
            eof = true;
        }
        const size_t n = carry + got;
        const uint8_t* d = buf.data();
        size_t lim = n;
        if (!eof) {  // hold back an incomplete trailing code point
            size_t q = n;
            int back = 0;
            while (q > 0 && back < 3 && (d[q - 1] & 0xC0) == 0x80) { --q; ++back; }
            if (q > 0 && d[q - 1] >= 0xC0) lim = q - 1;
        }
        bool ascii = true;
        for (size_t i = 0; i < lim;) {
            if (i + 8 <= lim) {  // 8 ASCII bytes at a time
                uint64_t w;
                std::memcpy(&w, d + i, 8);
                if (!(w & 0x8080808080808080ull)) { i += 8; continue; }
            }
            if (d[i] < 0x80) { ++i; continue; }
            ascii = false;
            uint32_t cp;
            const int k = utf8_next(d + i, d + lim, &cp);
            if (!k) {
                char msg[128];
                std::snprintf(msg, sizeof(msg), "'utf-8' codec can't decode byte 0x%02x in position %llu",
                              d[i], (unsigned long long)(consumed + i));
                return fail(MP_E_DECODE, msg);
            }
            i += (size_t)k;
        }
        const bool has_cr = std::memchr(d, '\r', lim) != nullptr;
        size_t i = 0;
        while (i < lim) {
            if (skip_lf) {  // "\r\n" is one line end
                skip_lf = false;
                if (d[i] == '\n') { ++i; continue; }
            }
            if (st == kLineStart) {
                const uint8_t c = d[i];
                if (c == '\n' || c == '\r') {  // blank line
                    skip_lf = c == '\r';
                    ++i;
                    continue;
                }
                uint32_t cp = c;
                const int k = c < 0x80 ? 1 : utf8_next(d + i, d + lim, &cp);
                if (py_space(cp)) { i += (size_t)k; continue; }
                if (c == '>') {
                    st = kHead;
                    head.clear();
                } else {
                    st = kSeq;
                }
                continue;
            }
            const size_t e = find_eol(d, i, lim, has_cr);
            if (st == kHead) {
                head.append((const char*)d + i, e - i);
            } else if (cur) {  // sequence before the first header is dropped
                filter_into(cur->seq, d + i, d + e, ascii);
            }
            if (e == lim) { i = lim; break; }
            if (st == kHead) {
                rstrip_py(head);
                f->recs.emplace_back();
                cur = &f->recs.back();
                cur->defline.swap(head);
            }
            st = kLineStart;
            skip_lf = d[e] == '\r';
            i = e + 1;
        }
        carry = n - lim;
        std::memmove(buf.data(), d + lim, carry);
        consumed += lim;
    }
    if (st == kHead) {
        rstrip_py(head);
        f->recs.emplace_back();
        f->recs.back().defline.swap(head);
    }
    return MP_OK;
}

// ---------------------------------------------------------------- parallel whole-file reader
// The same rules over a memory-mapped file on every host thread the process may use.  A
// record's sequence is the kept characters of everything between its header line's end and
// the next header line's start: blank lines, line ends and the whitespace str.strip() would
// remove are never in the keep set, so filtering whole lines equals strip-then-filter.  Four
// passes, each split over the threads: strict UTF-8 validation; header lines (a line start
// -- file start or after '\n' / '\r' -- whose first non-whitespace character is '>');
// kept-byte counts of every piece of every record; the kept bytes written at their final
// offsets.  c3's 3 GB FASTA: ~4 s streaming on one thread.

static unsigned host_threads() {
    unsigned n = std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = (unsigned)CPU_COUNT(&set);
    return std::max(1u, std::min(n, 64u));
}

// f(t) on threads 0..T-1 (0 is the caller); an allocation failure on any thread is
// rethrown here after all have joined.
template <class F>
static void run_threads(unsigned T, F&& f) {
    std::atomic<bool> oom{false};
    auto body = [&](unsigned t) {
        try {
            f(t);
        } catch (const std::bad_alloc&) {
            oom = true;
        }
    };
    std::vector<std::thread> th;
    th.reserve(T);
    for (unsigned t = 1; t < T; ++t) th.emplace_back(body, t);
    body(0u);
    for (auto& x : th) x.join();
    if (oom) throw std::bad_alloc();
}

// First byte at or after p that does not continue a UTF-8 sequence (at most 3 steps).
static size_t char_start(const uint8_t* d, size_t p, size_t n) {
    for (int k = 0; k < 3 && p < n && (d[p] & 0xC0) == 0x80; ++k) ++p;
    return p;
}

struct HeaderLine {
    size_t start;  // line start
    size_t gt;     // the '>'
    size_t eol;    // first '\n' / '\r' after it, or the file end
};

// Header lines starting in [a, b): line starts are scanned with memchr when the text has
// no '\r' (LF-only files), else byte by byte.
static void find_headers(const uint8_t* d, size_t n, size_t a, size_t b, bool has_cr, std::vector<HeaderLine>& out) {
    size_t i = a;
    if (i > 0 && d[i - 1] != '\n' && d[i - 1] != '\r') {  // skip to the first line start in range
        i = find_eol(d, i, n, has_cr);
        if (i < n) ++i;
    }
    while (i < b) {
        size_t j = i;  // leading str.strip() whitespace, inside the line
        for (;;) {
            if (j >= n) break;
            const uint8_t c = d[j];
            if (c == '\n' || c == '\r') break;
            uint32_t cp = c;
            const int k = c < 0x80 ? 1 : utf8_next(d + j, d + n, &cp);
            if (!k || !py_space(cp)) break;
            j += (size_t)k;
        }
        size_t e = find_eol(d, j, n, has_cr);
        if (j < n && d[j] == '>') out.push_back({i, j, e});
        if (e >= n) break;
        i = e + 1;
    }
}

static size_t count_kept(const uint8_t* s, const uint8_t* e) {  // ASCII text
    const uint8_t* keep = keep_table();
    size_t c = 0;
    for (const uint8_t* p = s; p < e; ++p) c += keep[*p];
    return c;
}

// 1 = use the streaming reader on the same descriptor (not a regular file, size 0 -- pipes,
// /dev/stdin and /proc files report that -- or mmap failed); MP_OK / errors otherwise.
// The caller owns fd.
static int load_parallel(int fd, Fasta* f, int threads) {
    struct stat sb;
    if (fstat(fd, &sb) != 0 || !S_ISREG(sb.st_mode) || sb.st_size == 0) return 1;
    const size_t n = (size_t)sb.st_size;
    void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) return 1;
    (void)madvise(m, n, MADV_SEQUENTIAL);
    const uint8_t* d = (const uint8_t*)m;
    struct Unmap {
        void* m;
        size_t n;
        ~Unmap() { munmap(m, n); }
    } unmap{m, n};

    // threads > 0 (tests): exactly that many, whatever the file size
    const unsigned T = threads > 0 ? (unsigned)std::min<size_t>((size_t)threads, n)
                                   : (unsigned)std::min<size_t>(host_threads(), std::max<size_t>(1, n >> 20));
    std::vector<size_t> cut(T + 1);
    for (unsigned t = 0; t <= T; ++t) cut[t] = t == T ? n : char_start(d, n * t / T, n);

    // 1. strict UTF-8 (the first invalid byte of the file is reported), ASCII and '\r' flags
    std::vector<size_t> bad(T, SIZE_MAX);
    std::vector<uint8_t> ascii(T, 1), cr(T, 0);
    run_threads(T, [&](unsigned t) {
        size_t i = cut[t];
        const size_t b = cut[t + 1];
        bool asc = true;
        while (i < b) {
            if (i + 8 <= b) {
                uint64_t w;
                std::memcpy(&w, d + i, 8);
                if (!(w & 0x8080808080808080ull)) { i += 8; continue; }
            }
            if (d[i] < 0x80) { ++i; continue; }
            asc = false;
            uint32_t cp;
            const int k = utf8_next(d + i, d + n, &cp);
            if (!k) { bad[t] = i; break; }
            i += (size_t)k;
        }
        ascii[t] = asc;
        cr[t] = std::memchr(d + cut[t], '\r', b - cut[t]) != nullptr;
    });
    for (unsigned t = 0; t < T; ++t)
        if (bad[t] != SIZE_MAX) {
            char msg[128];
            std::snprintf(msg, sizeof(msg), "'utf-8' codec can't decode byte 0x%02x in position %llu", d[bad[t]],
                          (unsigned long long)bad[t]);
            return fail(MP_E_DECODE, msg);
        }
    bool has_cr = false, all_ascii = true;
    for (unsigned t = 0; t < T; ++t) {
        has_cr = has_cr || cr[t];
        all_ascii = all_ascii && ascii[t];
    }

    // 2. header lines, in file order
    std::vector<std::vector<HeaderLine>> hv(T);
    run_threads(T, [&](unsigned t) { find_headers(d, n, cut[t], cut[t + 1], has_cr, hv[t]); });
    std::vector<HeaderLine> heads;
    for (auto& v : hv) heads.insert(heads.end(), v.begin(), v.end());
    const size_t R = heads.size();
    f->recs.resize(R);
    for (size_t r = 0; r < R; ++r) {
        f->recs[r].defline.assign((const char*)d + heads[r].gt, heads[r].eol - heads[r].gt);
        rstrip_py(f->recs[r].defline);
    }
    if (!R) return MP_OK;

    // 3./4. every record's text [eol_r, start_{r+1}) as one index space cut into ~8 pieces
    // per thread at character starts; piece sizes counted, then the kept bytes written
    struct Piece {
        size_t rec, a, b, off;
    };
    std::vector<size_t> rs(R), re(R), base(R + 1, 0);
    for (size_t r = 0; r < R; ++r) {
        rs[r] = heads[r].eol;
        re[r] = r + 1 < R ? heads[r + 1].start : n;
        base[r + 1] = base[r] + (re[r] - rs[r]);
    }
    const size_t total = base[R];
    const size_t np = std::max<size_t>(1, threads > 0 ? std::min<size_t>((size_t)T * 8, total)
                                                      : std::min<size_t>((size_t)T * 8, total >> 16));
    std::vector<Piece> pc;
    for (size_t r = 0, q = 0; r < R; ++r) {  // pieces: [q-th cut, (q+1)-th cut) clipped to records
        size_t a = rs[r];
        while (a < re[r]) {
            while (q + 1 < np && total * (q + 1) / np <= base[r] + (a - rs[r])) ++q;
            size_t b = q + 1 < np ? rs[r] + (total * (q + 1) / np - base[r]) : re[r];
            b = std::min(b, re[r]);
            if (b < re[r]) b = char_start(d, b, re[r]);
            if (b <= a) b = re[r];
            pc.push_back({r, a, b, 0});
            a = b;
        }
    }
    std::atomic<size_t> next{0};
    std::vector<size_t> kept(pc.size());
    run_threads(T, [&](unsigned) {
        for (size_t i; (i = next.fetch_add(1)) < pc.size();)
            kept[i] = all_ascii ? count_kept(d + pc[i].a, d + pc[i].b) : 0;
    });
    if (!all_ascii) {  // multi-byte text: the streaming filter's own count
        next = 0;
        std::vector<Bytes> tmp(pc.size());
        run_threads(T, [&](unsigned) {
            for (size_t i; (i = next.fetch_add(1)) < pc.size();) {
                filter_into(tmp[i], d + pc[i].a, d + pc[i].b, false);
                kept[i] = tmp[i].n;
            }
        });
        for (size_t i = 0, r = (size_t)-1, o = 0; i < pc.size(); ++i) {
            if (pc[i].rec != r) { r = pc[i].rec; o = 0; }
            pc[i].off = o;
            o += kept[i];
            Bytes& out = f->recs[r].seq;
            std::memcpy(out.grow(kept[i]), tmp[i].p, kept[i]);
            out.n += kept[i];
        }
        return MP_OK;
    }
    std::vector<size_t> rlen(R, 0);
    for (size_t i = 0; i < pc.size(); ++i) {
        pc[i].off = rlen[pc[i].rec];
        rlen[pc[i].rec] += kept[i];
    }
    for (size_t r = 0; r < R; ++r) {
        Bytes& out = f->recs[r].seq;
        if (rlen[r]) out.grow(rlen[r]);
        out.n = rlen[r];
    }
    next = 0;
    run_threads(T, [&](unsigned) {
        const uint8_t* keep = keep_table();
        for (size_t i; (i = next.fetch_add(1)) < pc.size();) {
            // a store per kept byte only: the unconditional store of filter_into would land
            // one byte past this piece, on the next piece's first byte
            uint8_t* o = f->recs[pc[i].rec].seq.p + pc[i].off;
            for (const uint8_t* p = d + pc[i].a, *e = d + pc[i].b; p < e; ++p)
                if (keep[*p]) *o++ = *p;
        }
    });
    return MP_OK;
}

static int load_stream(FILE* fp, const char* path, uint64_t chunk_bytes, void** out);

MP_EXPORT int mp_fasta_load(const char* path, void** out) { return mp_fasta_load_parallel(path, 0, out); }

MP_EXPORT int mp_fasta_load_parallel(const char* path, int32_t threads, void** out) {
    if (!path || !out || threads < 0) return fail(MP_E_ARG, "mp_fasta_load: bad argument");
    *out = nullptr;
    Fasta* f = new (std::nothrow) Fasta();
    if (!f) return fail(MP_E_NOMEM, "mp_fasta_load: out of host memory");
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) {
        delete f;
        return fail(MP_E_IO, std::string("cannot open FASTA file: ") + path);
    }
    int rc;
    try {
        rc = load_parallel(fd, f, threads);
    } catch (const std::bad_alloc&) {
        rc = fail(MP_E_NOMEM, "mp_fasta_load: out of host memory");
    }
    if (rc == 1) {  // not mappable: the streaming reader, on the descriptor already open (a pipe
                    // cannot be opened twice)
        delete f;
        FILE* fp = fdopen(fd, "rb");
        if (!fp) {
            ::close(fd);
            return fail(MP_E_IO, std::string("cannot open FASTA file: ") + path);
        }
        return load_stream(fp, path, 0, out);
    }
    ::close(fd);
    if (rc) {
        delete f;
        return rc;
    }
    for (const auto& r : f->recs) f->total += r.seq.n;
    *out = f;
    return MP_OK;
}

MP_EXPORT int mp_fasta_load_chunked(const char* path, uint64_t chunk_bytes, void** out) {
    if (!path || !out) return fail(MP_E_ARG, "mp_fasta_load: null pointer");
    if (chunk_bytes && chunk_bytes < 4) return fail(MP_E_ARG, "mp_fasta_load: chunk_bytes must be >= 4");
    *out = nullptr;
    FILE* fp = std::fopen(path, "rb");
    if (!fp) return fail(MP_E_IO, std::string("cannot open FASTA file: ") + path);
    return load_stream(fp, path, chunk_bytes, out);
}

// The streaming reader over an open stream, which it closes.
static int load_stream(FILE* fp, const char* path, uint64_t chunk_bytes, void** out) {
    const size_t chunk = chunk_bytes ? (size_t)chunk_bytes : (size_t)64 << 20;
    Fasta* f = new (std::nothrow) Fasta();
    int rc = f ? MP_OK : fail(MP_E_NOMEM, "mp_fasta_load: out of host memory");
    if (!rc) {
        try {
            rc = load_into(fp, path, chunk, f);
        } catch (const std::bad_alloc&) {
            rc = fail(MP_E_NOMEM, "mp_fasta_load: out of host memory");
        }
    }
    std::fclose(fp);
    if (rc) {
        delete f;
        return rc;
    }
    for (const auto& r : f->recs) f->total += r.seq.n;
    *out = f;
    return MP_OK;
}

MP_EXPORT int mp_fasta_info(void* fasta, uint64_t* n_records, uint64_t* total_bytes) {
    Fasta* f = (Fasta*)fasta;
    if (!f) return fail(MP_E_ARG, "mp_fasta_info: null handle");
    if (n_records) *n_records = f->recs.size();
    if (total_bytes) *total_bytes = f->total;
    return MP_OK;
}

MP_EXPORT int mp_fasta_record(void* fasta, uint64_t i, const uint8_t** defline, uint64_t* defline_len,
                              const uint8_t** seq, uint64_t* seq_len) {
    Fasta* f = (Fasta*)fasta;
    if (!f || i >= f->recs.size()) return fail(MP_E_ARG, "mp_fasta_record: bad handle or index");
    const FastaRec& r = f->recs[i];
    if (defline) *defline = (const uint8_t*)r.defline.data();
    if (defline_len) *defline_len = r.defline.size();
    if (seq) *seq = r.seq.p;
    if (seq_len) *seq_len = r.seq.n;
    return MP_OK;
}

MP_EXPORT int mp_fasta_record_ascii(void* fasta, uint64_t i, int32_t* ascii) {
    Fasta* f = (Fasta*)fasta;
    if (!f || !ascii || i >= f->recs.size()) return fail(MP_E_ARG, "mp_fasta_record_ascii: bad handle or index");
    const FastaRec& r = f->recs[i];  // the only multi-byte character the filter keeps is U+017F (C5 BF)
    *ascii = (r.seq.n == 0 || std::memchr(r.seq.p, 0xC5, r.seq.n) == nullptr) ? 1 : 0;
    return MP_OK;
}

// Large handles are freed on a detached thread: returning gigabytes of touched pages to
// the system took ~0.26 s of the CLI's wall time for c3's 3 GB genome.
MP_EXPORT void mp_fasta_destroy(void* fasta) {
    Fasta* f = (Fasta*)fasta;
    if (!f) return;
    if (f->total < ((uint64_t)64 << 20)) {
        delete f;
        return;
    }
    try {
        std::thread([f] { delete f; }).detach();
    } catch (...) {
        delete f;
    }
}
