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
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
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

MP_EXPORT int mp_fasta_load(const char* path, void** out) { return mp_fasta_load_chunked(path, 0, out); }

MP_EXPORT int mp_fasta_load_chunked(const char* path, uint64_t chunk_bytes, void** out) {
    if (!path || !out) return fail(MP_E_ARG, "mp_fasta_load: null pointer");
    if (chunk_bytes && chunk_bytes < 4) return fail(MP_E_ARG, "mp_fasta_load: chunk_bytes must be >= 4");
    *out = nullptr;
    const size_t chunk = chunk_bytes ? (size_t)chunk_bytes : (size_t)64 << 20;
    FILE* fp = std::fopen(path, "rb");
    if (!fp) return fail(MP_E_IO, std::string("cannot open FASTA file: ") + path);
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

MP_EXPORT void mp_fasta_destroy(void* fasta) { delete (Fasta*)fasta; }
