// Native STS parser: replaces MerPCR.load_sts_file + _parse_pcr_size + _hash_value +
// _reverse_complement + _insert_sts (src/merpcr/core/engine.py:193-359).
//
// Host code only.  The file is read as the reference reads it (strict UTF-8,
// readlines() with universal newlines), and each line follows engine.py:216-287:
//   * strip() with Python's whitespace set; skip blank lines and lines starting '#';
//   * split on '\t'; fewer than 4 fields stops the load (the records inserted so far
//     stay, as in the reference, and the caller returns False);
//   * primer1/primer2 = fields[1]/fields[2] upper-cased; size = _parse_pcr_size(fields[3]);
//     alias = fields[4] or "";
//   * a primer shorter than W skips the line; l1+l2 > size raises size to l1+l2;
//     max_pcr_size is the max over the kept lines;
//   * '+' record (p1, p2) keyed by hash(p1), '-' record (p2, revcomp(p1)) keyed by
//     hash(p2), each inserted only when its primer has an all-ACGTU W-window.
// Python's str.upper() and int() have Unicode rules (case mappings that change length,
// non-ASCII digits and spaces): a primer or size field holding a non-ASCII character,
// or a size beyond 2^62, sets status MP_STS_PYTHON and the caller parses the file with
// its own restatement of those rules.  Ids and aliases are copied verbatim (any UTF-8).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mp_internal.h"
#include "mp_text.h"

namespace mp {

struct Sts {
    int32_t status = MP_STS_OK;
    uint64_t bad_line = 0, n_short = 0, n_ambig = 0, n_badsize = 0, max_pcr = 0;
    std::vector<uint32_t> key, hash_off, text_idx;
    std::vector<uint64_t> pcr, line;
    std::vector<uint8_t> direct;  // '+' or '-'
    std::vector<uint8_t> p1, p2, text;
    std::vector<uint64_t> p1_off{0}, p2_off{0}, text_off{0};  // text: id0, alias0, id1, ...
    std::vector<uint8_t> rtext;       // mp_sts_record_texts, built on first request
    std::vector<uint64_t> rtext_off;
};

// Python int() of an ASCII field: surrounding whitespace, optional sign, decimal digits
// with single '_' separators.  Returns 1 on success, 0 for ValueError, -1 if |v| >= 2^62.
static int py_int(const uint8_t* b, const uint8_t* e, int64_t* v) {
    while (b < e && py_space(*b)) ++b;
    while (e > b && py_space(e[-1])) --e;
    bool neg = false;
    if (b < e && (*b == '+' || *b == '-')) neg = *b++ == '-';
    if (b == e || !(*b >= '0' && *b <= '9')) return 0;
    int64_t x = 0;
    bool prev_us = false;
    for (; b < e; ++b) {
        if (*b == '_') {
            if (prev_us) return 0;
            prev_us = true;
            continue;
        }
        if (!(*b >= '0' && *b <= '9')) return 0;
        prev_us = false;
        x = x * 10 + (*b - '0');
        if (x >= (int64_t(1) << 62)) return -1;
    }
    if (prev_us) return 0;
    *v = neg ? -x : x;
    return 1;
}

// _parse_pcr_size (engine.py:304-322); -1 in *ok asks for the Python parser.
static int64_t parse_size(const uint8_t* b, const uint8_t* e, int64_t dflt, int* ok) {
    *ok = 1;
    const uint8_t* dash = (const uint8_t*)std::memchr(b, '-', (size_t)(e - b));
    int64_t lo, hi;
    if (dash) {
        if (std::memchr(dash + 1, '-', (size_t)(e - dash - 1)) || dash == b || dash + 1 == e) return dflt;
        const int r1 = py_int(b, dash, &lo), r2 = r1 == 1 ? py_int(dash + 1, e, &hi) : 0;
        if (r1 < 0 || r2 < 0) { *ok = -1; return 0; }
        if (!r1 || !r2) return dflt;
        return (lo + hi) >> 1;  // both >= 0: no '-' inside the parts
    }
    const int r = py_int(b, e, &lo);
    if (r < 0) { *ok = -1; return 0; }
    return r && lo > 0 ? lo : dflt;
}

static int code2(uint8_t c) {
    switch (c) {
        case 'A': return 0;
        case 'C': return 1;
        case 'G': return 2;
        case 'T': case 'U': return 3;
        default: return -1;
    }
}

// _hash_value on an upper-cased primer (engine.py:331-355): first all-ACGTU W-window.
static bool hash_primer(const uint8_t* p, size_t L, int W, uint32_t* off, uint32_t* key) {
    if ((int64_t)L < W) return false;
    uint64_t v = 0;
    int run = 0;
    const uint64_t mask = (W >= 32) ? ~0ull : ((1ull << (2 * W)) - 1);
    for (size_t i = 0; i < L; ++i) {
        const int c = code2(p[i]);
        if (c < 0) { run = 0; v = 0; continue; }
        v = ((v << 2) | (uint64_t)c) & mask;
        if (++run >= W) {
            *off = (uint32_t)(i + 1 - W);
            *key = (uint32_t)v;
            return true;
        }
    }
    return false;
}

// _reverse_complement of an upper-cased primer (engine.py:112-135, 357-359).
static uint8_t compl_base(uint8_t c) {
    switch (c) {
        case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A';
        case 'U': return 'A'; case 'B': return 'V'; case 'V': return 'B'; case 'D': return 'H';
        case 'H': return 'D'; case 'K': return 'M'; case 'M': return 'K'; case 'R': return 'Y';
        case 'Y': return 'R'; case 'S': return 'S'; case 'W': return 'W'; case 'N': return 'N';
        case 'X': return 'X';
        default: return 'N';
    }
}

static void add_record(Sts* s, uint32_t key, uint32_t off, uint64_t size, uint64_t line_no, uint8_t dir,
                       const uint8_t* a, size_t la, const uint8_t* b, size_t lb, bool b_rc) {
    s->key.push_back(key);
    s->hash_off.push_back(off);
    s->pcr.push_back(size);
    s->line.push_back(line_no);
    s->direct.push_back(dir);
    s->text_idx.push_back((uint32_t)(s->text_off.size() / 2 - 1));
    s->p1.insert(s->p1.end(), a, a + la);
    s->p1_off.push_back(s->p1.size());
    if (b_rc) {
        for (size_t i = lb; i-- > 0;) s->p2.push_back(compl_base(b[i]));
    } else {
        s->p2.insert(s->p2.end(), b, b + lb);
    }
    s->p2_off.push_back(s->p2.size());
}

static void parse_line(Sts* s, const uint8_t* b, const uint8_t* e, uint64_t line_no, int W, int64_t dflt) {
    // strip()
    while (b < e) {
        uint32_t cp;
        const int k = utf8_next(b, e, &cp);
        if (!py_space(cp)) break;
        b += k;
    }
    while (e > b) {
        uint32_t cp;
        const int k = utf8_prev(b, e, &cp);
        if (!k || !py_space(cp)) break;
        e -= k;
    }
    if (b == e || *b == '#') return;
    const uint8_t* f[6];
    const uint8_t* fe[6];
    int nf = 0;
    for (const uint8_t* p = b;;) {
        const uint8_t* t = (const uint8_t*)std::memchr(p, '\t', (size_t)(e - p));
        if (nf < 6) { f[nf] = p; fe[nf] = t ? t : e; }
        ++nf;
        if (!t) break;
        p = t + 1;
    }
    if (nf < 4) {
        s->status = MP_STS_BAD_LINE;
        s->bad_line = line_no;
        return;
    }
    for (int i = 1; i <= 3; ++i)
        for (const uint8_t* p = f[i]; p < fe[i]; ++p)
            if (*p >= 0x80) { s->status = MP_STS_PYTHON; return; }
    std::string p1((const char*)f[1], (size_t)(fe[1] - f[1])), p2((const char*)f[2], (size_t)(fe[2] - f[2]));
    for (char& c : p1) if (c >= 'a' && c <= 'z') c -= 32;
    for (char& c : p2) if (c >= 'a' && c <= 'z') c -= 32;
    int ok;
    int64_t size = parse_size(f[3], fe[3], dflt, &ok);
    if (ok < 0) { s->status = MP_STS_PYTHON; return; }
    if ((int64_t)p1.size() < W || (int64_t)p2.size() < W) {
        ++s->n_short;
        return;
    }
    const int64_t lsum = (int64_t)(p1.size() + p2.size());
    if (lsum > size) {
        ++s->n_badsize;
        size = lsum;
    }
    if ((uint64_t)size > s->max_pcr) s->max_pcr = (uint64_t)size;
    // id and alias (shared by the line's two records)
    s->text.insert(s->text.end(), f[0], fe[0]);
    s->text_off.push_back(s->text.size());
    if (nf > 4) s->text.insert(s->text.end(), f[4], fe[4]);
    s->text_off.push_back(s->text.size());
    const uint8_t* a = (const uint8_t*)p1.data();
    const uint8_t* c = (const uint8_t*)p2.data();
    uint32_t off, key;
    if (hash_primer(a, p1.size(), W, &off, &key))
        add_record(s, key, off, (uint64_t)size, line_no, '+', a, p1.size(), c, p2.size(), false);
    else
        ++s->n_ambig;
    if (hash_primer(c, p2.size(), W, &off, &key))
        add_record(s, key, off, (uint64_t)size, line_no, '-', c, p2.size(), a, p1.size(), true);
    else
        ++s->n_ambig;
}

}  // namespace mp

using namespace mp;

MP_EXPORT int mp_sts_parse(const char* path, int32_t wordsize, int64_t default_pcr_size, void** out) {
    if (!path || !out) return fail(MP_E_ARG, "mp_sts_parse: null pointer");
    if (wordsize < 1 || wordsize > 16) return fail(MP_E_ARG, "mp_sts_parse: wordsize out of range");
    *out = nullptr;
    FILE* fp = std::fopen(path, "rb");
    if (!fp) return fail(MP_E_IO, std::string("cannot open STS file: ") + path);
    std::vector<uint8_t> data;
    try {
        uint8_t tmp[1 << 16];
        size_t got;
        while ((got = std::fread(tmp, 1, sizeof(tmp), fp)) > 0) data.insert(data.end(), tmp, tmp + got);
    } catch (const std::bad_alloc&) {
        std::fclose(fp);
        return fail(MP_E_NOMEM, "mp_sts_parse: out of host memory");
    }
    const bool err = std::ferror(fp);
    std::fclose(fp);
    if (err) return fail(MP_E_IO, std::string("read error: ") + path);
    const uint8_t* d = data.data();
    const size_t n = data.size();
    for (size_t i = 0; i < n;) {  // readlines() decodes the whole file first
        if (d[i] < 0x80) { ++i; continue; }
        uint32_t cp;
        const int k = utf8_next(d + i, d + n, &cp);
        if (!k) {
            char msg[128];
            std::snprintf(msg, sizeof(msg), "'utf-8' codec can't decode byte 0x%02x in position %llu", d[i],
                          (unsigned long long)i);
            return fail(MP_E_DECODE, msg);
        }
        i += (size_t)k;
    }
    Sts* s = new (std::nothrow) Sts();
    if (!s) return fail(MP_E_NOMEM, "mp_sts_parse: out of host memory");
    try {
        uint64_t line_no = 0;
        size_t b = 0;
        while (b < n && s->status == MP_STS_OK) {
            size_t e = b;
            while (e < n && d[e] != '\n' && d[e] != '\r') ++e;
            ++line_no;
            parse_line(s, d + b, d + e, line_no, wordsize, default_pcr_size);
            if (e < n && d[e] == '\r' && e + 1 < n && d[e + 1] == '\n') ++e;
            b = e + 1;
        }
    } catch (const std::bad_alloc&) {
        delete s;
        return fail(MP_E_NOMEM, "mp_sts_parse: out of host memory");
    }
    *out = s;
    return MP_OK;
}

MP_EXPORT int mp_sts_info(void* sts, int32_t* status, uint64_t* counts) {
    Sts* s = (Sts*)sts;
    if (!s || !status || !counts) return fail(MP_E_ARG, "mp_sts_info: null pointer");
    *status = s->status;
    counts[0] = s->key.size();
    counts[1] = s->bad_line;
    counts[2] = s->n_short;
    counts[3] = s->n_ambig;
    counts[4] = s->n_badsize;
    counts[5] = s->max_pcr;
    counts[6] = s->p1.size();
    counts[7] = s->p2.size();
    counts[8] = s->text.size();
    counts[9] = s->text_off.size() - 1;
    return MP_OK;
}

MP_EXPORT int mp_sts_arrays(void* sts, const void** ptrs) {
    Sts* s = (Sts*)sts;
    if (!s || !ptrs) return fail(MP_E_ARG, "mp_sts_arrays: null pointer");
    const void* v[] = {s->key.data(), s->hash_off.data(), s->pcr.data(), s->line.data(), s->direct.data(),
                       s->text_idx.data(), s->p1.data(), s->p1_off.data(), s->p2.data(), s->p2_off.data(),
                       s->text.data(), s->text_off.data()};
    std::memcpy(ptrs, v, sizeof(v));
    return MP_OK;
}

MP_EXPORT int mp_sts_record_texts(void* sts, const uint8_t** text, const uint64_t** off, uint64_t* n_bytes) {
    Sts* s = (Sts*)sts;
    if (!s || !text || !off || !n_bytes) return fail(MP_E_ARG, "mp_sts_record_texts: null pointer");
    const size_t n = s->key.size();
    if (s->rtext_off.size() != n + 1) {
        try {
            s->rtext_off.assign(n + 1, 0);
            uint64_t tot = 0;
            for (size_t i = 0; i < n; ++i) {
                const uint32_t t = s->text_idx[i];
                tot += (s->text_off[2 * t + 2] - s->text_off[2 * t]) + 5;  // id \t alias \t ( d )
                s->rtext_off[i + 1] = tot;
            }
            s->rtext.resize(tot);
            uint8_t* o = s->rtext.data();
            for (size_t i = 0; i < n; ++i) {
                const uint32_t t = s->text_idx[i];
                const uint64_t a0 = s->text_off[2 * t], a1 = s->text_off[2 * t + 1], a2 = s->text_off[2 * t + 2];
                std::memcpy(o, s->text.data() + a0, a1 - a0);
                o += a1 - a0;
                *o++ = '\t';
                std::memcpy(o, s->text.data() + a1, a2 - a1);
                o += a2 - a1;
                *o++ = '\t';
                *o++ = '(';
                *o++ = s->direct[i];
                *o++ = ')';
            }
        } catch (const std::bad_alloc&) {
            s->rtext_off.clear();
            return fail(MP_E_NOMEM, "mp_sts_record_texts: out of host memory");
        }
    }
    *text = s->rtext.data();
    *off = s->rtext_off.data();
    *n_bytes = s->rtext.size();
    return MP_OK;
}

MP_EXPORT void mp_sts_destroy(void* sts) { delete (Sts*)sts; }
