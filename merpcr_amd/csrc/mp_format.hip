// Native hit formatter: replaces the per-hit print of MerPCR.search
// (src/merpcr/core/engine.py:436-444):
//     f"{seq_label}\t{pos1 + 1}..{pos2 + 1}\t{sts.id}\t{sts.alias}\t({sts.direct})"
// one line per hit, '\n'-terminated, in the order given (the sorted mp_search output).
// The caller passes each sequence's label and each record's "{id}\t{alias}\t({direct})"
// text as UTF-8 bytes; the formatter only adds the tabs, the 1-based decimal
// coordinates and the newlines.  Host code; large outputs are split across threads
// (sizes first, then each thread writes its own byte range).
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "mp_internal.h"

namespace mp {

static inline int dec_len(uint64_t v) {
    int n = 1;
    while (v >= 10) { v /= 10; ++n; }
    return n;
}

static inline uint8_t* put_dec(uint8_t* o, uint64_t v) {
    const int n = dec_len(v);
    for (int i = n - 1; i >= 0; --i) { o[i] = (uint8_t)('0' + v % 10); v /= 10; }
    return o + n;
}

struct FormatIn {
    const mp_hit* hits;
    const uint8_t* labels;
    const uint64_t* label_off;
    const uint8_t* rec_text;
    const uint64_t* rec_off;
};

static inline uint64_t line_len(const FormatIn& in, const mp_hit& h) {
    return (in.label_off[h.seq + 1] - in.label_off[h.seq]) + 1 + dec_len(h.pos1 + 1) + 2 + dec_len(h.pos2 + 1) +
           1 + (in.rec_off[h.rec + 1] - in.rec_off[h.rec]) + 1;
}

static void format_range(const FormatIn& in, uint64_t b, uint64_t e, uint8_t* o) {
    for (uint64_t i = b; i < e; ++i) {
        const mp_hit& h = in.hits[i];
        const uint64_t l0 = in.label_off[h.seq], l1 = in.label_off[h.seq + 1];
        std::memcpy(o, in.labels + l0, l1 - l0);
        o += l1 - l0;
        *o++ = '\t';
        o = put_dec(o, h.pos1 + 1);
        *o++ = '.';
        *o++ = '.';
        o = put_dec(o, h.pos2 + 1);
        *o++ = '\t';
        const uint64_t r0 = in.rec_off[h.rec], r1 = in.rec_off[h.rec + 1];
        std::memcpy(o, in.rec_text + r0, r1 - r0);
        o += r1 - r0;
        *o++ = '\n';
    }
}

}  // namespace mp

using namespace mp;

MP_EXPORT int mp_format_hits(const mp_hit* hits, uint64_t n_hits, const uint8_t* labels, const uint64_t* label_off,
                             uint32_t n_seq, const uint8_t* rec_text, const uint64_t* rec_off, uint32_t n_rec,
                             uint8_t* out, uint64_t cap, uint64_t* n_bytes) {
    if (!n_bytes || (n_hits && (!hits || !label_off || !rec_off)))
        return fail(MP_E_ARG, "mp_format_hits: null pointer");
    const FormatIn in{hits, labels, label_off, rec_text, rec_off};
    for (uint64_t i = 0; i < n_hits; ++i)
        if (hits[i].seq >= n_seq || hits[i].rec >= n_rec)
            return fail(MP_E_ARG, "mp_format_hits: hit " + std::to_string(i) + " names an unknown sequence or record");

    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const uint64_t per = 1u << 13;  // hits per thread at least (c3: 200k hits over every core)
    const unsigned nt = (unsigned)std::min<uint64_t>(std::min(hw, 32u), (n_hits + per - 1) / per);
    std::vector<uint64_t> part(nt + 1, 0);
    auto bound = [&](unsigned t) { return n_hits * t / std::max(1u, nt); };
    if (nt <= 1) {
        uint64_t sz = 0;
        for (uint64_t i = 0; i < n_hits; ++i) sz += line_len(in, hits[i]);
        part.assign(2, 0);
        part[1] = sz;
    } else {
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                uint64_t sz = 0;
                for (uint64_t i = bound(t); i < bound(t + 1); ++i) sz += line_len(in, hits[i]);
                part[t + 1] = sz;
            });
        for (auto& x : th) x.join();
        for (unsigned t = 0; t < nt; ++t) part[t + 1] += part[t];
    }
    const uint64_t need = part.back();
    *n_bytes = need;
    if (!out) return MP_OK;  // size query
    if (cap < need) return fail(MP_E_CAP, "mp_format_hits: output buffer too small");
    if (nt <= 1) {
        format_range(in, 0, n_hits, out);
    } else {
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nt; ++t)
            th.emplace_back([&, t] { format_range(in, bound(t), bound(t + 1), out + part[t]); });
        for (auto& x : th) x.join();
    }
    return MP_OK;
}
