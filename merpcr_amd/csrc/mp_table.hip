// Seed table: host build + upload to HBM.
//
// Replaces MerPCR.sts_table / sts_records (src/merpcr/core/engine.py:193-329):
// the Python host hands over the oriented records in sts_records order with the
// (hash_offset, key) pair _hash_value computed for primer1 (engine.py:331-355);
// this file turns them into the device structures the scan kernel probes.
#include <sched.h>

#include <algorithm>
#include <cmath>
#include <chrono>
#include <cstring>
#include <unordered_map>

#include "mp_internal.h"

namespace mp {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
    set_error(msg);
    return code;
}

hipError_t poll_event(hipEvent_t ev, double timeout_s) {
    using clk = std::chrono::steady_clock;
    const clk::time_point t0 = clk::now();
    for (uint32_t i = 0;; ++i) {
        const hipError_t e = hipEventQuery(ev);
        if (e != hipErrorNotReady) return e;
        if (i < 4096) continue;  // ~20 us of tight spin
        if (timeout_s > 0 && (i & 255) == 0 &&
            std::chrono::duration<double>(clk::now() - t0).count() > timeout_s)
            return hipErrorNotReady;
        sched_yield();
    }
}

template <class T>
static int upload(T** dst, const T* src, size_t n, uint64_t* bytes) {
    const size_t nb = std::max<size_t>(n, 1) * sizeof(T);
    MP_HIP_CHECK(hipMalloc((void**)dst, nb));
    if (n) MP_HIP_CHECK(hipMemcpy(*dst, src, n * sizeof(T), hipMemcpyHostToDevice));
    *bytes += nb;
    return MP_OK;
}

static void free_table(Table* t) {
    if (!t) return;
    free_table(t->split_a); free_table(t->split_b); free_table(t->split_rest);
    hipFree(t->dents12);
    hipFree(t->filt); hipFree(t->lfilt); hipFree(t->rk); hipFree(t->dents); hipFree(t->dents8); hipFree(t->dents16); hipFree(t->kgrp); hipFree(t->kgrp4); hipFree(t->binfo); hipFree(t->dfilt); hipFree(t->dgrp); hipFree(t->dgesc); hipFree(t->dsum); hipFree(t->dents_pad); hipFree(t->slots); hipFree(t->ents);
    hipFree(t->recs); hipFree(t->rank); hipFree(t->inv_rank); hipFree(t->rank_rec); hipFree(t->planes); hipFree(t->prec);
    hipFree(t->pchars);
    delete t;
}

static inline uint8_t upcase(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }

// Accept planes of one primer: for every 32-base chunk, four spaced masks telling
// which genome base (A, C, G, T) satisfies the compare rule of engine.py:613-631
// at each primer position; positions past the primer end accept everything.
static void build_planes(const uint8_t* p, uint32_t L, int iupac, std::vector<uint64_t>& out) {
    const uint32_t chunks = (L + 31) / 32;
    for (uint32_t c = 0; c < chunks; ++c) {
        uint64_t acc[4] = {0, 0, 0, 0};
        for (uint32_t i = 0; i < 32; ++i) {
            const uint32_t pos = c * 32 + i;
            const int bit = 62 - 2 * (int)i;
            if (pos >= L) {
                for (int b = 0; b < 4; ++b) acc[b] |= 1ull << bit;
                continue;
            }
            const uint8_t ch = upcase(p[pos]);
            for (int b = 0; b < 4; ++b) {
                if (char_match((uint8_t)"ACGT"[b], ch, iupac)) acc[b] |= 1ull << bit;
            }
        }
        for (int b = 0; b < 4; ++b) out.push_back(acc[b]);
    }
}

}  // namespace mp

using namespace mp;

MP_EXPORT int32_t mp_abi_version(void) { return MP_ABI_VERSION; }

MP_EXPORT const char* mp_last_error(void) { return g_last_error.c_str(); }

MP_EXPORT int mp_device_count(int32_t* n) {
    if (!n) return fail(MP_E_ARG, "mp_device_count: null pointer");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *n = (e == hipSuccess) ? c : 0;
    return MP_OK;
}

// Builds one table.  rec_map (sub-tables of a split, see kSplitSeed): record r of these
// arrays is record rec_map[r] of the parent, which Entry::rec names.  gap_len > 0: the keys
// are gapped seeds (bases [0, gap_at) ++ [gap_at + gap_len, gap_at + gap_len + W - gap_at)):
// no compact heads (they restate a primer from a contiguous key), and the key groups hold
// the gap's bases and the gap_post bases after the seed's span for the gapped scan's
// one-mismatch test (kgrp_pass).
static int build_table(const mp_params& p, int32_t device, uint32_t n_rec, const uint32_t* key,
                       const uint32_t* hash_off, const uint64_t* pcr_size, const uint8_t* primer1,
                       const uint64_t* p1_off, const uint8_t* primer2, const uint64_t* p2_off,
                       const uint32_t* rec_map, uint32_t gap_at, uint32_t gap_len, uint32_t gap_post,
                       const mp_table_options& topt, Table** table_out) {
    Table* t = new Table();
    t->prm = p;
    t->topt = topt;
    t->device = device;
    t->n_rec = n_rec;
    t->gap_at = gap_at;
    t->gap_len = gap_len;
    t->gap_post = gap_post;
    const bool gapped = gap_len != 0;
    int rc = MP_OK;
    do {
        if (hipSetDevice(device) != hipSuccess) { rc = fail(MP_E_HIP, "hipSetDevice failed"); break; }
        const uint32_t W = (uint32_t)p.wordsize;
        const uint64_t key_limit = (W == 16) ? (1ull << 32) : (1ull << (2 * W));
        uint64_t dev_bytes_pre = 0;  // uploads made before the final batch (the 8-B IUPAC heads)

        // ---- buckets in first-appearance order, records in insertion order
        std::unordered_map<uint32_t, uint32_t> bucket_of;
        bucket_of.reserve(n_rec * 2 + 16);
        std::vector<uint32_t> bkey, bcount, rec_bucket(n_rec);
        for (uint32_t r = 0; r < n_rec; ++r) {
            if ((uint64_t)key[r] >= key_limit) { rc = fail(MP_E_ARG, "record key exceeds 4^W"); break; }
            auto it = bucket_of.find(key[r]);
            uint32_t b;
            if (it == bucket_of.end()) {
                b = (uint32_t)bkey.size();
                bucket_of.emplace(key[r], b);
                bkey.push_back(key[r]);
                bcount.push_back(0);
            } else {
                b = it->second;
            }
            rec_bucket[r] = b;
            bcount[b]++;
        }
        if (rc) break;
        const uint32_t nb = (uint32_t)bkey.size();
        t->n_keys = nb;
        std::vector<uint32_t> boff(nb + 1, 0);
        for (uint32_t b = 0; b < nb; ++b) {
            boff[b + 1] = boff[b] + bcount[b];
            t->max_bucket = std::max<uint64_t>(t->max_bucket, bcount[b]);
        }
        std::vector<uint32_t> fillp(boff.begin(), boff.end() - 1), blist(n_rec);
        for (uint32_t r = 0; r < n_rec; ++r) blist[fillp[rec_bucket[r]]++] = r;


        // ---- presence filter: direct bitmap for small W, hashed filter above
        t->filt_direct = (W <= (uint32_t)kDirectFilterMaxW);
        t->filt_log2 = t->filt_direct ? 2 * W : (uint32_t)kHashedFilterLog2;
        std::vector<uint32_t> filt(std::max<uint64_t>((1ull << t->filt_log2) / 32, 1), 0);
        for (uint32_t b = 0; b < nb; ++b) {
            const uint32_t idx = t->filt_direct ? bkey[b] : filter_index(bkey[b], t->filt_log2);
            filt[idx >> 5] |= 1u << (idx & 31);
        }
        t->lds_exact = (2 * W <= (uint32_t)kLdsFilterLog2);
        std::vector<uint32_t> lfilt(kLdsFilterWords, 0);
        const bool blocked = !t->lds_exact && t->filt_direct;  // W 11..13: lds_block_mask
        t->lds_k = blocked && nb > kLdsK2Keys ? 2 : 1;
        // mp_table_options.lds_k 1..3 forces the bits per key (the level-1 A/B of DESIGN 4.2; the
        // scan launches k = 3 only on its key-group and 16-B-head paths)
        if (topt.lds_k && blocked) t->lds_k = std::min(3, std::max(1, (int)topt.lds_k));
        for (uint32_t b = 0; b < nb; ++b) {
            const uint32_t idx = lds_bit(bkey[b], W, t->lds_exact);
            if (blocked) {
                const uint32_t x = bkey[b] << (32u - 2u * W);
                lfilt[idx >> 5] |= lds_block_mask(x, 32u - 2u * W, t->lds_k);
            } else {
                lfilt[idx >> 5] |= 1u << (idx & 31);
            }
        }

        // ---- records, primer planes and bytes
        std::vector<DevRec> recs(n_rec);
        std::vector<uint64_t> planes;
        std::vector<uint8_t> pchars;
        for (uint32_t r = 0; r < n_rec; ++r) {
            const uint64_t a1 = p1_off[r], b1 = p1_off[r + 1];
            const uint64_t a2 = p2_off[r], b2 = p2_off[r + 1];
            if (b1 < a1 || b2 < a2 || b1 - a1 > 65535 || b2 - a2 > 65535) {
                rc = fail(MP_E_ARG, "primer length out of range (max 65535)");
                break;
            }
            DevRec& d = recs[r];
            d.l1 = (uint32_t)(b1 - a1);
            d.l2 = (uint32_t)(b2 - a2);
            d.hash_off = hash_off[r];
            if ((uint64_t)d.hash_off + W > d.l1) { rc = fail(MP_E_ARG, "hash offset outside primer1"); break; }
            d.size = (uint32_t)std::min<uint64_t>(pcr_size[r], 0xFFFFFFFFull);
            if ((uint64_t)d.l1 + d.l2 > pcr_size[r]) {
                rc = fail(MP_E_ARG, "pcr size below primer length sum");
                break;
            }
            t->max_hash_off = std::max(t->max_hash_off, d.hash_off);
            t->max_reach = std::max<uint64_t>(t->max_reach, (uint64_t)d.size + (uint64_t)p.margin);
            d.p1_pl = (uint32_t)(planes.size() / 4);
            build_planes(primer1 + a1, d.l1, p.iupac_mode, planes);
            d.p2_pl = (uint32_t)(planes.size() / 4);
            build_planes(primer2 + a2, d.l2, p.iupac_mode, planes);
            d.p1_ch = (uint32_t)pchars.size();
            for (uint64_t i = a1; i < b1; ++i) pchars.push_back(upcase(primer1[i]));
            d.p2_ch = (uint32_t)pchars.size();
            for (uint64_t i = a2; i < b2; ++i) pchars.push_back(upcase(primer2[i]));
            if (planes.size() / 4 > 0xFFFFFFF0ull || pchars.size() > 0xFFFFFFF0ull) {
                rc = fail(MP_E_ARG, "primer set too large");
                break;
            }
        }
        if (rc) break;
        // ---- bucket-ordered entries with primer-1 fingerprints
        std::vector<Entry> ents(n_rec);
        for (uint32_t i = 0; i < n_rec; ++i) {
            const uint32_t r = blist[i];
            Entry& e = ents[i];
            std::memset(&e, 0, sizeof(e));
            e.rec = rec_map ? rec_map[r] : r;
            e.hash_off = (uint16_t)recs[r].hash_off;
            e.l1 = (uint16_t)recs[r].l1;
            const uint64_t* pl = &planes[(size_t)recs[r].p1_pl * 4];
            const uint32_t lim = std::min<uint32_t>(recs[r].l1, 32);
            for (uint32_t q = 0; q < lim; ++q) {
                const int bit = 62 - 2 * (int)q;
                int nacc = 0, base = 0;
                for (int b = 0; b < 4; ++b)
                    if ((pl[b] >> bit) & 1) { ++nacc; base = b; }
                if (nacc == 1) {
                    e.code |= (uint64_t)base << bit;
                    e.pmask |= 1ull << bit;
                } else if (nacc == 0) {
                    e.pmask |= 1ull << (bit + 1);
                }
            }
        }
        for (uint32_t b = 0; b < nb; ++b) {  // bucket heads carry the bucket's size
            ents[boff[b]].count = bcount[b];
            ents[boff[b]].xstart = boff[b] + 1;
            for (uint32_t j = 1; j < bcount[b]; ++j) ents[boff[b] + j].count = bcount[b] - 1;  // tail length
        }
        // 8-B form of an entry: rec, l1 - W and primer-1 bases W..W+15, for plain
        // single-chunk primers seeded at their first base; others are flagged full
        auto entry8 = [&](const Entry& e) {
            const uint64_t plain_all = e.l1 >= 32 ? 0x5555555555555555ull
                                                  : (e.l1 ? (0x5555555555555555ull & (~0ull << (64 - 2 * e.l1))) : 0ull);
            const bool fast = !gapped && e.hash_off == 0 && e.l1 >= W && e.l1 - W <= 16 && e.pmask == plain_all &&
                              e.rec < (1u << kHead8RecBits);
            uint2 c;
            c.x = fast ? (uint32_t)((e.code << (2 * W)) >> 32) : 0u;  // bases W..W+15
            c.y = fast ? (e.rec | ((uint32_t)(e.l1 - W) << kHead8RecBits)) : kHead8Full;
            return c;
        };
        // kHead8Filt bits of a full head (0 when some record does not qualify)
        auto head8_filter = [&](uint32_t b) -> uint32_t {
            const uint32_t cnt = bcount[b];
            if (gapped || cnt < 1 || cnt > 3) return 0u;
            const uint32_t F = head8_filt_bases(cnt);
            const uint64_t fmask = 0x5555555555555555ull & ~(~0ull >> (2 * F));  // bases 0..F-1, spaced
            uint32_t bits = kHead8Filt | ((cnt - 1u) << 28);
            for (uint32_t j = 0; j < cnt; ++j) {
                const Entry& e = ents[boff[b] + j];
                if (e.hash_off != 0 || e.l1 < W + F || W + F > 32) return 0u;
                const uint64_t pm = e.pmask << (2 * W);
                if ((pm & fmask) != fmask || ((pm >> 1) & fmask) != 0) return 0u;  // plain, never "never"
                bits |= (uint32_t)((e.code << (2 * W)) >> (64 - 2 * F)) << (2 * F * j);
            }
            return bits;
        };
        std::vector<uint2> rk;
        std::vector<Entry> dents;
        std::vector<uint2> binfo;
        std::vector<uint16_t> dfilt;
        std::vector<Entry> dents_pad;
        std::vector<uint2> dgrp;
        std::vector<uint32_t> dgesc;
        std::vector<uint16_t> dsum;
        std::vector<uint2> dents8;
        std::vector<uint4> dents16;
        std::vector<uint64_t> kgrp;
        std::vector<uint4> kgrp4;
        std::vector<Slot> slots;
        if (t->filt_direct) {
            // rank bitmap over the exact 4^W presence bitmap; heads in key order
            rk.resize(filt.size());
            uint32_t acc = 0;
            for (size_t w = 0; w < filt.size(); ++w) {
                rk[w].x = filt[w];
                rk[w].y = acc;
                acc += (uint32_t)__builtin_popcount(filt[w]);
            }
            dents.resize(std::max<uint32_t>(nb, 1));
            dents8.resize(std::max<uint32_t>(nb, 1));
            std::vector<uint32_t> qfirst;
            if (W <= kDenseMaxW) {
                // plain run after the seed of every record seeded at its primer start
                auto plain_run = [&](const Entry& e) -> uint32_t {
                    if (e.hash_off != 0 || e.l1 < W) return 0;
                    uint32_t r = 0;
                    while (W + r < std::min<uint32_t>(e.l1, 32) && r < kDenseMaxF &&
                           ((e.pmask >> (62 - 2 * (W + r))) & 3ull) == 1ull)
                        ++r;
                    return r;
                };
                // F: the longest filter that at least 95% of the records can carry
                std::vector<uint32_t> hist(kDenseMaxF + 1, 0);
                for (uint32_t i = 0; i < n_rec; ++i) ++hist[plain_run(ents[i])];
                uint32_t F = 0, atleast = 0;
                for (int f = (int)kDenseMaxF; f >= 1; --f) {
                    atleast += hist[f];
                    if ((uint64_t)atleast * 20 >= (uint64_t)n_rec * 19) { F = (uint32_t)f; break; }
                }
                t->dense_F = F;
                // mismatch mask of the bases, both 16-bit halves of a word pair
                const uint32_t m16 = F ? (0x5555u & ~(0xFFFFu >> (2 * F))) : 0u;
                t->dense_M = m16 | (m16 << 16);
                binfo.resize(std::max<uint32_t>(nb, 1), make_uint2(0, 0));
                qfirst.resize(nb);
                // padded layout in key order, group by group: buckets of up to kDenseOct
                // records take one oct (16 B of filter words), indexed inside the group by the
                // popcount of the group's inline keys below; longer buckets are stored after
                // every group and found through binfo (escape bit)
                const uint32_t nkeys = 1u << (2 * W);
                const uint32_t ngrp = std::max<uint32_t>(1, nkeys / 32);
                std::vector<uint32_t> by_key(nkeys, 0xFFFFFFFFu);
                for (uint32_t b = 0; b < nb; ++b) by_key[bkey[b]] = b;
                // inline: at most one oct of records, every one carrying the filter (the hot
                // loop then tests no flags); other buckets take the escape walk
                auto inline_ok = [&](uint32_t b) {
                    if (bcount[b] > kDenseOct || !F) return false;
                    for (uint32_t j = 0; j < bcount[b]; ++j)
                        if (plain_run(ents[boff[b] + j]) < F) return false;
                    return true;
                };
                dgrp.assign(ngrp, make_uint2(0, 0));
                dgesc.assign(ngrp, 0u);
                uint64_t np = 0;  // padded slots
                for (uint32_t g = 0; g < ngrp; ++g) {
                    if (np / kDenseOct >= 0x7FFFFFFFull) { rc = fail(MP_E_ARG, "seed table too large"); break; }
                    dgrp[g].y = (uint32_t)(np / kDenseOct);
                    for (uint32_t j = 0; j < 32 && g * 32 + j < nkeys; ++j) {
                        const uint32_t b = by_key[g * 32 + j];
                        if (b == 0xFFFFFFFFu) continue;
                        if (!inline_ok(b)) {
                            dgesc[g] |= 1u << j;
                            dgrp[g].y |= 0x80000000u;
                            continue;
                        }
                        dgrp[g].x |= 1u << j;
                        qfirst[b] = (uint32_t)np;
                        np += kDenseOct;
                    }
                }
                if (rc) break;
                for (uint32_t k = 0; k < nkeys; ++k) {
                    const uint32_t b = by_key[k];
                    if (b == 0xFFFFFFFFu || inline_ok(b)) continue;
                    qfirst[b] = (uint32_t)np;
                    np += (bcount[b] + kDenseOct - 1) / kDenseOct * kDenseOct;
                }
                if (np / kDenseOct >= 0xFFFFFFF0ull) { rc = fail(MP_E_ARG, "seed table too large"); break; }
                dfilt.assign(std::max<uint64_t>(np, kDenseOct), kDensePad);
                Entry zero{};
                dents_pad.assign(std::max<uint64_t>(np, kDenseOct), zero);
                for (uint32_t b = 0; b < nb; ++b) {
                    for (uint32_t j = 0; j < bcount[b]; ++j) {
                        const Entry& e = ents[boff[b] + j];
                        const uint32_t q = qfirst[b] + j;
                        dents_pad[q] = e;
                        dfilt[q] = (F && plain_run(e) >= F)
                                       ? (uint16_t)(((e.code << (2 * W)) >> 48) & ~(0xFFFFu >> (2 * F)))
                                       : (uint16_t)kDenseAlways;
                    }
                    // inline oct: the spare slots repeat slot 0's bases (so they pass exactly
                    // when it does) with the pad bit set; their Entry has l1 = 0 (skipped)
                    if (inline_ok(b))
                        for (uint32_t j = bcount[b]; j < kDenseOct; ++j)
                            dfilt[qfirst[b] + j] = (uint16_t)(dfilt[qfirst[b]] | kDensePad);
                }
                // per-key summary of the inline buckets' filter bases
                if (W <= kDenseSumMaxW && p.mismatches <= 1 && F >= (p.mismatches ? 2u : 1u)) {
                    t->dsum_mode = p.mismatches ? 2 : 1;
                    const uint32_t FB = F / 2, fbm = (1u << (2 * FB)) - 1u;
                    dsum.assign(nkeys, 0);
                    for (uint32_t k = 0; k < nkeys; ++k) {
                        const uint32_t b = by_key[k];
                        if (b == 0xFFFFFFFFu) continue;
                        if (!inline_ok(b)) { dsum[k] = 0xFFFFu; continue; }
                        uint32_t sm = 0;
                        for (uint32_t j = 0; j < bcount[b]; ++j) {
                            const uint32_t gf = (uint32_t)dfilt[qfirst[b] + j] >> (16 - 2 * F);  // F bases
                            if (p.mismatches == 0) sm |= 1u << dsum_hash4(gf);
                            else sm |= (1u << dsum_hash3(gf >> (2 * FB))) | (1u << (8 + dsum_hash3(gf & fbm)));
                        }
                        dsum[k] = (uint16_t)sm;
                    }
                }
            }
            // 16-B form of a single-record head seeded at its primer start, plain over the
            // seed, at most W + 16 bases: bases W..W+15 with their plain / never bits (an IUPAC
            // base under I=1 is neither); {0, 0, 0, kHead8Full} when the record does not fit
            auto entry16 = [&](const Entry& e) {
                const uint64_t seed = sp_lt((int)W);
                const bool fits = !gapped && e.count == 1 && e.hash_off == 0 && e.l1 >= W && e.l1 - W <= 16 &&
                                  e.rec < (1u << kHead8RecBits) && (e.pmask & seed) == seed &&
                                  ((e.pmask >> 1) & seed) == 0;
                if (!fits) return make_uint4(0u, 0u, 0u, kHead8Full);
                return make_uint4((uint32_t)((e.code << (2 * W)) >> 32),
                                  (uint32_t)(((e.pmask & kEven) << (2 * W)) >> 32),
                                  (uint32_t)((((e.pmask >> 1) & kEven) << (2 * W)) >> 32),
                                  e.rec | ((uint32_t)(e.l1 - W) << kHead8RecBits));
            };
            // 8-B IUPAC form (kHead12RecBits): bases W..W+11, their plain bits, l1 - W
            auto entry12 = [&](const Entry& e) {
                const uint64_t seed = sp_lt((int)W);
                const int cov = (int)std::min<uint32_t>(e.l1 > W ? e.l1 - W : 0u, kHead12Bases);
                const uint64_t covm = sp_lt((int)W + cov) & ~seed;  // the covered primer bases
                const bool fits = !gapped && e.count == 1 && e.hash_off == 0 && e.l1 >= W && e.l1 - W <= 31 &&
                                  e.rec < (1u << kHead12RecBits) && (e.pmask & seed) == seed &&
                                  ((e.pmask >> 1) & seed) == 0 && ((e.pmask >> 1) & covm) == 0;
                if (!fits) return make_uint2(0u, kHead8Full);
                uint32_t plain = 0;
                for (uint32_t j = 0; j < kHead12Bases; ++j)
                    if ((e.pmask >> (62 - 2 * (W + j))) & 1ull) plain |= 1u << (kHead12Bases - 1 - j);
                return make_uint2((uint32_t)(((e.code << (2 * W)) >> 40) << 8) | (uint32_t)(e.l1 - W),
                                  e.rec | (plain << kHead12RecBits));
            };
            uint64_t n_full8 = 0, n_full16 = 0, n_full12 = 0;
            for (uint32_t b = 0; b < nb; ++b) {
                const Entry& e = ents[boff[b]];
                n_full8 += (e.count != 1 || (entry8(e).y & kHead8Full)) ? 1u : 0u;
                n_full16 += (entry16(e).w & kHead8Full) ? 1u : 0u;
                n_full12 += (entry12(e).y & kHead8Full) ? 1u : 0u;
            }
            // 16-B heads when they make the deferring drain possible (full heads under 5%) and
            // the 8-B heads do not (c4: 10% IUPAC primer bases); held in the 8-B IUPAC form when
            // that keeps full heads under 5% too (mp_table_options.no_h12: the 16-B form, A/B)
            t->h16 = W >= 10 && n_full16 * 20 < (uint64_t)nb && n_full8 * 20 >= (uint64_t)nb;
            t->h12 = t->h16 && n_full12 * 20 < (uint64_t)nb;
            if (topt.no_h12) t->h12 = 0;
            if (t->h16 && !t->h12) dents16.resize(std::max<uint32_t>(nb, 1));
            std::vector<uint2> dents12;
            if (t->h12) dents12.resize(std::max<uint32_t>(nb, 1));
            uint64_t n_full = 0;
            std::vector<uint32_t> rank_bucket(std::max<uint32_t>(nb, 1));
            for (uint32_t b = 0; b < nb; ++b) {
                const uint32_t k = bkey[b];
                const uint32_t rank = rk[k >> 5].y + (uint32_t)__builtin_popcount(rk[k >> 5].x & ((1u << (k & 31)) - 1u));
                const Entry& e = ents[boff[b]];
                rank_bucket[rank] = b;
                dents[rank] = e;
                // a full head names its bucket's first entry: the ranked drain can hand the whole
                // bucket to tail_kernel without reading the 32-B head
                dents8[rank] = e.count == 1 ? entry8(e) : make_uint2(boff[b], kHead8Full);
                if (dents8[rank].y & kHead8Full) {
                    dents8[rank].x = boff[b];
                    dents8[rank].y = kHead8Full | head8_filter(b);
                    if (!t->h16) ++n_full;
                }
                if (t->h12) {
                    dents12[rank] = entry12(e);
                    if (dents12[rank].y & kHead8Full) {
                        dents12[rank] = make_uint2(boff[b], kHead8Full | head8_filter(b));
                        ++n_full;
                    }
                } else if (t->h16) {
                    dents16[rank] = entry16(e);
                    if (dents16[rank].w & kHead8Full) {
                        dents16[rank] = make_uint4(boff[b], 0u, 0u, kHead8Full | head8_filter(b));
                        ++n_full;
                    }
                }
                if (W <= kDenseMaxW) binfo[rank] = make_uint2(qfirst[b], bcount[b]);
            }
            // few full heads (multi-record buckets, IUPAC/long/inner-seed primers): the ranked
            // drain tests only compact heads and defers every full-head bucket to tail_kernel
            // (a gapped table's heads are all full: its scan sends every seed that passes the key
            // groups to tail_kernel, the deferring form, whatever the share)
            t->defer_full = gapped || n_full * 20 < (uint64_t)nb;
            // key groups (kKgrpKeys keys per u64) for the scan's level-2 probe: it shuffles
            // bases [i, i + 17) of window i from the owning lane (i < 32 of its 48), so
            // F <= 17 - W, and a field holds <= 7 bases
            if (gapped && W >= 11 && W <= 13) {
                // gapped seed: a field per single-record key holding the record's gap bases
                // [gap_at, gap_at + gap_len) and then the gap_post bases after the seed's span
                // (bases [gap_at + 2 gap_len, + gap_post)); the gapped scan keeps a window only
                // when its gap differs in 1..N positions (or holds an invalid base: no mismatch
                // there, the contiguous seed finds the window) and gap + post differ in <= N
                const uint32_t F = gap_len + gap_post;
                const uint32_t post_at = gap_at + 2 * gap_len;
                t->kgrp_F = F;
                const uint64_t nkeys = 1ull << (2 * W);
                kgrp.assign(nkeys / kKgrpKeys, 0ull);
                const uint64_t gm = (sp_lt((int)(gap_at + gap_len)) & ~sp_lt((int)gap_at)) |
                                    (sp_lt((int)(post_at + gap_post)) & ~sp_lt((int)post_at));  // plain bits needed
                for (uint64_t g = 0; g < kgrp.size(); ++g) {
                    const uint32_t pres = (uint32_t)((filt[g >> 1] >> ((g & 1) * 16)) & 0xFFFFu);
                    uint64_t w = pres;
                    uint32_t j = 0;
                    for (uint32_t bit = 0; bit < 16 && j < kKgrpFields; ++bit) {
                        if (!((pres >> bit) & 1u)) continue;
                        const uint32_t k = (uint32_t)(g * kKgrpKeys + bit);
                        const uint32_t b = rank_bucket[rk[k >> 5].y + (uint32_t)__builtin_popcount(rk[k >> 5].x & ((1u << (k & 31)) - 1u))];
                        const Entry& e = ents[boff[b]];
                        if (bcount[b] == 1 && e.hash_off == 0 && e.l1 >= post_at + gap_post && (e.pmask & gm) == gm &&
                            ((e.pmask >> 1) & gm) == 0) {
                            const uint32_t gb = (uint32_t)((e.code << (2 * gap_at)) >> (64 - 2 * gap_len));
                            const uint32_t pb = gap_post ? (uint32_t)((e.code << (2 * post_at)) >> (64 - 2 * gap_post)) : 0u;
                            w |= (uint64_t)(kKgrpFlag | (gb << (2 * gap_post)) | pb) << (16u + 16u * j);
                        } else if (bcount[b] == 2 && gap_len <= 3) {  // kKgrpPair: each record's gap bases
                            const uint64_t am = sp_lt((int)(gap_at + gap_len)) & ~sp_lt((int)gap_at);
                            uint32_t f = kKgrpPair;
                            bool ok = true;
                            for (uint32_t r = 0; r < 2; ++r) {
                                const Entry& er = ents[boff[b] + r];
                                ok = ok && er.hash_off == 0 && (er.pmask & am) == am && ((er.pmask >> 1) & am) == 0;
                                f |= (uint32_t)((er.code << (2 * gap_at)) >> (64 - 2 * gap_len)) << (6 * (1 - r));
                            }
                            if (ok) w |= (uint64_t)f << (16u + 16u * j);
                        }
                        ++j;
                    }
                    kgrp[g] = w;
                }
            } else if (W >= 11 && W <= 13 && p.iupac_mode) {
                // I = 1 (c4: degenerate primers): two 24-bit fields per group, one per present
                // key, each the 2-bit codes of primer-1 bases W..W+F-1 (12 bits) and, at the
                // even bit positions of the next 12, the bases that are not plain (an IUPAC
                // base: any genome base may match it) -- skipped by the mismatch count.  A key
                // with no field (a bucket of several records, a seed inside the primer, a
                // primer shorter than W + F, or the third present key of the group) has every
                // base marked: it always passes.
                const uint32_t F = std::min<uint32_t>(6u, 17u - W);
                t->kgrp_F = F;
                const uint32_t m2 = (1u << (2 * F)) - 1u;
                // expected pass rate of a random window's field test: P(<= N mismatches over
                // the field's plain bases, each a mismatch with p = 3/4); absent fields pass
                auto pass_rate = [&](uint32_t plain_bases) {
                    double pr = 0.0, c = 1.0;
                    for (uint32_t k = 0; k <= plain_bases && k <= (uint32_t)p.mismatches; ++k) {
                        if (k) c = c * (double)(plain_bases - k + 1) / (double)k;
                        pr += c * std::pow(0.75, (double)k) * std::pow(0.25, (double)(plain_bases - k));
                    }
                    return pr;
                };
                double pass_sum = 0.0;
                uint64_t pass_n = 0;
                const uint64_t nkeys = 1ull << (2 * W);
                kgrp.assign(nkeys / kKgrpKeys, 0ull);
                for (uint64_t g = 0; g < kgrp.size(); ++g) {
                    const uint32_t pres = (uint32_t)((filt[g >> 1] >> ((g & 1) * 16)) & 0xFFFFu);
                    uint64_t w = pres;
                    uint32_t j = 0;
                    for (uint32_t bit = 0; bit < 16 && j < kKgrpWildFields; ++bit) {
                        if (!((pres >> bit) & 1u)) continue;
                        const uint32_t k = (uint32_t)(g * kKgrpKeys + bit);
                        const uint32_t rank = rk[k >> 5].y + (uint32_t)__builtin_popcount(rk[k >> 5].x & ((1u << (k & 31)) - 1u));
                        const uint32_t b = rank_bucket[rank];
                        const Entry& e = ents[boff[b]];
                        uint32_t field = (m2 & 0x555u) << 12;  // every base wild: always passes
                        double pr = 1.0;
                        if (bcount[b] == 1 && e.hash_off == 0 && e.l1 >= W + F) {
                            const uint32_t codes = (uint32_t)((e.code << (2 * W)) >> (64 - 2 * F));
                            const uint32_t plain = (uint32_t)(((e.pmask & kEven) << (2 * W)) >> (64 - 2 * F));
                            field = codes | ((~plain & m2 & 0x555u) << 12);
                            pr = pass_rate((uint32_t)__builtin_popcount(plain & m2 & 0x555u));
                        }
                        pass_sum += pr;
                        ++pass_n;
                        w |= (uint64_t)field << (16u + 24u * j);
                        ++j;
                    }
                    for (; j < kKgrpWildFields; ++j) w |= (uint64_t)((m2 & 0x555u) << 12) << (16u + 24u * j);
                    kgrp[g] = w;
                }
                // the scan takes the key groups only when they reject most seeds (c3's fields
                // pass ~0.5%); c4's (N = 2, ~30% IUPAC bases after the seed) pass ~30% and stay
                // on the 16-B heads, which test 16 bases
                t->kgrp_wild = pass_n && pass_sum / (double)pass_n < 0.08 ? 1 : 0;
                // wide key groups (kKgrp4Keys) when the 8-B fields are too short to end most
                // seeds and the heads are in the 8-B IUPAC form (h12): ten bases per field; a
                // key without one (several records, a seed inside the primer, the fourth
                // present key of its group) always passes.  Taken when fewer than a quarter of
                // a random window's seeds would pass (c4: ~0.12 with the keys without a field
                // counted, against ~0.30 for the 8-B fields)
                // mp_table_options.kgrp4 (A/B runs and tests): 1 = never, -1 = whenever the
                // table can carry them (the pass-rate estimate skipped)
                const int no4v = topt.kgrp4;
                if (!t->kgrp_wild && t->h12 && t->defer_full && no4v <= 0) {
                    const uint32_t F4 = kKgrp4F;
                    const uint64_t seedm = sp_lt((int)W);
                    double pass4 = 0.0;
                    uint64_t n4 = 0;
                    kgrp4.assign(nkeys / kKgrp4Keys, make_uint4(0u, 0u, 0u, 0u));
                    for (uint64_t g = 0; g < kgrp4.size(); ++g) {
                        // this group's keys: a word of the exact bitmap, or half of one
                        const uint64_t g0 = g * kKgrp4Keys;
                        const uint32_t pres = kKgrp4Keys == 32 ? filt[g] : (filt[g0 >> 5] >> (g0 & 31)) & 0xFFFFu;
                        uint32_t fields[kKgrp4Fields] = {0u, 0u, 0u};
                        uint32_t j = 0;
                        for (uint32_t bit = 0; bit < kKgrp4Keys; ++bit) {
                            if (!((pres >> bit) & 1u)) continue;
                            ++n4;
                            if (j >= kKgrp4Fields) {
                                pass4 += 1.0;
                                continue;
                            }
                            const uint32_t k = (uint32_t)(g0 + bit);
                            const uint32_t rank = rk[k >> 5].y + (uint32_t)__builtin_popcount(rk[k >> 5].x & ((1u << (k & 31)) - 1u));
                            const uint32_t b = rank_bucket[rank];
                            const Entry& e = ents[boff[b]];
                            uint32_t f = 0;
                            double pr = 1.0;
                            if (bcount[b] == 1 && e.hash_off == 0 && e.l1 > W && (e.pmask & seedm) == seedm &&
                                ((e.pmask >> 1) & seedm) == 0) {
                                uint32_t plain = 0;
                                for (uint32_t i = 0; i < F4 && W + i < e.l1 && W + i < 32; ++i)
                                    if ((e.pmask >> (62 - 2 * (W + i))) & 1ull) plain |= 1u << (F4 - 1 - i);
                                f = (plain << (2 * F4)) | (uint32_t)((e.code << (2 * W)) >> (64 - 2 * F4));
                                pr = pass_rate((uint32_t)__builtin_popcount(plain));
                            }
                            fields[j] = f;
                            pass4 += pr;
                            ++j;
                        }
                        kgrp4[g] = make_uint4(pres, fields[0], fields[1], fields[2]);
                    }
                    if (!(n4 && (no4v < 0 || pass4 / (double)n4 < 0.25))) kgrp4.clear();
                }
            } else if (W >= 11 && W <= 13) {
                const uint32_t F = std::min<uint32_t>(7u, 17u - W);
                t->kgrp_F = F;
                const uint64_t nkeys = 1ull << (2 * W);
                kgrp.assign(nkeys / kKgrpKeys, 0ull);
                for (uint64_t g = 0; g < kgrp.size(); ++g) {
                    const uint32_t pres = (uint32_t)((filt[g >> 1] >> ((g & 1) * 16)) & 0xFFFFu);
                    uint64_t w = pres;
                    uint32_t j = 0;
                    for (uint32_t bit = 0; bit < 16 && j < kKgrpFields; ++bit) {
                        if (!((pres >> bit) & 1u)) continue;
                        const uint32_t k = (uint32_t)(g * kKgrpKeys + bit);
                        const uint32_t rank = rk[k >> 5].y + (uint32_t)__builtin_popcount(rk[k >> 5].x & ((1u << (k & 31)) - 1u));
                        const uint2 h = dents8[rank];
                        // compact head (single record, seeded at its primer start, plain, <= W + 16
                        // bases) carrying at least F bases after the seed
                        if (!(h.y & kHead8Full) && ((h.y >> kHead8RecBits) & 31u) >= F) {
                            w |= (uint64_t)(kKgrpFlag | (h.x >> (32u - 2u * F))) << (16u + 16u * j);
                        } else if (F >= 3 && bcount[rank_bucket[rank]] == 2) {  // kKgrpPair
                            const uint32_t b = rank_bucket[rank];
                            const uint64_t m3 = sp_lt((int)W + 3) & ~sp_lt((int)W);
                            uint32_t f = kKgrpPair;
                            bool ok = true;
                            for (uint32_t r = 0; r < 2; ++r) {
                                const Entry& e = ents[boff[b] + r];
                                ok = ok && e.hash_off == 0 && e.l1 >= W + 3 && (e.pmask & m3) == m3 && ((e.pmask >> 1) & m3) == 0;
                                f |= (uint32_t)((e.code << (2 * W)) >> 58) << (6 * (1 - r));
                            }
                            if (ok) w |= (uint64_t)f << (16u + 16u * j);
                        }
                        ++j;
                    }
                    kgrp[g] = w;
                }
            }
            filt.assign(1, 0);
            if ((rc = upload(&t->dents12, dents12.data(), dents12.size(), &dev_bytes_pre))) break;
        } else {
            uint32_t lg = 6;
            while ((1ull << lg) < 2ull * nb) ++lg;
            t->slot_log2 = lg;
            slots.resize(1ull << lg);
            std::memset(slots.data(), 0, slots.size() * sizeof(Slot));
            for (uint32_t b = 0; b < nb; ++b) {
                uint32_t s = table_slot(bkey[b], lg);
                while (slots[s].used) s = (s + 1) & ((1u << lg) - 1);
                slots[s].key = bkey[b];
                slots[s].used = 1;
                slots[s].e0 = ents[boff[b]];
            }
        }
        // Ties at equal amplicon start are ordered by (hash_offset, record index):
        // rank[] encodes that order in 32 bits for the device sort.
        std::vector<uint32_t> order(n_rec), rank(n_rec);
        for (uint32_t r = 0; r < n_rec; ++r) order[r] = r;
        std::stable_sort(order.begin(), order.end(),
                         [&](uint32_t a, uint32_t b) { return recs[a].hash_off < recs[b].hash_off; });
        for (uint32_t i = 0; i < n_rec; ++i) rank[order[i]] = i;
        t->rank_bits = 1;
        while ((1ull << t->rank_bits) < (uint64_t)n_rec) ++t->rank_bits;

        uint64_t bytes = 0;
        t->layout = (t->lds_exact ? MP_LAYOUT_LDS_EXACT : 0u) | (rk.empty() ? 0u : MP_LAYOUT_RANK) |
                    (kgrp.empty() ? 0u : MP_LAYOUT_KGRP) | (kgrp4.empty() ? 0u : MP_LAYOUT_KGRP4) |
                    (dgrp.empty() ? 0u : MP_LAYOUT_DENSE) | (slots.empty() ? 0u : MP_LAYOUT_HASHED) |
                    (t->defer_full ? MP_LAYOUT_DEFER_FULL : 0u);
        if ((rc = upload(&t->filt, filt.data(), filt.size(), &bytes))) break;
        if ((rc = upload(&t->lfilt, lfilt.data(), lfilt.size(), &bytes))) break;
        if ((rc = upload(&t->slots, slots.data(), slots.size(), &bytes))) break;
        if ((rc = upload(&t->rk, rk.data(), rk.size(), &bytes))) break;
        if ((rc = upload(&t->dents, dents.data(), dents.size(), &bytes))) break;
        if ((rc = upload(&t->dents8, dents8.data(), dents8.size(), &bytes))) break;
        if ((rc = upload(&t->dents16, dents16.data(), dents16.size(), &bytes))) break;
        if ((rc = upload(&t->kgrp, kgrp.data(), kgrp.size(), &bytes))) break;
        if (!kgrp4.empty() && (rc = upload(&t->kgrp4, kgrp4.data(), kgrp4.size(), &bytes))) break;
        if ((rc = upload(&t->binfo, binfo.data(), binfo.size(), &bytes))) break;
        if ((rc = upload(&t->dfilt, dfilt.data(), dfilt.size(), &bytes))) break;
        if ((rc = upload(&t->dgrp, dgrp.data(), dgrp.size(), &bytes))) break;
        if ((rc = upload(&t->dgesc, dgesc.data(), dgesc.size(), &bytes))) break;
        if ((rc = upload(&t->dsum, dsum.data(), dsum.size(), &bytes))) break;
        if ((rc = upload(&t->dents_pad, dents_pad.data(), dents_pad.size(), &bytes))) break;
        if ((rc = upload(&t->ents, ents.data(), ents.size(), &bytes))) break;
        if ((rc = upload(&t->recs, recs.data(), recs.size(), &bytes))) break;
        if ((rc = upload(&t->rank, rank.data(), rank.size(), &bytes))) break;
        if ((rc = upload(&t->inv_rank, order.data(), order.size(), &bytes))) break;
        {
            std::vector<uint2> rr(n_rec);
            for (uint32_t i = 0; i < n_rec; ++i) rr[i] = make_uint2(order[i], recs[order[i]].size);
            if ((rc = upload(&t->rank_rec, rr.data(), rr.size(), &bytes))) break;
        }
        planes.push_back(0); planes.push_back(0); planes.push_back(0); planes.push_back(0);
        {
            std::vector<PairRec> prec(n_rec);
            for (uint32_t r = 0; r < n_rec; ++r) {
                PairRec& q = prec[r];
                std::memset(&q, 0, sizeof(q));
                q.d = recs[r];
                q.rank = rank[r];
                for (int k = 0; k < 4; ++k) {
                    q.p1q[k] = planes[(uint64_t)recs[r].p1_pl * 4 + k];
                    q.p2q[k] = planes[(uint64_t)recs[r].p2_pl * 4 + k];
                }
            }
            if ((rc = upload(&t->prec, prec.data(), prec.size(), &bytes))) break;
        }
        if ((rc = upload(&t->planes, planes.data(), planes.size(), &bytes))) break;
        t->planes_words = planes.size();
        pchars.resize(pchars.size() + 40, 0);  // chunk_ok reads 36 bytes from a 4-aligned offset
        if ((rc = upload(&t->pchars, pchars.data(), pchars.size(), &bytes))) break;
        t->dev_bytes = bytes + dev_bytes_pre;
    } while (0);
    if (rc) {
        free_table(t);
        return rc;
    }
    *table_out = t;
    return MP_OK;
}

// Split seeds (kSplitSeed): the sub-tables of a W 7..9, I = 0, N <= 1 table.  A record takes
// the seeds when it is seeded at its primer start and its primer 1 is plain over the bases
// the seeds, the pigeonhole cut and the gapped key groups need (N = 1: [0, S + post), S =
// split_span(W); N = 0: [0, kSplitSeed)); the rest stay in a dense table of their own.  Not
// split when under half the records qualify.
static int build_split(Table* t, uint32_t n_rec, const uint32_t* key, const uint32_t* hash_off,
                       const uint64_t* pcr_size, const uint8_t* primer1, const uint64_t* p1_off,
                       const uint8_t* primer2, const uint64_t* p2_off) {
    const mp_params& p = t->prm;
    const uint32_t W = (uint32_t)p.wordsize;
    if (W < 7 || W > 9 || p.iupac_mode != 0 || p.mismatches > 1 || n_rec == 0) return MP_OK;
    if (t->topt.no_split) return MP_OK;
    const uint32_t S = split_span(W), A = kSplitSeed - W;  // span of the cut stretch, bases of A (= of B)
    const uint32_t need = p.mismatches ? S + split_post(W) : kSplitSeed;
    auto code = [](uint8_t c) -> int {
        switch (upcase(c)) { case 'A': return 0; case 'C': return 1; case 'G': return 2; case 'T': return 3; default: return -1; }
    };
    std::vector<uint32_t> yes, rest;
    for (uint32_t r = 0; r < n_rec; ++r) {
        bool ok = hash_off[r] == 0 && p1_off[r + 1] - p1_off[r] >= need;
        for (uint32_t i = 0; ok && i < need; ++i) ok = code(primer1[p1_off[r] + i]) >= 0;
        (ok ? yes : rest).push_back(r);
    }
    if (yes.size() * 2 < n_rec) return MP_OK;
    // one sub-table's record arrays: the chosen records, in parent order
    struct Sub {
        std::vector<uint32_t> key, hoff, map;
        std::vector<uint64_t> size, o1, o2;
        std::vector<uint8_t> b1, b2;
    };
    auto subset = [&](const std::vector<uint32_t>& recs, int form) {
        Sub s;
        s.o1.push_back(0);
        s.o2.push_back(0);
        for (uint32_t r : recs) {
            const uint8_t* q = primer1 + p1_off[r];
            uint32_t k = 0;
            if (form == 0) {  // A: [0, W + a)
                for (uint32_t i = 0; i < kSplitSeed; ++i) k = (k << 2) | (uint32_t)code(q[i]);
            } else if (form == 1) {  // B: [0, W) ++ [W + a, S)
                for (uint32_t i = 0; i < W; ++i) k = (k << 2) | (uint32_t)code(q[i]);
                for (uint32_t i = W + A; i < S; ++i) k = (k << 2) | (uint32_t)code(q[i]);
            } else {
                k = key[r];
            }
            s.key.push_back(k);
            s.hoff.push_back(form == 2 ? hash_off[r] : 0u);
            s.map.push_back(r);
            s.size.push_back(pcr_size[r]);
            s.b1.insert(s.b1.end(), primer1 + p1_off[r], primer1 + p1_off[r + 1]);
            s.b2.insert(s.b2.end(), primer2 + p2_off[r], primer2 + p2_off[r + 1]);
            s.o1.push_back(s.b1.size());
            s.o2.push_back(s.b2.size());
        }
        return s;
    };
    auto make = [&](const Sub& s, uint32_t w, uint32_t gap_at, uint32_t gap_len, uint32_t gap_post, Table** out) {
        mp_params q = p;
        q.wordsize = (int32_t)w;
        return build_table(q, t->device, (uint32_t)s.key.size(), s.key.data(), s.hoff.data(), s.size.data(),
                           s.b1.data(), s.o1.data(), s.b2.data(), s.o2.data(), s.map.data(), gap_at, gap_len,
                           gap_post, t->topt, out);
    };
    int rc = MP_OK;
    {
        const Sub a = subset(yes, 0);
        rc = make(a, kSplitSeed, 0, 0, 0, &t->split_a);
    }
    if (!rc && p.mismatches) {
        const Sub b = subset(yes, 1);
        rc = make(b, kSplitSeed, W, A, split_post(W), &t->split_b);
    }
    if (!rc && !rest.empty()) {
        const Sub r = subset(rest, 2);
        rc = make(r, W, 0, 0, 0, &t->split_rest);
    }
    if (rc) {
        free_table(t->split_a); free_table(t->split_b); free_table(t->split_rest);
        t->split_a = t->split_b = t->split_rest = nullptr;
    }
    return rc;
}

MP_EXPORT int mp_table_create(const mp_params* prm, int32_t device, uint32_t n_rec,
                              const uint32_t* key, const uint32_t* hash_off,
                              const uint64_t* pcr_size, const uint8_t* primer1,
                              const uint64_t* p1_off, const uint8_t* primer2,
                              const uint64_t* p2_off, void** table_out) {
    return mp_table_create_ex(prm, device, n_rec, key, hash_off, pcr_size, primer1, p1_off, primer2, p2_off, nullptr,
                              table_out);
}

MP_EXPORT int mp_table_create_ex(const mp_params* prm, int32_t device, uint32_t n_rec,
                                 const uint32_t* key, const uint32_t* hash_off,
                                 const uint64_t* pcr_size, const uint8_t* primer1,
                                 const uint64_t* p1_off, const uint8_t* primer2,
                                 const uint64_t* p2_off, const mp_table_options* options, void** table_out) {
    if (!prm || !table_out) return fail(MP_E_ARG, "mp_table_create: null pointer");
    const mp_table_options topt = options ? *options : mp_table_options{};
    if (topt.lds_k < 0 || topt.lds_k > 3 || topt.kgrp4 < -1 || topt.kgrp4 > 1)
        return fail(MP_E_ARG, "mp_table_create_ex: option out of range");
    *table_out = nullptr;
    const mp_params& p = *prm;
    if (p.wordsize < 3 || p.wordsize > 16) return fail(MP_E_ARG, "Word size must be between 3 and 16");
    if (p.mismatches < 0 || p.mismatches > 10)
        return fail(MP_E_ARG, "Number of mismatches must be between 0 and 10");
    if (p.margin < 0 || p.margin > 10000) return fail(MP_E_ARG, "Margin must be between 0 and 10000");
    if (p.three_prime_match < 0) return fail(MP_E_ARG, "Three prime match must be at least 0");
    if (p.iupac_mode != 0 && p.iupac_mode != 1) return fail(MP_E_ARG, "iupac_mode must be 0 or 1");
    if (n_rec >= 0x80000000u) return fail(MP_E_ARG, "too many records (max 2^31 - 1)");
    if (n_rec && (!key || !hash_off || !pcr_size || !primer1 || !p1_off || !primer2 || !p2_off))
        return fail(MP_E_ARG, "mp_table_create: null record array");
    Table* t = nullptr;
    int rc = build_table(p, device, n_rec, key, hash_off, pcr_size, primer1, p1_off, primer2, p2_off, nullptr, 0, 0, 0,
                         topt, &t);
    if (rc) return rc;
    rc = build_split(t, n_rec, key, hash_off, pcr_size, primer1, p1_off, primer2, p2_off);
    if (rc) {
        free_table(t);
        return rc;
    }
    *table_out = t;
    return MP_OK;
}

MP_EXPORT int mp_table_stats(void* table, uint64_t* n_keys, uint64_t* max_bucket, uint64_t* dev_bytes) {
    Table* t = (Table*)table;
    if (!t) return fail(MP_E_ARG, "mp_table_stats: null table");
    if (n_keys) *n_keys = t->n_keys;
    if (max_bucket) *max_bucket = t->max_bucket;
    if (dev_bytes) *dev_bytes = t->dev_bytes;
    return MP_OK;
}

MP_EXPORT int mp_table_split(void* table, uint32_t* seed_tables, uint32_t* rest_records) {
    Table* t = (Table*)table;
    if (!t) return fail(MP_E_ARG, "mp_table_split: null table");
    if (seed_tables) *seed_tables = (t->split_a ? 1u : 0u) + (t->split_b ? 1u : 0u);
    if (rest_records) *rest_records = t->split_a ? (t->split_rest ? t->split_rest->n_rec : 0u) : t->n_rec;
    return MP_OK;
}

MP_EXPORT int mp_table_layout(void* table, uint32_t* flags) {
    Table* t = (Table*)table;
    if (!t || !flags) return fail(MP_E_ARG, "mp_table_layout: null pointer");
    *flags = t->layout | (t->split_a ? MP_LAYOUT_SPLIT : 0u);
    return MP_OK;
}

MP_EXPORT void mp_table_destroy(void* table) { free_table((Table*)table); }
