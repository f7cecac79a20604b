// Internal definitions shared by the libmerpcr_hip translation units.
//
// Data layout in HBM (DESIGN.md "Data layout"):
//   genome  g2   : 2 bits/base, big-endian inside each u64 (base j of a word at
//                  bits [63-2j, 62-2j]), A=0 C=1 G=2 T=U=3, other = 0
//           ginv : 1 bit/base, big-endian (bit 63-j), set where the base is not
//                  A/C/G/T/U: such a base makes every W-mer through it unseeded
//                  (engine.py:464-503)
//           gexc : 1 bit/base, set where the base is not exactly A/C/G/T: the
//                  primer compare must look the character up (engine.py:599-642)
//           gwild: 1 bit/base, set where the base is 'N' (either case): under I = 1 every
//                  IUPAC primer base matches it (engine.py:613-631), so the pair check
//                  treats it as a wildcard without looking the character up
//           xr_* : sorted run index of the exception characters (start, char)
//   Sequences are laid end to end, each padded to a multiple of 64 bases; the
//   padding is marked ginv = gexc = 1.  A "global" coordinate is the index in
//   that padded space.
//   table   lfilt: 64 KiB seed prefilter, staged in LDS by every workgroup (exact
//                  4^W bitmap for W <= 9, hashed above)
//           W <= 13: rk: {presence bits, prefix popcount} per 32 keys of the exact
//                  4^W bitmap; the rank of a present key indexes dents, one 32-B
//                  bucket-head Entry per distinct key
//           W >= 14: filt: hashed 2^27-bit presence filter, slots: open-addressed
//                  key -> 64-B Slot holding the bucket-head Entry
//           Entry: record id, seed offset and a primer-1 fingerprint (2-bit code +
//                  plain/never masks of its first 32 bases) that rejects almost
//                  every random seed hit; ents: all Entries in bucket order
//                  (records of one key in insertion order), read for bucket tails
//           recs : one 32-B DevRec per record (sts_records order), primer accept
//                  planes (4 x u64 per 32 primer bases) and raw primer bytes, read
//                  only for fingerprint survivors.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <vector>

#include "../../include/merpcr_hip.h"

#define MP_EXPORT extern "C" __attribute__((visibility("default")))

namespace mp {

// ---------------------------------------------------------------- errors
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define MP_HIP_CHECK(expr)                                                     \
    do {                                                                       \
        hipError_t _e = (expr);                                                \
        if (_e != hipSuccess)                                                  \
            return ::mp::fail(MP_E_HIP, std::string(#expr) + " (" + __FILE__ +   \
                                            ":" + std::to_string(__LINE__) +   \
                                            "): " + hipGetErrorString(_e));    \
    } while (0)

// Wait for an event by polling (hipEventQuery) instead of a blocking synchronisation: a
// tight spin for the first ~20 us (a search's counter readback is on every step's critical
// path), then the CPU is yielded between polls.  timeout_s > 0 bounds the wait: it returns
// hipErrorNotReady when the event has not completed by then (a peer rank that never joins
// a collective would otherwise hold this thread forever).
hipError_t poll_event(hipEvent_t ev, double timeout_s = 0.0);

// ---------------------------------------------------------------- constants
constexpr uint64_t kEven = 0x5555555555555555ull;  // the low bit of every 2-bit slot
constexpr int kHashedFilterLog2 = 27;               // 16 MiB hashed filter for W >= 14
constexpr int kDirectFilterMaxW = 13;               // 4^13 bits = 8 MiB direct bitmap
constexpr int kBlock = 1024;                        // threads per scan workgroup (one per CU)
constexpr int kWaves = kBlock / 64;
constexpr uint32_t kPutRing = 64;  // mp_search_put_hits: pinned count slots in flight per handle
constexpr int kLanePos = 32;                        // consecutive window positions per lane
constexpr uint32_t kSuper = 64 * kLanePos;          // positions per wave super-step
constexpr int kBlocksPerCU = 1;                     // persistent grid: resident workgroups per CU
constexpr int kDirShift = 12;                       // exception-run directory granularity
#ifndef MP_LDS_LOG2
#define MP_LDS_LOG2 20  // A/B builds only (the c5 single-pass question): 19 = 64 KiB
#endif
constexpr int kLdsFilterLog2 = MP_LDS_LOG2;         // 128 KiB seed prefilter staged in LDS
constexpr uint32_t kLdsFilterWords = (1u << kLdsFilterLog2) / 32;
constexpr int kSub = 8;                             // filter probes in flight per lane

struct DevRec {            // one oriented STS record, 32 bytes
    uint32_t hash_off;     // offset of the seed W-mer inside primer1
    uint32_t l1, l2;       // primer lengths
    uint32_t size;         // expected product size (clamped to u32)
    uint32_t p1_pl, p2_pl; // first 32-base chunk of each primer in the plane array
    uint32_t p1_ch, p2_ch; // byte offset of each primer in the raw primer array
};
static_assert(sizeof(DevRec) == 32, "DevRec layout");

// The pair check's view of one record in one 128-B line (round 4): its DevRec, its tie
// rank and the accept planes of both primers' first 32 bases.  Three random record-indexed
// loads per survivor (recs, rank, two plane chunks) become one line; on c4 (2.8M survivors)
// those loads missed L2 and the pair kernel fetched ~2 GB per launch.
struct alignas(128) PairRec {
    DevRec d;
    uint32_t rank, pad0;
    uint64_t p1q[4];       // planes of primer-1 bases [0, 32)
    uint64_t p2q[4];       // planes of primer-2 bases [0, 32)
    uint64_t pad1[3];
};
static_assert(sizeof(PairRec) == 128, "PairRec is one 128-B line");

struct Entry {             // one oriented record, 32 bytes
    uint64_t code;         // 2-bit code of primer-1 bases [0, 32) (big-endian slots)
    uint64_t pmask;        // even bits: base is a single A/C/G/T for the compare rule
                           // (plain); odd bits: no A/C/G/T matches it (never)
    uint32_t rec;          // index in sts_records
    uint16_t hash_off;     // seed offset inside primer 1
    uint16_t l1;           // primer-1 length
    uint32_t xstart;       // bucket head only: ents index of the bucket's 2nd record
    uint32_t count;        // bucket head only: records with this key
};
static_assert(sizeof(Entry) == 32, "Entry layout");

struct Slot {              // open-addressed seed-table slot (W >= 14), 64 bytes
    uint32_t key;
    uint32_t used;         // 0 = empty slot
    uint32_t pad0, pad1;
    Entry e0;              // the bucket head
    uint64_t pad2, pad3;
};
static_assert(sizeof(Slot) == 64, "Slot layout");

struct SeqSpan {           // per-sequence work description for one search run
    uint64_t super0;       // first global super-step of this sequence (sentinel: total)
    uint32_t seq;          // sequence index in the genome handle
    uint32_t p_lo, p_hi;   // window positions [p_lo, p_hi) scanned
    uint32_t p_al;         // p_lo rounded down to a multiple of kLanePos (super-step origin)
};

// ---------------------------------------------------------------- handles
struct Table {
    mp_params prm{};
    mp_table_options topt{};  // layout choices of the build (all zero = automatic)
    int device = 0;
    uint32_t n_rec = 0;
    uint64_t n_keys = 0, max_bucket = 0, dev_bytes = 0;
    uint32_t max_hash_off = 0;
    uint64_t max_reach = 0;   // max(size) + M: bases past an amplicon start any compare reads
    int filt_direct = 1;
    uint32_t filt_log2 = 0;   // log2(filter bits)
    int lds_exact = 0;        // LDS prefilter is the exact 4^W bitmap (W <= 10)
    uint32_t layout = 0;      // MP_LAYOUT_* bits of the structures built (empty arrays are 1-element stubs)
    int lds_k = 1;            // bits per key in the blocked LDS filter (W 11..13)
    int defer_full = 0;       // < 5% full heads: the ranked drain defers them to tail_kernel
    uint32_t* lfilt = nullptr;  // kLdsFilterWords words
    uint32_t slot_log2 = 0;
    uint32_t* filt = nullptr;     // W >= 14: hashed presence filter
    uint2* rk = nullptr;          // W <= 13: rank bitmap
    Entry* dents = nullptr;       // W <= 13: bucket heads by key rank
    uint2* dents8 = nullptr;      // W <= 13: 8-B heads {primer-1 bases W..W+15, rec | (l1-W)<<26 | full<<31}
    uint4* dents16 = nullptr;     // h16: 16-B heads {bases W..W+15, plain bits, never bits, as dents8.y}
    int h16 = 0;                  // many heads need plain/never masks (IUPAC primers): 16-B heads
    uint2* dents12 = nullptr;     // h12: the IUPAC heads in 8 B (kHead12RecBits), in place of dents16
    int h12 = 0;                  // h16 tables whose heads fit the 8-B IUPAC form (c4)
    uint64_t* kgrp = nullptr;     // W 11..13: key groups, one u64 per 16 keys (see kKgrpKeys)
    uint32_t kgrp_F = 0;          // primer-1 bases W..W+F-1 a key-group field holds (0: no key groups)
    int kgrp_wild = 0;            // I = 1 field form: two 24-bit fields with the non-plain bases marked
    uint4* kgrp4 = nullptr;       // I = 1, W 11..13: wide key groups, one uint4 per 32 keys (kKgrp4Keys)
    uint2* binfo = nullptr;       // W <= kDenseMaxW: per key rank {first padded entry, records}
    uint16_t* dfilt = nullptr;    // W <= kDenseMaxW: 2-B filter word per padded entry (kDenseAlways...)
    uint2* dgrp = nullptr;        // W <= kDenseMaxW: per 32 keys {inline-bucket bits, first oct | any escape << 31}
    uint32_t* dgesc = nullptr;    // W <= kDenseMaxW: per 32 keys, keys of more than kDenseOct records
    Entry* dents_pad = nullptr;   // W <= kDenseMaxW: ents with every bucket padded to a multiple of 4
    uint32_t dense_F = 0;         // bases after the seed the filter words hold
    uint32_t dense_M = 0;         // their mismatch mask in both halves of a 32-bit word pair
    uint16_t* dsum = nullptr;     // W <= kDenseSumMaxW, N <= 1: per-key summary (see kDenseSumMaxW)
    int dsum_mode = 0;            // 0: none, 1: N = 0 form, 2: N = 1 form
    Slot* slots = nullptr;        // W >= 14
    Entry* ents = nullptr;
    DevRec* recs = nullptr;
    uint32_t* rank = nullptr;      // rec -> position in (hash_off, rec) order
    uint32_t* inv_rank = nullptr;  // position -> rec
    uint2* rank_rec = nullptr;     // position -> {rec, its size}: the hit decode's one load
    uint64_t* planes = nullptr;    // 4 u64 per 32-base primer chunk
    PairRec* prec = nullptr;       // per record: DevRec, rank, both primers' first plane chunks
    uint64_t planes_words = 0;
    uint8_t* pchars = nullptr;
    uint32_t rank_bits = 1;
    // Split seeds (W 7..9, I = 0, N <= 1; see kSplitSeed): the dense table's search as scans of
    // longer exact seeds.  Sub-tables hold only the scan side; their Entry::rec are this
    // table's record indices, and the pair check, ranks and decode use this table's arrays.
    Table* split_a = nullptr;     // seed = primer-1 bases [0, kSplitSeed)
    Table* split_b = nullptr;     // N = 1: the gapped seed [0, W) ++ [kSplitSeed, split_span(W))
    Table* split_rest = nullptr;  // records neither seed can carry: dense_kernel on them alone
    // gapped table: key = bases [0, gap_at) ++ [gap_at + gap_len, gap_at + 2 gap_len); its key
    // groups hold the gap's bases and the gap_post bases after the seed's span
    uint32_t gap_at = 0, gap_len = 0, gap_post = 0;
};

// Split seeds.  Under I = 0 a window within N <= 1 mismatches of a record seeded at its
// primer start, plain over bases [0, S) (S = split_span(W) = W + 2a, a = kSplitSeed - W),
// matches the key [0, W) exactly and has at most one mismatch in [W, S).  Cut that stretch
// into A = [W, W + a) and B = [W + a, S): one of them is exact (pigeonhole), so the window is
// found by the exact seed [0, W + a) or by the gapped seed [0, W) ++ B -- both kSplitSeed = 11
// bases, the c3 word size: scan_kernel's LDS prefilter and 2 MB key groups (which stay in an
// XCD's 4 MB L2; 12-base seeds' 8 MB groups did not: 17 GB of L2 fills per scan) handle them
// as they handle c3, where dense_kernel loads a filter oct for ~60% of all windows.  The
// gapped scan keeps only windows whose A has a mismatch (or an invalid base), so no window
// is found twice; its key groups also test the split_post(W) bases after S.  Every base the
// gapped scan reads lies within a lane's 48 (window 31 + S + post <= 48).
constexpr uint32_t kSplitSeed = 11;
__host__ __device__ constexpr uint32_t split_span(uint32_t W) { return 2 * kSplitSeed - W; }
__host__ __device__ constexpr uint32_t split_post(uint32_t W) { return 17 - split_span(W) < 3 ? 17 - split_span(W) : 3; }

struct Genome {
    int device = 0;
    uint32_t n_seq = 0;
    std::vector<uint64_t> len, base;  // host copies
    uint64_t total = 0;               // padded bases
    uint64_t* g2 = nullptr;
    uint64_t* gexc = nullptr;
    uint64_t* gwild = nullptr;                // 'N' bases (pair check under I = 1: they match any primer base)
    // The pair check's planes interleaved (round 5, built at seal): per 64-base block b the
    // 32 B {g2 word 2b, g2 word 2b + 1, gexc word b, gwild word b}, so a survivor's stretch
    // of ~130 bases is one or two 128-B lines instead of one or two per plane (c4's pair
    // kernel fetched ~1.6 GB per launch, ~580 B per survivor).
    uint64_t* gpair = nullptr;
    uint64_t* ginv = nullptr;
    uint64_t* d_base = nullptr;
    uint64_t* d_len = nullptr;
    uint64_t* xr_start = nullptr;
    uint8_t* xr_char = nullptr;
    uint64_t xr_cap = 0, n_xr = 0;
    uint32_t* xr_dir = nullptr;               // last run starting at or before b * 4096
    uint64_t n_dir = 0;
    unsigned long long* d_ucount = nullptr;   // U bases seen by the packer
    bool has_u = false;
    unsigned long long* d_counter = nullptr;  // run-count scratch
    uint8_t* staging = nullptr;
    uint64_t staging_cap = 0;
    bool sealed = false;
    uint64_t dev_bytes = 0;
    uint64_t plane_cap = 0;   // padded bases the planes hold
    uint32_t seq_cap = 0;     // sequences d_base / d_len hold
    uint32_t n_pending = 0;   // search runs enqueued over this genome and not yet completed
};

struct Search {
    Table* table = nullptr;
    Genome* genome = nullptr;
    uint64_t cap = 0;
    uint64_t* keys = nullptr;    // 2 x u64 per raw hit (hi, lo), unsorted
    uint64_t* tmp_hi = nullptr;  // sort buffers
    uint64_t* tmp_lo = nullptr;
    mp_hit* out = nullptr;
    void* sort_tmp = nullptr;
    size_t sort_tmp_bytes = 0;
    unsigned long long* counters = nullptr;  // [0] hits, [1] candidates, [2] survivors
    uint4* surv = nullptr;                   // fingerprint survivors {gk lo, gk hi, rec|exact, seq}
    uint64_t surv_cap = 0;
    uint4* tails = nullptr;                  // multi-record buckets {seed gpos lo, hi, xstart, seq}
    uint64_t tails_cap = 0;
    SeqSpan* spans = nullptr;
    uint64_t spans_cap = 0;
    int n_cu = 0;
    uint64_t n_hits = 0;
    uint64_t n_windows = 0, n_candidates = 0, n_survivors = 0;
    float scan_ms = 0.f, tail_ms = 0.f, pair_ms = 0.f, order_ms = 0.f;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev3 = nullptr, evt = nullptr;
    uint32_t* bucket = nullptr;  // device sort: bucket counts, offsets, cursors
    uint64_t* slots = nullptr;   // order mode 0: every bucket's keys at bucket * slot_cap
    size_t slots_bytes = 0;
    // Hit order, sticky per handle and only ever raised (a crowded bucket seen once is
    // likely seen again): 0 = bucket slots written by pair_kernel + one sort/decode kernel;
    // 1 = scatter by the fused offsets + per-bucket LDS sort (up to kSortCap keys);
    // 2 = rocPRIM on the host-known count.  Keys over 64 bits always take 2.
    int order_mode = 0;
    mp_search_options opt{};     // kernel-path selection (all zero = automatic)
    uint32_t pair_per_cu = 0;    // resident pair_kernel blocks per CU (occupancy query at create)
    uint32_t dense_per_cu = 0;   // resident dense_kernel blocks per CU
    size_t dense_lds = 0;        // dense_kernel dynamic LDS bytes
    uint64_t n_regrowths = 0;    // list regrowths over the handle's life (tests)
    std::vector<SeqSpan> last_spans;        // spans on the device (a rerun of the same range uploads nothing)
    // pinned, device-mapped host words: [0, 8) counters[0..8) written by finish_kernel at
    // the end of every run (the run's one readback, no copy); [8] staging for a host upload
    unsigned long long* h_cnt = nullptr;
    unsigned long long* d_hcnt = nullptr;   // h_cnt as the device sees it
    hipEvent_t evd = nullptr;               // the run's completion (polled, not slept on)
    unsigned long long* h_put = nullptr;    // mp_search_put_hits: pinned ring of hit counts in flight
    hipEvent_t* put_ev = nullptr;           // per ring slot (kPutRing): its count's copy has run (slot reuse)
    hipEvent_t put_done = nullptr;          // the last put has read the hit list (next enqueue waits)
    bool put_wait = false;
    uint32_t put_seq = 0;
    bool stage_timing = true;               // events around tail/pair/order too (mp_search_set_stage_timing)
    bool scan_timing = true;                // the scan kernel's own two events (mp_search_set_scan_timing)
    bool dirty = false;                     // counters not known to be zero (an abandoned run): memset first
    // an enqueued run waiting for mp_search_complete
    bool pending = false;
    bool pend_empty = false;                // nothing to scan: completes with no hits
    hipStream_t pend_st = nullptr;
    uint64_t pend_tiles = 0;                // super-steps of the enqueued run
    int pend_mode = 0;                      // its order mode
    alignas(16) unsigned char pend_args[640];  // its ScanArgs (mp_search.hip)
};

// ---------------------------------------------------------------- device helpers
// 32 bases (64 bits) of the 2-bit plane starting at global base j, base j on top.
__device__ __forceinline__ uint64_t ext2(const uint64_t* __restrict__ p, uint64_t j) {
    const uint64_t w = j >> 5;
    const uint32_t s = (uint32_t)(j & 31) * 2;
    const uint64_t a = p[w];
    const uint64_t b = p[w + 1];
    return s ? (a << s) | (b >> (64 - s)) : a;
}

// Genome::gpair words: 2-bit word w, exception / 'N' word e.
__device__ __forceinline__ uint64_t gp_g2(const uint64_t* __restrict__ p, uint64_t w) { return p[((w >> 1) << 2) | (w & 1)]; }
__device__ __forceinline__ uint64_t gp_exc(const uint64_t* __restrict__ p, uint64_t e) { return p[(e << 2) | 2]; }
__device__ __forceinline__ uint64_t gp_wild(const uint64_t* __restrict__ p, uint64_t e) { return p[(e << 2) | 3]; }
// ext2 / ext1 over Genome::gpair (kPlane 2: gexc, 3: gwild)
__device__ __forceinline__ uint64_t ext2p(const uint64_t* __restrict__ p, uint64_t j) {
    const uint64_t w = j >> 5;
    const uint32_t s = (uint32_t)(j & 31) * 2;
    const uint64_t a = gp_g2(p, w), b = gp_g2(p, w + 1);
    return s ? (a << s) | (b >> (64 - s)) : a;
}
template <int kPlane>
__device__ __forceinline__ uint64_t ext1p(const uint64_t* __restrict__ p, uint64_t j) {
    const uint64_t w = j >> 6;
    const uint32_t s = (uint32_t)(j & 63);
    const uint64_t a = p[(w << 2) | kPlane], b = p[((w + 1) << 2) | kPlane];
    return s ? (a << s) | (b >> (64 - s)) : a;
}

// 64 bits of a 1-bit plane starting at global base j, base j on top.
__device__ __forceinline__ uint64_t ext1(const uint64_t* __restrict__ p, uint64_t j) {
    const uint64_t w = j >> 6;
    const uint32_t s = (uint32_t)(j & 63);
    const uint64_t a = p[w];
    const uint64_t b = p[w + 1];
    return s ? (a << s) | (b >> (64 - s)) : a;
}

// Spaced mask (bit 62-2i) for primer-chunk positions i < b, 0 <= b <= 32.
__host__ __device__ __forceinline__ uint64_t sp_lt(int b) {
    return b <= 0 ? 0ull : (b >= 32 ? kEven : (kEven & (~0ull << (64 - 2 * b))));
}

__host__ __device__ __forceinline__ uint32_t iupac_mask(uint8_t c) {
    // A=1 C=2 G=4 T=U=8 (engine.py:138-172 expansion sets, as bit masks)
    switch (c) {
        case 'A': return 1; case 'C': return 2; case 'G': return 4;
        case 'T': case 'U': return 8;
        case 'R': return 5; case 'Y': return 10; case 'M': return 3; case 'K': return 12;
        case 'S': return 6; case 'W': return 9; case 'B': return 14; case 'D': return 13;
        case 'H': return 11; case 'V': return 7; case 'N': return 15;
        default: return 0;
    }
}

// engine.py:613-631: one genome character against one primer character.
__host__ __device__ __forceinline__ bool char_match(uint8_t g, uint8_t c, int iupac) {
    if (iupac) {
        const uint32_t mg = iupac_mask(g), mc = iupac_mask(c);
        if (mg && mc) return (mg & mc) != 0;
    }
    return g == c;
}

__host__ __device__ __forceinline__ uint32_t table_slot(uint32_t key, uint32_t log2cap) {
    return (uint32_t)(((uint64_t)key * 0x9E3779B97F4A7C15ull) >> (64 - log2cap));
}

__host__ __device__ __forceinline__ uint32_t filter_index(uint32_t key, uint32_t log2bits) {
    return (uint32_t)(((uint64_t)key * 0xD6E8FEB86659FD93ull) >> (64 - log2bits));
}

// 8-B bucket head: for a single-record bucket whose seed is primer 1's first W bases,
// primer 1 plain (one A/C/G/T per position) and at most W + 16 bases long, the seed
// key plus the 2-bit code of bases W..W+15 restate the whole 32-B Entry; any other
// head sets kHead8Full and the lookup reads the full Entry.
constexpr uint32_t kHead8Full = 0x80000000u;
constexpr uint32_t kHead8RecBits = 26;
// A full head of a bucket of 1-3 records that are all seeded at primer 1's first base and
// plain over bases W..W+F-1 (F = 14 / records) may carry kHead8Filt: bits 28-29 hold
// records - 1 and bits [2F j, 2F j + 2F) record j's 2-bit bases W..W+F-1 (base W on
// top).  The ranked drain hands such a bucket to tail_kernel only when some record's F
// bases are within N mismatches of the genome (a lower bound on primer-1 mismatches).
constexpr uint32_t kHead8Filt = 0x40000000u;
// 8-B IUPAC head (Table::h12, round 3): the 16-B head's information for bases W..W+11 only --
// .x = their 2-bit codes (bits 31..8, base W on top) | l1 - W (bits 4..0, <= 31); .y = record
// (bits 0..17) | their plain bits (bit 29 = base W ... bit 18 = base W+11); a record with a
// "never" base there, a longer primer or more records is a full head (as dents8's).  Bases
// past W+11 are not tested in the drain, so a survivor of a primer longer than W+12 is not
// exact (pair_kernel compares it whole).  c4's 195k heads take 1.6 MB instead of 3.1 MB,
// and with the 1 MB rank words they stay in an XCD's 4 MB L2.
constexpr uint32_t kHead12RecBits = 18;
constexpr uint32_t kHead12Bases = 12;
__host__ __device__ __forceinline__ uint32_t head8_filt_bases(uint32_t records) { return 14u / records; }
// Tables with W <= 9 run dense_kernel: the rank bitmap (4^W / 4 bytes <= 64 KiB) lives in
// LDS and each lane walks its own seeds' buckets.
constexpr uint32_t kDenseMaxW = 9;
// Filter word of a dense_kernel entry (16 bits): primer-1 bases W..W+F-1 (2-bit, base W
// in bits 15:14), F <= 7 fixed per table, flags in bits 1:0.  A seed window whose bases
// W..W+F-1 differ from them in more than N positions cannot be a survivor (a mismatch at a
// plain primer position is a real one; a genome exception base there reads as 'A' and can
// only hide mismatches under I=0, and windows with exception bases take the full test
// under I=1), so only the words that pass reach the 32-B Entry.  Buckets of up to eight
// records, all carrying the filter, take one 16-B oct of filter words: one load per seed
// window, and the hot loop tests no flags (spare slots repeat slot 0's bases); other buckets
// (longer, or holding a record the filter cannot carry) are walked through binfo.
constexpr uint32_t kDenseAlways = 1u;   // entry not filterable (seed inside the primer, short or IUPAC primer)
constexpr uint32_t kDensePad = 2u;      // spare slot of an oct
constexpr uint32_t kDenseMaxF = 7;
// Per-key summary (W <= kDenseSumMaxW, N <= 1; 16 bits per key, staged in LDS beside the
// bucket index): a window's oct is loaded only when some record of its key could pass the
// filter.  N = 0: bit dsum_hash4(all F bases) of each record.  N = 1: F bases split into
// A (first FA = ceil(F/2)) and B (last F - FA); a window within one mismatch of a record
// matches it exactly on A or on B (pigeonhole), so bits dsum_hash3(A) and 8 + dsum_hash3(B)
// are set per record and the window needs one of its two bits.  A hashed bit can only make
// a window pass that the exact rule rejects, never the reverse.  Buckets the filter cannot
// carry (escape) have every bit set.
constexpr uint32_t kDenseSumMaxW = 8;
__host__ __device__ __forceinline__ uint32_t dsum_hash3(uint32_t v) { return (v ^ (v >> 3) ^ (v >> 6)) & 7u; }
__host__ __device__ __forceinline__ uint32_t dsum_hash4(uint32_t v) { return (v ^ (v >> 4) ^ (v >> 8) ^ (v >> 12)) & 15u; }
constexpr uint32_t kDenseOct = 8;

// LDS prefilter bit of a seed key.  Exact (bit = key) when 4^W fits (W <= 10);
// above, the top 20 bits of the key left-aligned in 32 bits: keys that differ only in
// their last 2W-20 bits share a bit.  In the scan the left-aligned form is the
// alignbit funnel itself, so a probe costs one shift, one mask and one extract --
// no multiply (v_mul_lo_u32 issues at quarter rate).
__host__ __device__ __forceinline__ uint32_t lds_bit(uint32_t key, uint32_t W, bool exact) {
    return exact ? key : (key << (32u - 2u * W)) >> (32 - kLdsFilterLog2);
}

// W 11..13 (the rank-bitmap tables): a blocked filter -- the word is the key's top 15 bits
// (as above) and k bits inside it are set: the next 5 bits and, for k = 2, the key's last
// 5 bits.  One LDS read per window either way; the second bit cuts the windows that reach
// the global rank-word probe (c3: 17.4% -> 12.9%) and is worth its extra VALU only for
// large tables (more than kLdsK2Keys distinct keys: above ~16 filter bits per key the
// single bit already rejects nearly all random windows).
constexpr uint64_t kLdsK2Keys = 65536;
__host__ __device__ __forceinline__ uint32_t lds_block_mask(uint32_t x, uint32_t shw, int k) {
    // x: the key left-aligned in 32 bits (x >> shw = key)
    uint32_t m = 1u << ((x >> (32 - kLdsFilterLog2)) & 31u);
    if (k >= 2) m |= 1u << ((x >> shw) & 31u);
    if (k >= 3) m |= 1u << (((((x >> shw) & 127u) * 37u) >> 2) & 31u);  // a third function of the word's 7 free key bits
    return m;
}

// Key groups (kgrp), the level-2 table of the scan for W 11..13 under I = 0: one u64 per 16
// consecutive keys of the exact 4^W presence bitmap -- bits 0-15 presence, then three 16-bit
// fields for the group's first three present keys.  A field with its top bit set belongs to a
// key whose bucket is one record seeded at its primer start and plain (the 8-B compact head)
// and holds that primer's bases W..W+F-1 (2-bit, base W on top, in the low 2F bits).  The
// probe that confirms a seed thus also filters it: a window whose bases there differ in more
// than N positions cannot be a survivor (each counted position is a real mismatch under
// I = 0; a genome exception base reads as 'A' and can only hide one), so the seed ends at
// the probe.  Other seeds leave as key references for tail_kernel.
constexpr uint32_t kKgrpKeys = 16;
constexpr uint32_t kKgrpFields = 3;
constexpr uint32_t kKgrpFlag = 0x8000u;
// A field of a key with exactly two records, both seeded at their primer start and plain over
// bases W..W+2 (round 3): kKgrpPair, then each record's bases W..W+2 (record 0 in bits 11..6).
// The window passes when either record is within N of them.  Without it every seed of such a
// key went to tail_kernel: c3's ~5k two-record keys gave most of its 3.4M bucket-tail references.
constexpr uint32_t kKgrpPair = 0x4000u;
constexpr uint32_t kKgrpWildFields = 2;  // I = 1 key groups: two 24-bit fields {codes, wild bases}
// Wide I = 1 key groups (kgrp4, round 4; c4: degenerate primers, N = 2): one 16-B word per 32
// keys of the exact 4^W bitmap, for tables whose heads are in the 8-B IUPAC form (Table::h12).
// .x the 32 presence bits; .y, .z, .w a 32-bit field for each of the group's first three
// present keys: bits 0..2F-1 the 2-bit codes of primer-1 bases W..W+F-1 (base W on top), bits
// 2F..3F-1 their plain flags (base W on top).  A key whose bucket is not one record seeded at
// its primer start has no plain flag set, nor has an IUPAC base or a base past the primer's
// end.  The probe counts mismatches at the plain bases only, a lower bound on primer-1
// mismatches when the window's first W + F genome bases are all A/C/G/T/U (other windows pass
// on presence), so more than N ends the seed at the probe; the rest leave as key references,
// whose bucket tail_kernel finds by the rank word and the 8-B IUPAC head.  One 16-B load per
// level-1 positive replaces the rank word, and the drain with its head load per seed is gone
// (c4: ~12% of seeds pass, against ~30% for the 8-B groups' six bases).  2 MB at W = 11.
#ifndef MP_KGRP4_KEYS
#define MP_KGRP4_KEYS 32
#endif
constexpr uint32_t kKgrp4Keys = MP_KGRP4_KEYS;  // 16 or 32
constexpr uint32_t kKgrp4Log2 = kKgrp4Keys == 16 ? 4 : 5;
static_assert(kKgrp4Keys == 16 || kKgrp4Keys == 32, "key-group size");
constexpr uint32_t kKgrp4Fields = 3;
constexpr uint32_t kKgrp4F = 10;

__host__ __device__ __forceinline__ uint32_t try_rank(int32_t d) {
    return d == 0 ? 0u : (d < 0 ? (uint32_t)(-2 * d - 1) : (uint32_t)(2 * d));
}

__host__ __device__ __forceinline__ int32_t try_offset(uint32_t r) {
    return r == 0 ? 0 : ((r & 1) ? -(int32_t)((r + 1) >> 1) : (int32_t)(r >> 1));
}

inline uint64_t round_up(uint64_t x, uint64_t m) { return (x + m - 1) / m * m; }

// internal entry points shared across TUs
// rocPRIM order of the run's n hits (the regions compacted first); the sorted (hi, lo)
// arrays are returned for decode_kernel
int sort_hits(Search* s, uint64_t n, hipStream_t st, const uint64_t** hi_out, const uint64_t** lo_out);
bool sort_hits_device_ok(const Search* s);
// The device sort's packing and bucketing of the 64-bit order key (k << low_bits | record
// rank << try_bits | try rank; bucket = key >> shift), fixed per search before the scan.
struct SortPlan {
    unsigned try_bits = 0, low_bits = 0, shift = 0;
    uint32_t nb = 0;
    uint32_t slot_cap = 0;  // order mode 0: keys per bucket slot
};
constexpr uint32_t kSlotCap = 256;  // order mode 0: bucket slot capacity (~8x the planned mean)
SortPlan sort_plan(const Search* s);
// pair_kernel already wrote the packed keys (tmp_lo) and the bucket counts; mode 0: the keys
// also in their bucket slots.  Bucket offsets, then the sort.  Hit count read on the device;
// writes s->out.
// finish: the offsets launch also copies counters[0..8) to the mapped host words and zeroes
// the counters (the run's end; see bucket_offsets).
int sort_hits_device(Search* s, hipStream_t st, int mode, bool finish);
size_t counter_bytes();  // the run counters' size (mp_search.hip)
uint32_t* sort_bucket_counts(Search* s);          // the bucket count array (zeroed by the scan kernels)
uint32_t* sort_bucket_offsets(Search* s);         // nb + 1 offsets
uint32_t* sort_bucket_cursors(Search* s);
unsigned long long* sort_region_counts(Search* s);  // the run's hit-region counts (finish_fold)
uint32_t* sort_crowded(Search* s);                 // [0] count, then the crowded buckets of a mode-1 run
int alloc_sort_slots(Search* s, const SortPlan& P);  // mode 0's slot array for plan P

// Raw hits arrive in runs of one bucket (a survivor's tries, a wave's batch of nearby
// survivors; IUPAC primers over N runs pile thousands on a few positions).  Same-address
// atomics serialise at the L2, so each wave collapses its runs of equal buckets: the run
// head adds the run length once and hands the base to the run's other lanes.  Wave-uniform.
__device__ __forceinline__ void bucket_runs(uint32_t b, bool on, int lane, uint32_t& head, uint32_t& len) {
    const uint32_t prev = (uint32_t)__shfl_up((int)b, 1, 64);
    const uint64_t heads = __ballot(on && (lane == 0 || prev != b));
    const uint64_t upto = heads & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
    head = upto ? 63u - (uint32_t)__clzll(upto) : 0u;  // this lane's run head
    const uint64_t above = heads & ~((2ull << lane) - 1ull);
    const uint64_t onm = __ballot(on);
    const uint32_t end = above ? (uint32_t)__ffsll((long long)above) - 1u : 64u - (uint32_t)__clzll(onm);
    len = end - (uint32_t)lane;  // meaningful on heads only
}
// Exclusive scan of nb bucket counts by one 1024-thread workgroup: off[0..nb] (off[nb] =
// total) and cursor[0..nb) = off.  The counts pass through LDS (s_v4: kOffTile counts) in
// tiles: coalesced loads and stores (all kOffTile / 1024 loads of a thread in flight at once:
// one memory round trip per tile), kOffPer consecutive counts per thread inside a tile, a
// wave shuffle scan and one LDS word per wave (s_w: 16).  (64 consecutive counts per thread
// straight from memory made every access a 64-line gather: c4's 65,536 buckets took 80 us;
// tiles of 8,192 took 36 us, eight round trips and 24 barriers; 32,768 spilled.)
constexpr uint32_t kOffTile = 16384;
constexpr uint32_t kOffPer = kOffTile / 1024;
// crowded (optional): the buckets of more than crowd_lo and at most crowd_hi counts are
// listed at crowded[1..] (in no order), their number in *s_crowd (LDS, zeroed by the caller).
__device__ __forceinline__ void bucket_offsets_block(const uint32_t* cnt, uint32_t nb, uint32_t* off,
                                                     uint32_t* cursor, uint4* s_v4, uint32_t* s_w,
                                                     uint32_t* crowded = nullptr, uint32_t* s_crowd = nullptr,
                                                     uint32_t crowd_lo = 0, uint32_t crowd_hi = 0) {
    static_assert(kOffPer % 4 == 0, "whole uint4 per thread");
    uint32_t* s_v = reinterpret_cast<uint32_t*>(s_v4);
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nb; base += kOffTile) {
        uint32_t ld[kOffPer];
#pragma unroll
        for (uint32_t j = 0; j < kOffPer; ++j) {
            const uint32_t i = j * 1024 + t;
            ld[j] = base + i < nb ? cnt[base + i] : 0u;
        }
#pragma unroll
        for (uint32_t j = 0; j < kOffPer; ++j) s_v[j * 1024 + t] = ld[j];
        if (crowded) {
#pragma unroll
            for (uint32_t j = 0; j < kOffPer; ++j)
                if (ld[j] > crowd_lo && ld[j] <= crowd_hi) crowded[1 + atomicAdd(s_crowd, 1u)] = base + j * 1024 + t;
        }
        __syncthreads();
        uint32_t sum = 0;  // the thread's counts are read twice from LDS: sum, then the scan
#pragma unroll
        for (uint32_t j = 0; j < kOffPer / 4; ++j) {
            const uint4 q = s_v4[(kOffPer / 4) * t + j];
            sum += q.x + q.y + q.z + q.w;
        }
        uint32_t x = sum;  // inclusive scan over the wave
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
            if ((int)lane >= o) x += y;
        }
        if (lane == 63) s_w[w] = x;
        __syncthreads();
        uint32_t wpre = 0, tot = 0;
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            const uint32_t sw = s_w[k];
            wpre += k < w ? sw : 0u;
            tot += sw;
        }
        uint32_t run = carry + wpre + x - sum, v;
#pragma unroll
        for (uint32_t j = 0; j < kOffPer / 4; ++j) {
            uint4 q = s_v4[(kOffPer / 4) * t + j];
            v = q.x; q.x = run; run += v;
            v = q.y; q.y = run; run += v;
            v = q.z; q.z = run; run += v;
            v = q.w; q.w = run; run += v;
            s_v4[(kOffPer / 4) * t + j] = q;
        }
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < kOffPer; ++j) {
            const uint32_t i = j * 1024 + t;
            if (base + i < nb) {
                const uint32_t o = s_v[i];
                off[base + i] = o;
                cursor[base + i] = o;
            }
        }
        carry += tot;
        __syncthreads();  // s_v and s_w are rewritten by the next tile
    }
    if (t == 0) off[nb] = carry;
}

int alloc_sort_buckets(Search* s);                // the device sort's bucket arrays (at create)
constexpr int kSortOverflow = 6;                  // counters[6]: a device-sort bucket overflowed

// Run counters (Search::counters, uint64 words).  Statistics and work queues live 256 B apart
// (kStatStride words): thousands of waves on one address serialise (~88 returning atomics per
// microsecond, MI355X_MICROARCH.md "dequeue").
//   [0..8)          run results, copied to the host words at the run's finish
//   kStatBase       64 candidate / survivor statistic slots
//   kPairQBase      8 pair_kernel batch counters (one per XCD group)
//   kSchedBase      8 scan super-step chunk counters
//   kHitBase        8 hit-list reservation counters: region x of the hit list (hit_hi / hit_lo /
//                   sort_keys at [x * cap_r, (x + 1) * cap_r)) belongs to the pair blocks of
//                   XCD group x, so the hit flushes of a run spread over eight words (c4: 25k
//                   flushes on one word were ~0.28 ms of serialised atomics)
constexpr int kStatBase = 32, kStatSlots = 64, kStatStride = 32;
constexpr int kPairQBase = kStatBase + kStatSlots * kStatStride;
constexpr int kSchedBase = kPairQBase + 8 * kStatStride;
constexpr int kHitBase = kSchedBase + 8 * kStatStride;
constexpr int kHitRegions = 8;
//   kSchedSplit     two more sets of 8 chunk counters: the gapped and the rest scans of a split
//                   run (kSplitSeed) -- every scan of a run claims from counters zeroed by the
//                   previous run's finish
constexpr int kSchedSplit = kHitBase + kHitRegions * kStatStride;
constexpr size_t kCounterBytes = (size_t)(kSchedSplit + 2 * 8 * kStatStride) * 8;
constexpr int kHitMaxRegion = 8;                  // host word 8: the largest region count of the run
constexpr int kHostWords = 16;                    // device-mapped host words per search

// The run's finish, by one workgroup after the last producer (pair_kernel): counters[0..8)
// to the host words with word 0 = the hit total (the sum of the region counts), words 1 and 3
// = the candidate and survivor statistics (the sums of the add_stats slots), word
// kHitMaxRegion = the largest region count (capacity check), the region counts to rcount
// (device copy for the order kernels), then every counter zeroed for the next run.
__device__ __forceinline__ void finish_fold(unsigned long long* __restrict__ counters, uint32_t n_words,
                                            unsigned long long* __restrict__ h_out,
                                            unsigned long long* __restrict__ rcount) {
    unsigned long long v = 0, r = 0, sc = 0, ss = 0;
    if (threadIdx.x < 8) {
        v = counters[threadIdx.x];
        r = counters[kHitBase + threadIdx.x * kStatStride];
    }
    if (threadIdx.x < kStatSlots) {  // the candidate / survivor statistic slots (add_stats)
        sc = counters[kStatBase + threadIdx.x * kStatStride];
        ss = counters[kStatBase + threadIdx.x * kStatStride + 1];
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n_words; i += blockDim.x) counters[i] = 0ull;
    if (threadIdx.x < 64) {  // wave 0: the region sum and maximum over lanes 0..7, the statistics' sums
        static_assert(kStatSlots == 64, "one statistic slot per lane of wave 0");
        unsigned long long sum = r, mx = r;
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) {
            const unsigned long long ys = (unsigned long long)__shfl_xor((long long)sum, o, 64);
            const unsigned long long ym = (unsigned long long)__shfl_xor((long long)mx, o, 64);
            sum += ys;
            mx = ym > mx ? ym : mx;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            sc += (unsigned long long)__shfl_xor((long long)sc, o, 64);
            ss += (unsigned long long)__shfl_xor((long long)ss, o, 64);
        }
        if (threadIdx.x < 8) {
            rcount[threadIdx.x] = r;
            h_out[threadIdx.x] = threadIdx.x == 0 ? sum : threadIdx.x == 1 ? sc : threadIdx.x == 3 ? ss : v;
            if (threadIdx.x == 0) h_out[kHitMaxRegion] = mx;
            __threadfence_system();  // the host polls the run's event, then reads these
        }
    }
}
int sort_runs(Genome* g, hipStream_t st);

}  // namespace mp
