// The hot path: seed scan -> primer-1 verify -> amplicon pair-check -> hits.
//
// Replaces, with T=1 semantics, MerPCR._process_thread (engine.py:453-505),
// _match_sts (engine.py:507-597) and _compare_seqs (engine.py:599-642), all in
// src/merpcr/core/engine.py of the reference.
//
// Kernel structure: a persistent grid of one 1024-thread workgroup per CU.  Each
// workgroup first stages the 64 KiB seed prefilter in LDS; then every wave walks
// "super-steps" of 2048 consecutive window positions of one sequence (32 per lane):
//   1. seed stage: the lane's two 2-bit words and one ambiguity word cover its 32
//      windows (coalesced loads, prefetched one super-step ahead).  Every W-mer comes
//      from registers (alignbit), the "all A/C/G/T/U" test of engine.py:464-503 is one
//      smear of the ambiguity word, the LDS prefilter is probed by ds_read and, where
//      it passes and is not exact, the global presence bitmap (8 probes in flight).
//   2. compaction: seed hits (about 4.6% of windows at W=11 / 100k STS) become u16
//      offsets in a per-wave LDS queue (popcount + wave prefix).
//   3. drain: one lane per queued seed.  Its W-mer and the genome window of the
//      candidate primer come from the wave's registers by cross-lane shuffles.  The
//      bucket head (exact rank bitmap for W <= 13, open-addressed slot above) holds a
//      primer-1 fingerprint; a 2-bit XOR/popcount lower bound on the mismatches
//      rejects almost every random seed from that one 32-B entry.  Buckets with more
//      records are expanded 64 candidates per pass.
//   4. survivors (at most 64 per pass) are verified and pair-checked by the whole
//      wave (primer_ok: bit-sliced accept planes, exception bases resolved through the
//      run index; lanes split the amplicon-end offsets) and emit 128-bit order keys.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <utility>

#include "mp_internal.h"

// survivors per pair-check batch (lanes of the prologue); smaller batches spread the
// per-survivor loop over more waves
#ifndef MP_PBATCH
#define MP_PBATCH 64
#endif


namespace mp {

struct ScanArgs {
    const uint64_t* g2;
    const uint64_t* gexc;
    const uint64_t* ginv;
    const uint64_t* gwild;  // 'N' bases: under I = 1 they match every primer base with an IUPAC meaning
    const uint64_t* gpair;  // the pair check's planes interleaved (Genome::gpair)
    const uint64_t* xr_start;
    const uint8_t* xr_char;
    const uint32_t* xr_dir;
    uint64_t n_xr;
    const uint64_t* seq_base;
    const uint64_t* seq_len;
    const SeqSpan* spans;
    uint32_t n_spans;
    const uint32_t* filt;   // W >= 14: hashed presence filter
    uint32_t filt_log2;
    const uint2* rk;        // W <= 13: rank bitmap
    const uint2* kgrp;      // W 11..13: key groups (u64 per 16 keys, see kKgrpKeys)
    uint32_t kgrp_F;
    int kgrp_wild;          // I = 1 field form (kgrp_pass)
    const uint4* kgrp4;     // I = 1 wide key groups (uint4 per kKgrp4Keys keys; kgrp_pass4)
    uint32_t sched_short;   // super-steps per claim in short scans (SuperSched)
    const Entry* dents;     // W <= 13: bucket heads by rank
    const uint2* dents8;    // W <= 13: 8-B heads
    const uint4* dents16;   // W <= 13, Table::h16: 16-B heads (primers with IUPAC bases after the seed)
    const uint2* dents12;   // Table::h12: the same heads in the 8-B IUPAC form (kHead12RecBits)
    const uint2* binfo;     // W <= kDenseMaxW: bucket {first padded entry, records} by key rank
    const uint16_t* dfilt;  // W <= kDenseMaxW: filter word per padded entry
    const uint2* dgrp;      // W <= kDenseMaxW: per-32-key bucket index
    const uint32_t* dgesc;  // W <= kDenseMaxW: per-32-key escape bits
    const Entry* dents_pad; // W <= kDenseMaxW: Entry per padded entry
    uint32_t dense_M;       // filter mismatch mask
    const uint16_t* dsum;   // W <= kDenseSumMaxW, N <= 1: per-key summary of the filter bases
    int dsum_mode;          // 0: none, 1: N = 0 form, 2: N = 1 form
    uint32_t dense_F;       // filter bases per word
    int defer_full;         // ranked drain: full-head buckets go whole to tail_kernel
    const uint32_t* lfilt;
    const Slot* slots;
    uint32_t slot_log2;
    const Entry* ents;
    const DevRec* recs;
    const uint32_t* rank;
    const uint64_t* planes;
    const PairRec* prec;      // the pair check's per-record lines (Table::prec)
    const uint8_t* pchars;
    int W, M, N, X, I;
    int has_u;              // genome holds U: exception bits come from gexc, not ginv
    uint64_t g_lo, g_hi;
    uint64_t* hit_hi;
    uint64_t* hit_lo;
    unsigned long long* counters;
    uint64_t cap;
    uint64_t cap_r;         // hit-list region capacity (cap / kHitRegions), see kHitBase
    uint4* surv;
    uint64_t surv_cap;
    uint4* tails;           // bucket-tail references (2 x uint4 each), see tail_kernel
    uint64_t tails_cap;
    // device sort fused into the pair check (SortPlan): pair_kernel writes each hit's packed
    // order key and counts its bucket; the scan kernels zero the counts (null: not fused)
    uint64_t* sort_keys;
    uint32_t* sort_cnt;
    uint32_t sort_nb, sort_shift, sort_try_bits, sort_low_bits;
    uint64_t* sort_slots;   // order mode 0: keys straight into their bucket slot (null: mode 1)
    uint32_t slot_cap;
    // gapped seed (split tables, kSplitSeed): key = bases [0, gap_at) ++ the W - gap_at bases
    // after the gap_len-base gap; gap_len 0: contiguous.  Its key-group fields hold the gap's
    // bases and the gap_post bases after the seed's span.
    uint32_t gap_at, gap_len, gap_post;
    uint32_t tail_ctr;      // counters[] slot of this scan's bucket-tail list (4; 5 for the gapped scan)
    uint64_t tail_static;   // bucket-tail slots reserved statically, kStaticRefs per scan wave (the
                            // list is [0, tail_static + counters[tail_ctr]))
    uint32_t ref16;         // key references in the 16-B form (Ref16); else 32-B bucket references
    uint32_t sched_base;    // counters[] index of this scan's 8 chunk counters (kSchedBase, kSchedSplit...)
};

// The gapped key of a 16-base funnel x (base 0 on top), left-aligned like a contiguous key:
// the top gap_at bases, then the bases after the gap (the low bits below the key are junk,
// as in the contiguous form).  One shift and one bit-field insert.
// kGap = kGapW8 (c5's split): the W = 8 gapped seed's shape as compile-time constants, so that
// its level 1 needs no key assembly for the filter word and the second filter bit (below),
// and the scan holds three fewer scalars (its SGPRs spill into VGPR lanes)
constexpr int kGapW8 = 8;
constexpr uint32_t kGapW8At = 8, kGapW8Len = 3, kGapW8Post = 3;
__device__ __forceinline__ uint32_t gap_key(uint32_t x, uint32_t gap_at, uint32_t gap_len) {
    const uint32_t hm = ~(0xFFFFFFFFu >> (2u * gap_at));
    return (x & hm) | ((x << (2u * gap_len)) & ~hm);
}

// Bucket counts of the fused device sort, zeroed by every block of a scan kernel.
__device__ __forceinline__ void zero_sort_counts(const ScanArgs& a) {
    if (!a.sort_cnt) return;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < a.sort_nb; i += gridDim.x * blockDim.x) a.sort_cnt[i] = 0;
}

// 64-bit min/max as plain compares (HIP's templated min/max on 64-bit integers went
// through f64 conversions in the scan kernel's loop header).
__device__ __forceinline__ int64_t smin64(int64_t x, int64_t y) { return x < y ? x : y; }
__device__ __forceinline__ int64_t smax64(int64_t x, int64_t y) { return x > y ? x : y; }
__device__ __forceinline__ uint64_t umin64(uint64_t x, uint64_t y) { return x < y ? x : y; }
__device__ __forceinline__ uint64_t umax64(uint64_t x, uint64_t y) { return x > y ? x : y; }

// Candidate / survivor statistics (counters[1], counters[3]) are summed from 64 slots
// 256 B apart (counter layout: mp_internal.h): thousands of waves ending together serialise
// on one address (~11 ns per atomic, MI355X_MICROARCH.md) -- measured ~0.1 ms on
// tail_kernel's exit.  pair_kernel folds the slots into counters[1] and counters[3] before
// the host reads them.
size_t counter_bytes() { return kCounterBytes; }
#ifndef MP_PDYN_BATCH
#define MP_PDYN_BATCH 64
#endif
#ifndef MP_PAIR_MINB
#define MP_PAIR_MINB 4
#endif

__device__ __forceinline__ void add_stats(const ScanArgs& a, uint32_t cand, uint32_t surv, int lane) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        cand += __shfl_xor(cand, o, 64);
        surv += __shfl_xor(surv, o, 64);
    }
    const uint32_t slot = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (kStatSlots - 1);
    unsigned long long* c = a.counters + kStatBase + slot * kStatStride;
    if (lane == 0 && cand) atomicAdd(&c[0], (unsigned long long)cand);
    if (lane == 0 && surv) atomicAdd(&c[1], (unsigned long long)surv);
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Run of exception base j: the run index entry with the largest start <= j, searched
// between the directory bounds of j's 4096-base block.
__device__ __forceinline__ uint64_t exc_run(const ScanArgs& a, uint64_t j) {
    const uint64_t b = j >> kDirShift;
    uint64_t lo = a.xr_dir[b];
    uint64_t hi = umin64((uint64_t)a.xr_dir[b + 1] + 1, a.n_xr);
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a.xr_start[mid] <= j) lo = mid;
        else hi = mid;
    }
    return lo;
}


// Exception bases of a window (bit 31-i of ex): their characters come from the run
// index, walked forward once from the first one; each is compared with the primer
// character as engine.py:613-631 does and its mismatch bit (62-2i of mmv) set or
// cleared.  Rare (windows touching non-ACGT bases), so kept out of line.
__device__ __forceinline__ uint64_t exception_mismatches(const ScanArgs& a, uint32_t ex, uint64_t gpos_c, uint32_t ch_c,
                                                     uint64_t mmv) {
    uint64_t j = exc_run(a, gpos_c + (uint32_t)__clz(ex));
    uint8_t gch = a.xr_char[j];
    uint64_t nxt = j + 1 < a.n_xr ? a.xr_start[j + 1] : ~0ull;
    while (ex) {
        const int i = __clz(ex);
        ex &= ~(0x80000000u >> i);
        const uint64_t pos = gpos_c + (uint32_t)i;
        while (pos >= nxt) {  // a later run starts inside the window
            ++j;
            gch = a.xr_char[j];
            nxt = j + 1 < a.n_xr ? a.xr_start[j + 1] : ~0ull;
        }
        // the primer character straight from memory (a register array indexed by i went
        // to scratch, which every wave of the kernel then paid for)
        const bool ok = char_match(gch, a.pchars[ch_c + (uint32_t)i], a.I);
        const uint64_t bit = 1ull << (62 - 2 * i);
        mmv = ok ? (mmv & ~bit) : (mmv | bit);
    }
    return mmv;
}

// 32-bit per-base mask (bit 31-i) -> spaced form (bit 62-2i).
__device__ __forceinline__ uint64_t spread32(uint32_t v) {
    uint64_t x = v;
    x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
    x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
    x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    x = (x | (x << 1)) & kEven;
    return x;
}

// Spaced form (bit 62-2i) -> 32-bit per-base mask (bit 31-i); inverse of spread32.
__device__ __forceinline__ uint32_t compress_even(uint64_t x) {
    x &= kEven;
    x = (x | (x >> 1)) & 0x3333333333333333ull;
    x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
    x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
    x = (x | (x >> 16)) & 0x00000000FFFFFFFFull;
    return (uint32_t)x;
}

// One chunk (bases c .. c+len-1, len <= 32) of _compare_seqs (engine.py:599-642):
// genome window G (2-bit, base c on top) and its exception bits ex (bit 31-i) against
// the primer's accept planes P.  Adds the chunk's mismatches to mm; false on a
// protected mismatch or more than N.
__device__ __forceinline__ bool chunk_ok(const ScanArgs& a, uint64_t G, uint32_t ex, uint64_t P0, uint64_t P1,
                                         uint64_t P2, uint64_t P3, uint64_t gpos_c, uint32_t ch_c, int len, uint32_t c,
                                         uint32_t L, bool plus, int& mm, uint32_t wild = 0u) {
    const uint64_t lo = G & kEven, hi = (G >> 1) & kEven;
    const uint64_t nlo = lo ^ kEven, nhi = hi ^ kEven;
    const uint64_t match = (nhi & nlo & P0) | (nhi & lo & P1) | (hi & nlo & P2) | (hi & lo & P3);
    const uint64_t inside = sp_lt(len);
    uint64_t mmv = ~match & inside;
    if (len < 32) ex &= ~(0xFFFFFFFFu >> len);
    if (a.I && (ex & wild)) {
        // I = 1: a genome 'N' (wild, a subset of ex) matches exactly the primer bases with an
        // IUPAC meaning -- the positions with an accept-plane bit (char_match) -- so it
        // needs no run lookup; its 2-bit code (A) already left the other positions mismatched
        wild &= ex;
        mmv &= ~(spread32(wild) & (P0 | P1 | P2 | P3) & kEven);
        ex &= ~wild;
    }
    if (ex && !a.I) {
        // literal compare (I=0): where the primer base is one of A/C/G/T (a plane bit set),
        // a genome exception character (never exactly A/C/G/T) cannot equal it -- a
        // mismatch without looking the character up; only the other positions need it
        const uint64_t acgt = (P0 | P1 | P2 | P3) & kEven;
        mmv |= spread32(ex) & acgt & inside;
        ex &= ~compress_even(acgt);
    }
    if (ex) mmv = exception_mismatches(a, ex, gpos_c, ch_c, mmv);
    uint64_t prot;
    if (plus) {
        const int64_t a0 = (int64_t)L - a.X - (int64_t)c;  // first protected local position
        prot = inside & ~sp_lt((int)smax64(smin64(a0, 32), 0));
    } else {
        const int64_t b0 = (int64_t)a.X - (int64_t)c;  // protected local positions < b0
        prot = sp_lt((int)smax64(smin64(b0, len), 0));
    }
    if (mmv & prot) return false;
    mm += __popcll(mmv);
    return mm <= a.N;
}

// _compare_seqs (engine.py:599-642) of the L genome bases at global gpos against
// one primer: protected positions are i >= L-X on the '+' strand (plus == true)
// and i < X on the '-' strand; any protected mismatch or more than N fails.
__device__ __forceinline__ bool primer_ok(const ScanArgs& a, uint64_t gpos, uint32_t L, uint32_t pl, uint32_t ch,
                                          bool plus, const uint64_t* __restrict__ q0 = nullptr) {
    int mm = 0;
    for (uint32_t c = 0; c < L; c += 32) {
        const int len = (int)min(32u, L - c);
        const uint64_t G = ext2p(a.gpair, gpos + c);  // the interleaved planes: one line, not three
        const uint32_t ex = (uint32_t)(ext1p<2>(a.gpair, gpos + c) >> 32);
        const uint32_t wl = a.I && ex ? (uint32_t)(ext1p<3>(a.gpair, gpos + c) >> 32) : 0u;
        // chunk 0's planes from the record's pair line (q0) when given
        const uint64_t* P = c == 0 && q0 ? q0 : a.planes + (uint64_t)(pl + (c >> 5)) * 4;
        if (!chunk_ok(a, G, ex, P[0], P[1], P[2], P[3], gpos + c, ch + c, len, c, L, plus, mm, wl)) return false;
    }
    return true;
}

// Lower bound on primer-1 mismatches from the fingerprint, over the first min(l1, 32)
// bases of the genome window G (exception bits ex, bit 31-i): plain primer positions
// whose genome base differs, plus "never" positions.  A genome exception base is
// counted only where it certainly mismatches: at a plain position in literal mode
// (I=0: an exception character never equals A/C/G/T); with I=1 it may match and is
// skipped.  Every counted position is a real mismatch of engine.py:599-642, so a
// rejection here is exact.
__device__ __forceinline__ bool fp_reject(const ScanArgs& a, uint64_t G, uint32_t ex, uint32_t l1, uint64_t code,
                                          uint64_t pmask, bool& exact) {
    const int len = (int)min(l1, 32u);
    const uint64_t inside = sp_lt(len);
    const uint64_t x = G ^ code;
    const uint64_t plain = pmask & kEven;
    // the bound is the exact mismatch count when every position was decidable: primer
    // within 32 bases, each base plain or never, no genome exception base
    exact = l1 <= 32u && ex == 0 && (inside & ~((pmask | (pmask >> 1)) & kEven)) == 0;
    uint64_t d = (((x | (x >> 1)) & plain) | ((pmask >> 1) & kEven)) & inside;
    if (ex) {
        const uint64_t es = spread32(ex) & inside;
        d &= ~es;
        if (!a.I) d |= es & plain;
    }
    const int64_t a0 = (int64_t)l1 - a.X;  // '+' strand: positions >= l1 - X are protected
    const uint64_t prot = inside & ~sp_lt((int)smax64(smin64(a0, 32), 0));
    if (d & prot) return true;
    return __popcll(d) > a.N;
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}

// Per-wave hit staging (pair kernel): hits collect in LDS and leave in batches of up
// to 127 with one atomic reservation -- a returning atomic on one global counter
// sustains only ~88 per microsecond (MI355X_MICROARCH.md, dequeue), far below the hit rate.
struct HitStage {
    uint64_t hi[128];
    uint64_t lo[128];
    uint32_t n;
};

// The block's hit-list region (kHitBase): one per XCD group of pair blocks.
__device__ __forceinline__ uint32_t hit_region() { return blockIdx.x & (uint32_t)(kHitRegions - 1); }

// The stage's hits at slots off, off + 1, ... of the block's hit-list region: the raw
// (hi, lo) pair and, for the fused device sort, the packed order key and its bucket count.
// Wave-uniform (the bucket runs ballot).
__device__ __forceinline__ void write_hits(const ScanArgs& a, const HitStage& S, uint64_t off, int lane) {
    const uint64_t r0 = (uint64_t)hit_region() * a.cap_r;
    for (uint32_t b0 = 0; b0 < S.n; b0 += 64) {
        const uint32_t i = b0 + (uint32_t)lane;
        const bool on = i < S.n && off + i < a.cap_r;
        uint32_t bk = 0xFFFFFFFFu;
        uint64_t key = 0;
        if (on) {
            const uint64_t hi = S.hi[i], lo = S.lo[i];
            a.hit_hi[r0 + off + i] = hi;
            a.hit_lo[r0 + off + i] = lo;
            if (a.sort_cnt) {
                key = (hi << a.sort_low_bits) | ((lo >> 32) << a.sort_try_bits) | (lo & 0xFFFFFFFFull);
                a.sort_keys[r0 + off + i] = key;
                bk = (uint32_t)(key >> a.sort_shift);
            }
        }
        if (a.sort_cnt) {
            uint32_t head, len;
            bucket_runs(bk, on, lane, head, len);
            if (a.sort_slots) {  // order mode 0: the run's place in its bucket slot, one returning atomic
                uint32_t at = 0;
                if (on && head == (uint32_t)lane) at = atomicAdd(&a.sort_cnt[bk], len);
                at = (uint32_t)__shfl((int)at, (int)(head & 63u), 64) + ((uint32_t)lane - head);
                if (on && at < a.slot_cap) a.sort_slots[(uint64_t)bk * a.slot_cap + at] = key;
            } else if (on && head == (uint32_t)lane) {
                atomicAdd(&a.sort_cnt[bk], len);
            }
        }
    }
}

__device__ __forceinline__ void stage_flush(const ScanArgs& a, HitStage& S, int lane) {
    const uint32_t cnt = S.n;
    if (!cnt) return;
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(&a.counters[kHitBase + hit_region() * kStatStride], (unsigned long long)cnt);
    base = (unsigned long long)__shfl((long long)base, 0, 64);
    write_hits(a, S, base, lane);
    wave_sync_lds();
    if (lane == 0) S.n = 0;
    wave_sync_lds();
}

// One block of tries: the lanes whose try hit append (order key: k, record rank, try
// rank) to the wave's stage, which leaves once it holds 64 or more.
__device__ __forceinline__ void stage_try_hit(const ScanArgs& a, HitStage& S, int lane, bool hit, uint64_t jgk,
                                              uint32_t jrk, int d) {
    const uint64_t m = __ballot(hit);
    if (!m) return;
    const uint32_t at = S.n;
    if (hit) {
        const uint32_t idx = at + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        S.hi[idx] = jgk;
        S.lo[idx] = ((uint64_t)jrk << 32) | try_rank(d);
    }
    wave_sync_lds();
    if (lane == 0) S.n = at + (uint32_t)__popcll(m);
    wave_sync_lds();
    if (S.n >= 64) stage_flush(a, S, lane);
}

// Pair-check staging per survivor: kPW 2-bit words, kPE exception words (I = 0) or 'N'
// words (I = 1) and the four primer-2 accept planes, [slot][survivor] in the wave's LDS.
// At M=50 and primers of <= 25 bases every survivor fits (the tries span <= 125 bases).
constexpr int kPW = 6, kPE = 4, kPSlots = kPW + kPE + 4;
static_assert(kPW + 1 < 2 * kPE, "staged 2-bit words lie in the staged 64-base blocks");
static_assert(MP_PBATCH <= 64, "pair-check batch is one survivor per lane");

__device__ __forceinline__ uint32_t rl32(uint32_t v, int j) { return (uint32_t)__builtin_amdgcn_readlane((int)v, j); }
__device__ __forceinline__ uint64_t rl64(uint64_t v, int j) {
    return ((uint64_t)rl32((uint32_t)(v >> 32), j) << 32) | rl32((uint32_t)v, j);
}

// _match_sts (engine.py:507-597) for the fingerprint survivors of a wave, 64 at a time.
// Phase 1, lane per survivor: the survivor, its sequence and record, the product-size
// bounds e/lo/hi and (unless the fingerprint was exact) the primer-1 compare, all in
// parallel.  Phase 2, one survivor at a time (its values broadcast from its lane): the
// genome bases every try reads, [P0, last], are staged in registers as 2-bit words and
// exception words (one each per lane, one load round trip for ~2000 bases; longer
// stretches restage per block of tries and primer chunk), each lane takes the window of
// one amplicon-end offset d by shuffles and compares primer 2 -- by one 2-bit XOR and
// popcount when primer 2 is plain (one base per position) and no exception base is in
// the windows, else through the accept planes.  The reference's try order 0, -1, +1,
// ... is restored by the device sort through try_rank(d).
// The lane's survivor v (kEmptySurv: none); batch = the wave's survivors (lanes 0..batch-1),
// which sets how the lane-parallel tries split over lane groups.
constexpr uint4 kEmptySurv = {0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u};
__device__ void pair_check_lanes(const ScanArgs& a, uint4 v, uint32_t batch, int lane, HitStage& S,
                                 uint64_t* __restrict__ pst) {
    bool keep = !(v.x == 0xFFFFFFFFu && v.y == 0xFFFFFFFFu);
    const uint64_t gk = (uint64_t)v.x | ((uint64_t)v.y << 32);
    const uint32_t rec = v.z & 0x7FFFFFFFu;
    uint64_t sbase = 0;
    uint32_t n = 0;
    DevRec r{};
    uint32_t rk = 0;
    const PairRec* pr = a.prec + rec;  // one 128-B line: the record, its rank, both primers' chunk-0 planes
    if (keep) {
        sbase = a.seq_base[v.w];
        n = (uint32_t)a.seq_len[v.w];
        r = pr->d;
        rk = pr->rank;
    }
    const uint32_t k = (uint32_t)(gk - sbase);
    keep = keep && n - k - r.l1 >= r.l2;
    uint32_t e = 0;
    int hi = 0;
    if (r.size > n - k) {
        e = n - k;
    } else {
        e = r.size;
        hi = (int)min<uint32_t>((uint32_t)a.M, n - k - e);
    }
    const int lo = (int)smax64(0, smin64(a.M, (int64_t)e - r.l1 - r.l2));
    // Staged survivors: primer 2 within 32 bases and every try inside kPW 2-bit words and
    // kPE exception words.  The lane loads its survivor's words and primer-2 planes now,
    // in parallel with the primer-1 compare, into the wave's LDS stage ([slot][lane], so
    // the writes are conflict-free), and phase 2 reads them from LDS instead of issuing
    // one dependent global round trip per survivor.
    bool fast = false, clean = false;
    const uint64_t P0l = gk + e - r.l2 - (uint32_t)lo;
    {
        const uint64_t lastl = P0l + (uint64_t)(lo + hi) + r.l2 - 1;
        const uint64_t w0 = P0l >> 5, e0 = P0l >> 6;
        const uint64_t wl = (lastl >> 5) + 1, el = (lastl >> 6) + 1;  // last words any try reads
        fast = keep && r.l2 <= 32u && wl - w0 < (uint64_t)kPW && el - e0 < (uint64_t)kPE;
        if (fast) {
            // exception bits of the stretch [P0l, lastl] (at most 4 words of 64 bases).  Under
            // I = 1 an 'N' matches every primer base with an IUPAC meaning (char_match,
            // engine.py:613-631) -- exactly the positions with an accept-plane bit -- so the
            // lane-parallel tries take 'N' as a wildcard from the staged 'N' words, and only
            // the other exception characters make a stretch unclean
            uint64_t ew[kPE];
            // whole 32-B gpair blocks e0..el, two 16-B loads each: 2-bit words 2b, 2b+1, then the
            // exception and 'N' words (word w0 is in block e0).  Round 5: one 16-B load per two
            // words instead of one 8-B load per word (up to 14 loads per lane -> 8): c4 pair
            // 0.387 -> 0.342 ms, c3 0.079 -> 0.074 ms (`gpurun_out/pblk_*`).  Block el holds
            // no stretch base, only (when wl is its first word) a try's last 2-bit word and
            // its 'N' bits: loaded only then, c4 pair 0.342 -> 0.336 ms (`gpurun_out/pv_*`)
            uint64_t g2w[2 * kPE];
            const ulonglong2* gq = reinterpret_cast<const ulonglong2*>(a.gpair);
#pragma unroll
            for (int t = 0; t < kPE; ++t) {
                ulonglong2 q0 = make_ulonglong2(0ull, 0ull), q1 = q0;
                if (e0 + t <= (wl >> 1)) {  // up to the block of the last 2-bit word a try reads
                    q0 = gq[2 * (e0 + t)];
                    q1 = gq[2 * (e0 + t) + 1];
                }
                g2w[2 * t] = q0.x;
                g2w[2 * t + 1] = q0.y;
                ew[t] = q1.x;
                if (a.I) {
                    ew[t] &= ~q1.y;
                    pst[(kPW + t) * MP_PBATCH + lane] = q1.y;
                } else {
                    pst[(kPW + t) * MP_PBATCH + lane] = ew[t];
                }
            }
            const bool odd = (w0 & 1u) != 0u;
#pragma unroll
            for (int t = 0; t < kPW; ++t) pst[t * MP_PBATCH + lane] = w0 + t <= wl ? (odd ? g2w[t + 1] : g2w[t]) : 0ull;
            const uint32_t f0 = (uint32_t)(P0l & 63), f1 = (uint32_t)(lastl - (e0 << 6));  // stretch bits in word order
            uint64_t any = 0;
#pragma unroll
            for (int t = 0; t < kPE; ++t) {
                const uint32_t b0 = 64u * (uint32_t)t, b1 = b0 + 63u;  // bases of word t, relative to e0 << 6
                const uint32_t s0 = f0 > b0 ? f0 - b0 : 0u, s1 = f1 < b1 ? f1 - b0 : 63u;
                if (f0 <= b1 && f1 >= b0)
                    any |= ew[t] & ((~0ull >> s0) & ~(s1 >= 63u ? 0ull : (~0ull >> (s1 + 1u))));
            }
            clean = any == 0;
            const uint64_t* pp = pr->p2q;  // primer 2 <= 32 bases here: its planes are chunk 0
#pragma unroll
            for (int t = 0; t < 4; ++t) pst[(kPW + kPE + t) * MP_PBATCH + lane] = pp[t];
        }
    }
    wave_sync_lds();
    if (keep && !(v.z >> 31)) keep = primer_ok(a, gk, r.l1, r.p1_pl, r.p1_ch, true, pr->p1q);
    // Lane-parallel tries: a survivor whose stretch holds no exception base takes its tries
    // in its own lane -- a 32-base window slid one base per try through the staged words,
    // primer 2 compared by XOR/popcount (plain) or the accept planes -- one wave-wide pass
    // per try offset instead of one per survivor.
    const bool lp = keep && fast && clean;
    if (__any(lp)) {
        // A batch of B <= 32 survivors leaves 64 - B lanes idle, so the tries are split:
        // the wave is 64 / Bp groups of Bp lanes (Bp = B rounded up to a power of two),
        // lane L takes survivor L % Bp and the L / Bp-th slice of its tries.  The survivor's
        // values come from its own lane by shuffles; its staged words and planes are its LDS
        // column.  c2 (8 survivors per wave): the try loop from 101 passes to 13.
        uint32_t Bp = 1;
        while (Bp < batch) Bp <<= 1;
        const int s = (int)((uint32_t)lane & (Bp - 1u));
        const uint32_t grp = (uint32_t)lane / Bp, ngrp = 64u / Bp;
        const bool slp = __shfl((int)lp, s, 64) != 0;
        const uint32_t sl1 = (uint32_t)__shfl((int)r.l1, s, 64), sl2 = (uint32_t)__shfl((int)r.l2, s, 64);
        const int slo = __shfl(lo, s, 64), shi = __shfl(hi, s, 64);
        const uint32_t se = (uint32_t)__shfl((int)e, s, 64);
        const uint64_t sP0 = shfl64(P0l, s), sgk = shfl64(gk, s);
        const uint32_t srk = (uint32_t)__shfl((int)rk, s, 64);
        const uint64_t* sj = pst + s;
        const uint64_t Q0 = sj[(kPW + kPE) * MP_PBATCH], Q1 = sj[(kPW + kPE + 1) * MP_PBATCH];
        const uint64_t Q2 = sj[(kPW + kPE + 2) * MP_PBATCH], Q3 = sj[(kPW + kPE + 3) * MP_PBATCH];
        // per-base 32-bit masks (bit 31-i = primer-2 position i): the accept planes, the
        // positions compared, the protected ones ('-' strand: positions < X)
        const uint32_t q0 = compress_even(Q0), q1 = compress_even(Q1), q2 = compress_even(Q2),
                       q3 = compress_even(Q3);
        const uint32_t in32 = sl2 >= 32u ? ~0u : ~(~0u >> sl2);
        const uint32_t px = (uint32_t)min(a.X, (int)sl2);
        const uint32_t prot32 = px >= 32u ? ~0u : ~(~0u >> px);
        const uint32_t anyq = (q0 | q1 | q2 | q3) & in32;
        // try t (d = t - lo) is in bounds for t in [ta, lo + hi] (engine.py:548-560: a
        // non-positive offset needs the product to end past primer 1, and the window inside
        // the sequence, which hi already guarantees)
        const int64_t ta = smin64((int64_t)slo + 1, smax64(0, (int64_t)sl1 + sl2 + slo - (int64_t)se));
        const int32_t tb = slp ? slo + shi : -1;
        // this lane's slice [t0, t0 + chunk) of tries; chunk from the batch's largest count
        int32_t tmax = tb + 1;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tmax = max(tmax, __shfl_xor(tmax, o, 64));
        const int32_t chunk = (tmax + (int32_t)ngrp - 1) / (int32_t)ngrp;
        const int32_t t0 = (int32_t)grp * chunk;
        // The window of try t0 + k is bases u0 + k .. u0 + k + 31 of the staged stretch, held as
        // three bit planes -- the low and high bit of each base's 2-bit code and (I = 1) its
        // 'N' bit -- in 64-bit shift registers whose top 32 bits are the window: one shift per
        // plane per try, 32 new bases every 32 tries.  Compared through the planes with three
        // bit selects (match = hi ? (lo ? q3 : q2) : (lo ? q1 : q0)), where the 2-bit form
        // spent ~70 VALU per try (c4's pair kernel was VALU-bound, 80% of its issue cycles).
        const uint32_t u0 = (uint32_t)(sP0 & 31) + (uint32_t)t0;  // staged-word base of try t0
        const uint32_t a5 = u0 & 31u;
        const int w0 = min((int)(u0 >> 5), kPW - 2);
        // 'N' words are 64-base words from (P0 >> 6) << 6: 32-base word w of the 2-bit grid is
        // half wd of them, wd = w + ((P0 >> 5) & 1)
        const int wdel = (int)((sP0 >> 5) & 1u);
        auto word32 = [&](int w, uint32_t& lo_, uint32_t& hi_, uint32_t& wi_) {
            const uint64_t x = sj[min(w, kPW - 1) * MP_PBATCH];
            lo_ = compress_even(x);
            hi_ = compress_even(x >> 1);
            wi_ = 0u;
            if (a.I) {
                const int wd = min(w + wdel, 2 * kPE - 1);
                const uint64_t y = sj[(kPW + (wd >> 1)) * MP_PBATCH];
                wi_ = (wd & 1) ? (uint32_t)y : (uint32_t)(y >> 32);
            }
        };
        // 32 bases starting a5 into word w: the refill value of each plane
        auto fill = [&](int w, uint32_t& lo_, uint32_t& hi_, uint32_t& wi_) {
            uint32_t l0, h0, n0, l1, h1, n1;
            word32(w, l0, h0, n0);
            word32(w + 1, l1, h1, n1);
            lo_ = a5 ? (l0 << a5) | (l1 >> (32u - a5)) : l0;
            hi_ = a5 ? (h0 << a5) | (h1 >> (32u - a5)) : h0;
            wi_ = a5 ? (n0 << a5) | (n1 >> (32u - a5)) : n0;
        };
        uint64_t SL, SH, SW;
        {
            uint32_t l0, h0, n0, l1, h1, n1;
            fill(w0, l0, h0, n0);
            fill(w0 + 1, l1, h1, n1);
            SL = ((uint64_t)l0 << 32) | l1;
            SH = ((uint64_t)h0 << 32) | h1;
            SW = ((uint64_t)n0 << 32) | n1;
        }
        int nw = w0 + 2;
        for (int32_t k = 0; k < chunk; ++k) {  // wave-uniform trip count
            const int32_t t = t0 + k;
            const uint32_t glo = (uint32_t)(SL >> 32), ghi = (uint32_t)(SH >> 32);
            const uint32_t m01 = (glo & q1) | (~glo & q0), m23 = (glo & q3) | (~glo & q2);
            uint32_t match = (ghi & m23) | (~ghi & m01);
            if (a.I) match |= (uint32_t)(SW >> 32) & anyq;  // 'N': every base with an IUPAC meaning
            const uint32_t mm = ~match & in32;
            const bool hit = t >= ta && t <= tb && !(mm & prot32) && __popc(mm) <= a.N;
            stage_try_hit(a, S, lane, hit, sgk, srk, t - slo);
            SL <<= 1;
            SH <<= 1;
            SW <<= 1;
            if ((k & 31) == 31) {  // the next 32 bases
                uint32_t l, h, n;
                fill(nw, l, h, n);
                SL |= l;
                SH |= h;
                SW |= n;
                ++nw;
            }
        }
    }
    uint64_t todo = __ballot(keep && !lp);
    while (todo) {
        const int j = (int)__builtin_ctzll(todo);
        todo &= todo - 1;
        const uint64_t jgk = rl64(gk, j);
        const uint32_t jn = rl32(n, j), jk = rl32(k, j), je = rl32(e, j);
        const uint32_t jl1 = rl32(r.l1, j), jl2 = rl32(r.l2, j), jpl = rl32(r.p2_pl, j), jch = rl32(r.p2_ch, j);
        const uint32_t jrk = rl32(rk, j);
        const int jlo = (int)rl32((uint32_t)lo, j), jhi = (int)rl32((uint32_t)hi, j);
        const int ntry = jlo + jhi + 1;
        const uint64_t P0 = jgk + je - jl2 - (uint32_t)jlo;            // global start of the first try
        if (rl32((uint32_t)fast, j) && !a.I) {  // I = 1: the staged words are 'N' bits, not exceptions
            const uint64_t* sj = pst + j;
            const uint64_t Q0 = sj[(kPW + kPE) * MP_PBATCH], Q1 = sj[(kPW + kPE + 1) * MP_PBATCH];
            const uint64_t Q2 = sj[(kPW + kPE + 2) * MP_PBATCH], Q3 = sj[(kPW + kPE + 3) * MP_PBATCH];
            const uint64_t in2 = sp_lt((int)jl2);
            const uint64_t two = (Q0 & Q1) | (Q0 & Q2) | (Q0 & Q3) | (Q1 & Q2) | (Q1 & Q3) | (Q2 & Q3);
            const bool plain2 = two == 0 && ((Q0 | Q1 | Q2 | Q3) & in2) == in2;
            const uint64_t code2 = ((Q1 | Q3) & kEven) | (((Q2 | Q3) & kEven) << 1);
            const uint64_t prot2 = sp_lt(min(a.X, (int)jl2));  // '-' strand: positions < X
            const uint32_t a5 = (uint32_t)(P0 & 31), a6 = (uint32_t)(P0 & 63);
            for (int b = 0; b < ntry; b += 64) {
                const int d = -jlo + b + lane;
                const int64_t p2 = (int64_t)jk + je - jl2 + d;
                const bool inb = b + lane < ntry && !(d <= 0 && (int64_t)jk + jl1 > p2) && p2 + jl2 <= (int64_t)jn;
                const uint64_t q = P0 + (uint64_t)(b + lane);
                // lanes past the last try clamp their word index (their result is unused)
                const uint32_t rw = a5 + (uint32_t)(b + lane), re = a6 + (uint32_t)(b + lane);
                const uint32_t wi = min(rw >> 5, (uint32_t)kPW - 2), ei = min(re >> 6, (uint32_t)kPE - 2);
                const int rs = (int)(rw & 31), es = (int)(re & 63);
                const uint64_t x0 = sj[wi * MP_PBATCH], x1 = sj[(wi + 1) * MP_PBATCH];
                const uint64_t y0 = sj[(kPW + ei) * MP_PBATCH], y1 = sj[(kPW + ei + 1) * MP_PBATCH];
                const uint64_t G = rs ? (x0 << (2 * rs)) | (x1 >> (64 - 2 * rs)) : x0;
                const uint32_t ex = (uint32_t)((es ? (y0 << es) | (y1 >> (64 - es)) : y0) >> 32);
                const int len = (int)jl2;
                const uint32_t exl = len >= 32 ? ex : ex & ~(0xFFFFFFFFu >> len);
                bool ok = true;
                int mm = 0;
                // plain primer 2: one XOR/popcount; a genome exception base is a certain
                // mismatch under the literal rule (I=0), else the lanes need the lookup
                if (plain2 && (!a.I || __all(!inb || exl == 0))) {
                    const uint64_t x = G ^ code2;
                    const uint64_t dm = ((x | (x >> 1)) | (exl ? spread32(exl) : 0ull)) & in2;
                    ok = !(dm & prot2) && __popcll(dm) <= a.N;
                } else if (inb) {
                    ok = chunk_ok(a, G, ex, Q0, Q1, Q2, Q3, q, jch, len, 0, jl2, false, mm);
                }
                stage_try_hit(a, S, lane, inb && ok, jgk, jrk, d);
            }
            continue;
        }
        const uint64_t last = P0 + (uint64_t)(ntry - 1) + jl2 - 1;     // last base any try reads
        const uint64_t wlast = (last >> 5) + 1, elast = (last >> 6) + 1;
        uint64_t sw = ~0ull, se = ~0ull;  // staged word bases (wave-uniform)
        uint64_t gw = 0, ew = 0;
        uint32_t pchunk = ~0u;
        uint64_t Q0 = 0, Q1 = 0, Q2 = 0, Q3 = 0;
        // plain primer 2 within 32 bases: its 2-bit code and protected positions (uniform)
        bool plain2 = false;
        uint64_t code2 = 0, in2 = 0, prot2 = 0;
        for (int b = 0; b < ntry; b += 64) {
            const int d = -jlo + b + lane;
            const int64_t p2 = (int64_t)jk + je - jl2 + d;
            const bool inb = b + lane < ntry && !(d <= 0 && (int64_t)jk + jl1 > p2) && p2 + jl2 <= (int64_t)jn;
            const uint64_t gp = P0 + (uint64_t)(b + lane);
            bool ok = true;
            int mm = 0;
            for (uint32_t c = 0; c < jl2; c += 32) {
                const uint64_t lo_pos = P0 + (uint64_t)b + c;  // windows of this (block, chunk)
                const uint64_t hi_pos = lo_pos + 63 + 31;
                if ((lo_pos >> 5) < sw || (hi_pos >> 5) + 1 > sw + 63 || (lo_pos >> 6) < se ||
                    (hi_pos >> 6) + 1 > se + 63) {
                    sw = lo_pos >> 5;
                    se = lo_pos >> 6;
                    gw = sw + (uint64_t)lane <= wlast ? a.g2[sw + (uint64_t)lane] : 0ull;
                    ew = se + (uint64_t)lane <= elast ? a.gexc[se + (uint64_t)lane] : 0ull;
                }
                if ((c >> 5) != pchunk) {
                    pchunk = c >> 5;
                    const uint64_t* pp = a.planes + (uint64_t)(jpl + pchunk) * 4;
                    Q0 = pp[0]; Q1 = pp[1]; Q2 = pp[2]; Q3 = pp[3];
                    if (jl2 <= 32u) {
                        in2 = sp_lt((int)jl2);
                        const uint64_t two = (Q0 & Q1) | (Q0 & Q2) | (Q0 & Q3) | (Q1 & Q2) | (Q1 & Q3) | (Q2 & Q3);
                        plain2 = two == 0 && ((Q0 | Q1 | Q2 | Q3) & in2) == in2;
                        code2 = ((Q1 | Q3) & kEven) | (((Q2 | Q3) & kEven) << 1);
                        prot2 = sp_lt(min(a.X, (int)jl2));  // '-' strand: positions < X
                    }
                }
                const uint64_t q = gp + c;
                const int rw = (int)((q >> 5) - sw), rs = (int)(q & 31);
                const int re = (int)((q >> 6) - se), es = (int)(q & 63);
                const uint64_t x0 = shfl64(gw, rw & 63), x1 = shfl64(gw, (rw + 1) & 63);
                const uint64_t y0 = shfl64(ew, re & 63), y1 = shfl64(ew, (re + 1) & 63);
                const uint64_t G = rs ? (x0 << (2 * rs)) | (x1 >> (64 - 2 * rs)) : x0;
                const uint32_t ex = (uint32_t)((es ? (y0 << es) | (y1 >> (64 - es)) : y0) >> 32);
                const int len = (int)min(32u, jl2 - c);
                const uint32_t exl = len >= 32 ? ex : ex & ~(0xFFFFFFFFu >> len);
                // plain primer 2: one XOR/popcount; a genome exception base is a certain
                // mismatch under the literal rule (I=0), else the lanes need the lookup
                if (plain2 && (!a.I || __all(!inb || exl == 0))) {
                    const uint64_t x = G ^ code2;
                    const uint64_t dm = ((x | (x >> 1)) | (exl ? spread32(exl) : 0ull)) & in2;
                    ok = !(dm & prot2) && __popcll(dm) <= a.N;
                } else if (inb && ok) {
                    ok = chunk_ok(a, G, ex, Q0, Q1, Q2, Q3, q, jch + c, len, c, jl2, false, mm);
                }
            }
            stage_try_hit(a, S, lane, inb && ok, jgk, jrk, d);
        }
    }
}

// Inclusive wave64 prefix sum.  DPP form: row_shr 1/2/4/8 within each 16-lane row, then
// row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) -- six VALU ops with no LDS round
// trip, where the shuffle form is six dependent ds_bpermute waits.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
    (void)lane;
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

__device__ __forceinline__ void wave_sync() { wave_sync_lds(); }

// Per-wave seed queue: the super-step offsets of its seed hits, in window order.  The
// LDS left beside the 128 KiB prefilter (160 KiB per CU) holds 1008 per wave; a denser
// super-step is drained in rounds.
constexpr uint32_t kSeedQ = 1008;
// kMode 1 with 1: the level-2 probe already read each seed's rank word, so the queue
// carries the key rank beside the offset (6 B per seed) and the drain skips the rank word.
constexpr uint32_t kSeedQR = 340;
struct WaveLds {
    union {
        uint16_t q[kSeedQ];
        struct {
            uint16_t q[kSeedQR];
            uint32_t r[kSeedQR];
        } rq;
    };
};
static_assert(sizeof(WaveLds) <= 2048, "per-wave LDS beside the 128 KiB prefilter");
#ifndef MP_L2SLOTS
#define MP_L2SLOTS 12
#endif
// level 2 through a wave-wide LDS list of the positives (full-lane probes) instead of
// per-lane slots


// The current super-step as the wave holds it: lane L owns bases [base + 32L,
// base + 32L + 64) as two 2-bit words and one ambiguity word.
// A lane's 32 (+32) ambiguity bits from the two plane words around its first base: sh = 32
// when that base is in the second half of the first word.
__device__ __forceinline__ uint64_t inv_join(uint64_t v0, uint64_t v1, uint32_t sh) {
    return (v0 << sh) | ((v1 >> (63 - sh)) >> 1);
}

struct SuperRegs {
    uint64_t w0, w1, iv;
    uint32_t base;
    uint32_t seq;
    bool owned;   // every amplicon start k this super-step can produce is in [g_lo, g_hi)
};

// 32 bases (2-bit, base p on top) and their exception bits (bit 31-i) starting at
// sequence position p, with p - base in [0, kSuper): from the owning lane's registers.
// All lanes must call (shuffles); `p` of inactive lanes may be anything in range.
__device__ __forceinline__ void window_from_regs(const ScanArgs& a, const SuperRegs& R, uint64_t sbase,
                                                 uint32_t p, bool in_regs, uint64_t& G, uint32_t& ex) {
    const uint32_t off = in_regs ? p - R.base : 0u;
    const int src = (int)(off >> 5);
    const uint32_t r = off & 31u;
    const uint64_t x0 = shfl64(R.w0, src), x1 = shfl64(R.w1, src), v = shfl64(R.iv, src);
    if (in_regs) {
        G = r ? (x0 << (2 * r)) | (x1 >> (64 - 2 * r)) : x0;
        ex = (uint32_t)((v << r) >> 32);
    } else {
        G = ext2(a.g2, sbase + p);
        ex = (uint32_t)(ext1(a.ginv, sbase + p) >> 32);
    }
    if (a.has_u) ex = (uint32_t)(ext1(a.gexc, sbase + p) >> 32);
}

// One (seed position, record) candidate: the bounds of engine.py:486-489, the
// owned-range test and the fingerprint filter.  True = survivor (k returned).
// All lanes must call (shuffles); `act` marks lanes that hold a candidate.
__device__ __forceinline__ bool candidate(const ScanArgs& a, const SuperRegs& R, uint64_t sbase, uint32_t n,
                                          bool act, uint32_t pos, const Entry& e, uint32_t& ncand, uint32_t& k_out,
                                          uint64_t Gpos, uint32_t expos, bool reuse, bool& exact) {
    const uint32_t k = pos - e.hash_off;
    act = act && pos >= e.hash_off && (uint64_t)k + e.l1 <= n;
    if (!R.owned)
        act = act && sbase + k >= a.g_lo && sbase + k < a.g_hi;
    uint64_t G = Gpos;
    uint32_t ex = expos;
    if (!reuse || !__all(!act || e.hash_off == 0)) {  // some seed is not at the primer start
        const bool in_regs = k >= R.base && k - R.base < kSuper;
        window_from_regs(a, R, sbase, act ? k : R.base, !act || in_regs, G, ex);
    }
    // seed at the primer start and a plain primer: bases [0, W) matched exactly, so only
    // the <= 16 bases after the seed can mismatch -- one 32-bit XOR/popcount
    const uint32_t W = (uint32_t)a.W;
    const uint32_t L = (uint32_t)e.l1 - W;
    const uint32_t inm = L >= 16u ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> (2u * L));
    // (no exception base anywhere in the primer: a genome U in the seed is a literal
    // mismatch against the primer's T although their 2-bit codes agree)
    const bool fast = e.hash_off == 0 && e.l1 >= W && L <= 16u && (e.l1 >= 32u ? ex : ex & ~(0xFFFFFFFFu >> e.l1)) == 0 &&
                      e.pmask == sp_lt((int)e.l1);
    if (__all(!act || fast)) {
        if (!act) return false;
        ++ncand;
        const uint32_t g = (uint32_t)((G << (2u * W)) >> 32), c = (uint32_t)((e.code << (2u * W)) >> 32);
        const uint32_t x = g ^ c;
        const uint32_t d = (x | (x >> 1)) & 0x55555555u & inm;
        const int32_t p0 = (int32_t)L - a.X;  // protected: relative positions >= L - X
        const uint32_t prot = p0 <= 0 ? inm : (p0 >= 16 ? 0u : inm & (0xFFFFFFFFu >> (2 * p0)));
        exact = true;
        if ((d & prot) || __popc(d) > a.N) return false;
        k_out = k;
        return true;
    }
    if (!act) return false;
    ++ncand;
    if (fp_reject(a, G, ex, e.l1, e.code, e.pmask, exact)) return false;
    k_out = k;
    return true;
}

// Chunked output lists of a wave (fingerprint survivors, bucket-tail references):
// slots are reserved 64 at a time (one atomic per chunk); unused tail slots of a wave's
// last chunk are marked empty.
struct SurvChunk {
    uint64_t base;   // first slot of the current chunk
    uint32_t used;   // slots of it already written (kChunkNone: no chunk yet)
    uint32_t total;  // entries of this wave (statistics)
};
constexpr uint32_t kChunkNone = 0xFFFFFFFFu;
// Key references per reservation from the wide key groups (c4 leaves ~16M, where 64-slot
// reservations, ~94 per microsecond, saturated the list counter; c3's 5.5M keep 64: 256 was
// slower there, more empty slots for tail_kernel)
#ifndef MP_REF_CHUNK
#define MP_REF_CHUNK 256
#endif
constexpr uint32_t kRefChunk = MP_REF_CHUNK;
#ifndef MP_REF_CHUNK1
#define MP_REF_CHUNK1 64
#endif
constexpr uint32_t kRefChunk1 = MP_REF_CHUNK1;  // the 8-B key groups' references (c3: 5.5M)
constexpr uint32_t kStaticRefs = 64;  // bucket-tail slots each scan wave owns before its first reservation

// kChunk: slots per reservation (a multiple of 64).  Every reservation is one returning atomic
// on one address, and same-address atomics serialise at ~88 per microsecond: lists written at
// more than ~5M entries per millisecond of scan take larger chunks (kRefChunk).
// off0: the list's statically reserved slots (the counter counts from there).
template <int kStride = 1, uint32_t kChunk = 64>
__device__ __forceinline__ void append_chunked(unsigned long long* counter, uint4* buf, uint64_t cap, bool on,
                                               const uint4& v, int lane, SurvChunk& C, const uint4& v2 = uint4{},
                                               uint64_t off0 = 0) {
    static_assert(kChunk % 64u == 0u, "whole waves of slots");
    const uint64_t m = __ballot(on);
    if (!m) return;
    const uint32_t cnt = (uint32_t)__popcll(m);
    C.total += cnt;
    const uint32_t avail = C.used >= kChunk ? 0u : kChunk - C.used;
    uint64_t nbase = C.base;
    if (cnt > avail) {
        unsigned long long b = 0;
        if (lane == 0) b = atomicAdd(counter, (unsigned long long)kChunk);
        nbase = off0 + shfl64((uint64_t)b, 0);
    }
    if (on) {
        const uint32_t r = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        const uint64_t idx = r < avail ? C.base + C.used + r : nbase + (r - avail);
        if (idx < cap) {
            buf[idx * kStride] = v;
            if constexpr (kStride == 2) buf[idx * 2 + 1] = v2;
        }
    }
    if (cnt > avail) {
        C.base = nbase;
        C.used = cnt - avail;
    } else {
        C.used += cnt;
    }
}

__device__ __forceinline__ void flush_survivors(const ScanArgs& a, const SuperRegs& R, uint64_t sbase, bool surv,
                                                uint32_t k, uint32_t rec, bool exact, int lane, SurvChunk& C) {
    const uint64_t gk = sbase + k;
    append_chunked(&a.counters[2], a.surv, a.surv_cap, surv,
                   make_uint4((uint32_t)gk, (uint32_t)(gk >> 32), rec | (exact ? 0x80000000u : 0u), R.seq), lane, C);
}

template <int kStride = 1, uint32_t kChunk = 64>
__device__ __forceinline__ void close_chunked(uint4* buf, uint64_t cap, int lane, const SurvChunk& C) {
    if (C.used >= kChunk) return;
    for (uint32_t i = C.used + (uint32_t)lane; i < kChunk; i += 64u)  // the chunk's unused slots: empty
        if (C.base + i < cap) buf[(C.base + i) * kStride] = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u);
}

// Entry of an 8-B head (see kHead8Full): the seed key h supplies primer-1 bases [0, W).
__device__ __forceinline__ Entry head8_entry(const uint2 c, uint32_t h, uint32_t W) {
    Entry e;
    const uint32_t L = c.y >> kHead8RecBits;  // l1 - W (kHead8Full clear)
    e.code = ((uint64_t)h << (64 - 2 * W)) | ((uint64_t)c.x << (32 - 2 * W));
    e.rec = c.y & ((1u << kHead8RecBits) - 1u);
    e.hash_off = 0;
    e.l1 = (uint16_t)(W + L);
    e.pmask = sp_lt((int)e.l1);
    e.xstart = 0;
    e.count = 1;
    return e;
}

// Entry of a 16-B head (kHead8Full clear in .w): the seed key h supplies primer-1 bases
// [0, W) (plain), .x bases W..W+15, .y / .z their plain / never bits (bit 30-2j).
__device__ __forceinline__ Entry head16_entry(const uint4 c, uint32_t h, uint32_t W) {
    Entry e;
    const uint32_t L = (c.w >> kHead8RecBits) & 31u;
    e.code = ((uint64_t)h << (64 - 2 * W)) | ((uint64_t)c.x << (32 - 2 * W));
    e.rec = c.w & ((1u << kHead8RecBits) - 1u);
    e.hash_off = 0;
    e.l1 = (uint16_t)(W + L);
    e.pmask = sp_lt((int)W) | ((uint64_t)c.y << (32 - 2 * W)) | ((uint64_t)c.z << (33 - 2 * W));
    e.xstart = 0;
    e.count = 1;
    return e;
}

// The plain bits of an 8-B IUPAC head (bits 29..18 of .y, base W first) spread to the
// low bits of their 2-bit slots in a window of bases W..W+15 (base W at bit 30).
__device__ __forceinline__ uint32_t head12_plain(uint32_t y) {
    uint32_t v = (y >> kHead12RecBits) & 0xFFFu;
    v = (v | (v << 8)) & 0x00FF00FFu;
    v = (v | (v << 4)) & 0x0F0F0F0Fu;
    v = (v | (v << 2)) & 0x33333333u;
    v = (v | (v << 1)) & 0x55555555u;
    return v << 8;
}

// Entry of an 8-B IUPAC head (kHead8Full clear): the seed key h supplies bases [0, W), the
// head bases W..W+11 and their plain bits; later bases are neither plain nor never (skipped
// by fp_reject, which then reports the survivor not exact).
__device__ __forceinline__ Entry head12_entry(const uint2 c, uint32_t h, uint32_t W) {
    Entry e;
    e.code = ((uint64_t)h << (64 - 2 * W)) | ((uint64_t)(c.x & 0xFFFFFF00u) << (32 - 2 * W));
    e.rec = c.y & ((1u << kHead12RecBits) - 1u);
    e.hash_off = 0;
    e.l1 = (uint16_t)(W + (c.x & 31u));
    e.pmask = sp_lt((int)W) | ((uint64_t)head12_plain(c.y) << (32 - 2 * W));
    e.xstart = 0;
    e.count = 1;
    return e;
}

// Bucket head of seed key h (W <= 13: rank of h in the exact bitmap; above: slot).
template <int kMode>
__device__ __forceinline__ bool bucket_head(const ScanArgs& a, uint32_t h, Entry& e0) {
    if constexpr (kMode != 2) {
        const uint2 rw = a.rk[h >> 5];
        const uint32_t bit = h & 31u;
        if (!((rw.x >> bit) & 1u)) return false;
        e0 = a.dents[rw.y + (uint32_t)__popc(rw.x & ((1u << bit) - 1u))];
        return true;
    } else {
        const uint32_t mask = (1u << a.slot_log2) - 1;
        uint32_t s = table_slot(h, a.slot_log2);
        for (;;) {
            const uint4 head = *reinterpret_cast<const uint4*>(&a.slots[s]);  // key, used
            if (head.y == 0) return false;  // hashed-filter false positive
            if (head.x == h) break;
            s = (s + 1) & mask;
        }
        e0 = a.slots[s].e0;
        return true;
    }
}

// Candidate test of one bucket head per lane, then the bucket tails.  kInline (tables
// whose buckets are mostly multi-record, e.g. W=8 with 100k STS): the wave expands the
// tails itself, 64 candidates per pass, each lane finding its bucket by a shuffle
// search over the inclusive tail-count scan.  Otherwise a bucket with more records
// leaves a reference (seed position, bucket) for tail_kernel.
template <int kMode, bool kInline>
__device__ __forceinline__ void heads_and_tails(const ScanArgs& a, const SuperRegs& R, uint64_t sbase,
                                                uint32_t n, bool have, uint32_t pos, const Entry& e0, uint64_t Gp,
                                                uint32_t exp_, int lane, uint32_t& ncand, SurvChunk& C,
                                                SurvChunk& TC) {
    uint32_t sk = 0;
    bool ex0 = false;
    const bool surv = candidate(a, R, sbase, n, have, pos, e0, ncand, sk, Gp, exp_, true, ex0);
    flush_survivors(a, R, sbase, surv, sk, e0.rec, ex0, lane, C);
    const bool tail = have && e0.count > 1u;
    if (!__any(tail)) return;
    if constexpr (kInline) {
        const uint32_t xc = tail ? e0.count - 1u : 0u;
        const uint32_t incl = wave_incl_scan(xc, lane);
        const uint32_t total = rl32(incl, 63);
        for (uint32_t c0 = 0; c0 < total; c0 += 64) {
            const uint32_t c = c0 + (uint32_t)lane;
            const bool act = c < total;
            uint32_t src = 0;  // number of lanes whose inclusive count is <= c
#pragma unroll
            for (uint32_t step = 32; step; step >>= 1) {
                const uint32_t v = (uint32_t)__shfl((int)incl, (int)(src + step - 1), 64);
                if (v <= c) src += step;
            }
            src = min(src, 63u);
            const uint32_t xpos = (uint32_t)__shfl((int)pos, (int)src, 64);
            const uint32_t xstart = (uint32_t)__shfl((int)e0.xstart, (int)src, 64);
            const uint32_t xpre = (uint32_t)__shfl((int)(incl - xc), (int)src, 64);
            Entry ej{};
            if (act) ej = a.ents[xstart + (c - xpre)];
            bool ex2 = false;
            const bool s2 = candidate(a, R, sbase, n, act, xpos, ej, ncand, sk, 0, 0, false, ex2);
            flush_survivors(a, R, sbase, s2, sk, ej.rec, ex2, lane, C);
        }
    } else {
        // 32-B reference: seed position, bucket, sequence, and the seed window itself
        // (window, exception bits, bases left in the sequence), so that tail_kernel tests
        // records seeded at their primer start without touching the genome again
        const uint64_t gp = sbase + pos;
        append_chunked<2>(&a.counters[a.tail_ctr], a.tails, a.tails_cap, tail,
                          make_uint4((uint32_t)gp, (uint32_t)(gp >> 32), e0.xstart, R.seq), lane, TC,
                          make_uint4((uint32_t)Gp, (uint32_t)(Gp >> 32), exp_, n - pos), a.tail_static);
    }
}

// Drain a super-step's seeds, two per lane per pass (128 per pass): both lanes'
// lookup chains (rank word -> bucket head) are in flight together.
template <int kMode, bool kInline>
__device__ __forceinline__ void drain_seeds(const ScanArgs& a, const SuperRegs& R, uint64_t sbase, uint32_t n,
                                            uint32_t qn, int lane, uint32_t& ncand, WaveLds& L,
                                            SurvChunk& C, SurvChunk& TC) {
    const uint32_t shw = 64u - 2u * (uint32_t)a.W;
    for (uint32_t b = 0; b < qn; b += 128) {
        const uint32_t ea = b + (uint32_t)lane, eb = ea + 64;
        const bool la = ea < qn, lb = eb < qn;
        const uint32_t pa = R.base + (la ? (uint32_t)L.q[ea] : 0u);
        const uint32_t pb = R.base + (lb ? (uint32_t)L.q[eb] : 0u);
        uint64_t Ga, Gb;
        uint32_t xa, xb;
        window_from_regs(a, R, sbase, pa, true, Ga, xa);
        window_from_regs(a, R, sbase, pb, true, Gb, xb);
        const uint32_t ha = (uint32_t)(Ga >> shw), hb = (uint32_t)(Gb >> shw);
        Entry e0a{}, e0b{};
        bool hva, hvb;
        if constexpr (kMode != 2) {
            // unconditional loads (index 0 when unused): both lanes' chains issue together
            // instead of one branch-and-wait per load
            const uint2 ra = a.rk[la ? (ha >> 5) : 0u];
            const uint2 rb = a.rk[lb ? (hb >> 5) : 0u];
            hva = la && ((ra.x >> (ha & 31u)) & 1u);
            hvb = lb && ((rb.x >> (hb & 31u)) & 1u);
            const uint32_t qa = ra.y + (uint32_t)__popc(ra.x & ((1u << (ha & 31u)) - 1u));
            const uint32_t qb = rb.y + (uint32_t)__popc(rb.x & ((1u << (hb & 31u)) - 1u));
            const uint2 ca = a.dents8[hva ? qa : 0u];
            const uint2 cb = a.dents8[hvb ? qb : 0u];
            if (hva) {
                if (ca.y & kHead8Full) e0a = a.dents[qa];  // full entry: IUPAC/long primer or bucket tail
                else e0a = head8_entry(ca, ha, (uint32_t)a.W);
            }
            if (hvb) {
                if (cb.y & kHead8Full) e0b = a.dents[qb];
                else e0b = head8_entry(cb, hb, (uint32_t)a.W);
            }
        } else {
            hva = la && bucket_head<kMode>(a, ha, e0a);
            hvb = lb && bucket_head<kMode>(a, hb, e0b);
        }
        heads_and_tails<kMode, kInline>(a, R, sbase, n, hva, pa, e0a, Ga, xa, lane, ncand, C, TC);
        if (b + 64 < qn) heads_and_tails<kMode, kInline>(a, R, sbase, n, hvb, pb, e0b, Gb, xb, lane, ncand, C, TC);
    }
}

// One seed of the ranked drain when full heads are rare (Table::defer_full): a compact
// head (single record seeded at its primer start, plain, l1 <= W + 16) is tested right here
// by one 32-bit XOR/popcount over bases W..l1-1 (the seed matched bases [0, W) exactly); a
// full head sends its whole bucket to tail_kernel (its first entry is in the head's low
// word), so the drain never reads a 32-B Entry.  Compact heads whose primer span holds a
// genome exception base take the general candidate test (rare: all lanes must call).
// kH16 1: 16-B heads (Table::h16) -- .x bases W..W+15, .y plain bits, .z never bits, .w the
// 8-B head's second word; a position that is neither (an IUPAC base under I=1) is skipped,
// so the count is a lower bound and the survivor is not exact.  kH16 2: the 8-B IUPAC form
// (Table::h12: .x and .w as kHead12RecBits describes) -- bases W..W+11 only.
template <int kH16>
__device__ __forceinline__ void drain_compact(const ScanArgs& a, const SuperRegs& R, uint64_t sbase, uint32_t n,
                                              bool l, uint32_t p, const uint4 c4, uint64_t G, uint32_t x, int lane,
                                              uint32_t& ncand, SurvChunk& C, SurvChunk& TC) {
    const uint32_t W = (uint32_t)a.W;
    const uint2 c = make_uint2(c4.x, c4.w);  // the 8-B head's words
    const bool full = l && (c.y & kHead8Full);
    const uint32_t L = kH16 == 2 ? (c.x & 31u) : (c.y >> kHead8RecBits) & 31u;  // l1 - W
    const uint32_t l1 = W + L;
    const uint32_t exl = l1 >= 32u ? x : x & ~(0xFFFFFFFFu >> l1);
    const bool compact = l && !full;
    const bool general = compact && exl != 0u;
    bool act = compact && !general && (uint64_t)p + l1 <= n;
    if (!R.owned) act = act && sbase + p >= a.g_lo && sbase + p < a.g_hi;
    const uint32_t g = (uint32_t)((G << (2u * W)) >> 32);
    const uint32_t xx = g ^ (kH16 == 2 ? (c.x & 0xFFFFFF00u) : c.x);
    const uint32_t Lc = kH16 == 2 ? min(L, kHead12Bases) : L;  // bases the head covers
    const uint32_t inm = Lc >= 16u ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> (2u * Lc));
    uint32_t d;
    bool exact = true;
    if constexpr (kH16 == 2) {
        const uint32_t pl = head12_plain(c.y);
        d = (xx | (xx >> 1)) & pl & inm;
        exact = L <= kHead12Bases && (pl & inm) == (0x55555555u & inm);
    } else if constexpr (kH16 == 1) {
        d = (((xx | (xx >> 1)) & c4.y) | c4.z) & 0x55555555u & inm;
        exact = ((c4.y | c4.z) & 0x55555555u & inm) == (0x55555555u & inm);
    } else {
        d = (xx | (xx >> 1)) & 0x55555555u & inm;
    }
    const int32_t p0 = (int32_t)L - a.X;  // protected: relative positions >= L - X
    const uint32_t prot = p0 <= 0 ? inm : (p0 >= 16 ? 0u : inm & (0xFFFFFFFFu >> (2 * p0)));
    bool surv = act && !(d & prot) && __popc(d) <= a.N;
    ncand += act;
    if (__any(general)) {
        const uint32_t hk = (uint32_t)(G >> (64u - 2u * W));
        Entry e;
        if constexpr (kH16 == 2) e = head12_entry(c, hk, W);
        else if constexpr (kH16 == 1) e = head16_entry(c4, hk, W);
        else e = head8_entry(c, hk, W);
        uint32_t k2 = 0;
        bool ex2 = false;
        const bool s2 = candidate(a, R, sbase, n, general, p, e, ncand, k2, G, x, true, ex2);
        if (general) {
            surv = s2;
            exact = ex2;
        }
    }
    flush_survivors(a, R, sbase, surv, p, c.y & ((1u << (kH16 == 2 ? kHead12RecBits : kHead8RecBits)) - 1u), exact, lane, C);
    bool defer = full;
    if (full && (c.y & kHead8Filt)) {
        // bucket prefilter (kHead8Filt): every record's bases W..W+F-1 against the genome;
        // a window with an exception base among them is deferred untested
        const uint32_t cnt = ((c.y >> 28) & 3u) + 1u;
        const uint32_t F = head8_filt_bases(cnt);
        const uint32_t fm = (1u << (2u * F)) - 1u;
        const uint32_t gf = g >> (32u - 2u * F);
        const uint32_t xf = x & (0xFFFFFFFFu >> W) & ~(0xFFFFFFFFu >> (W + F));
        bool any = xf != 0u;
        for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t xj = gf ^ ((c.y >> (2u * F * j)) & fm);
            any = any || __popc((xj | (xj >> 1)) & 0x55555555u) <= a.N;
        }
        defer = any;
    }
    const uint64_t gp = sbase + p;
    append_chunked<2>(&a.counters[a.tail_ctr], a.tails, a.tails_cap, defer,
                      make_uint4((uint32_t)gp, (uint32_t)(gp >> 32), c.x, R.seq), lane, TC,
                      make_uint4((uint32_t)G, (uint32_t)(G >> 32), x, n - p), a.tail_static);
}

// drain_seeds for the ranked queue (kMode 1, 1): the head comes straight from the
// queued key rank -- one dependent load (the 8-B head) per seed instead of two.
template <bool kInline, bool kDefer, int kH16 = 0>
__device__ __forceinline__ void drain_ranked(const ScanArgs& a, const SuperRegs& R, uint64_t sbase, uint32_t n,
                                             uint32_t qn, int lane, uint32_t& ncand, WaveLds& L,
                                             SurvChunk& C, SurvChunk& TC) {
    const uint32_t shw = 64u - 2u * (uint32_t)a.W;
    for (uint32_t b = 0; b < qn; b += 128) {
        const uint32_t ea = b + (uint32_t)lane, eb = ea + 64;
        const bool la = ea < qn, lb = eb < qn;
        const uint32_t pa = R.base + (la ? (uint32_t)L.rq.q[ea] : 0u);
        const uint32_t pb = R.base + (lb ? (uint32_t)L.rq.q[eb] : 0u);
        const uint32_t qa = la ? L.rq.r[ea] : 0u, qb = lb ? L.rq.r[eb] : 0u;
        if constexpr (kH16 == 2) {  // deferring drain over 8-B IUPAC heads
            const uint2 ca = a.dents12[qa];
            const uint2 cb = a.dents12[qb];
            uint64_t Ga, Gb;
            uint32_t xa, xb;
            window_from_regs(a, R, sbase, pa, true, Ga, xa);
            window_from_regs(a, R, sbase, pb, true, Gb, xb);
            drain_compact<2>(a, R, sbase, n, la, pa, make_uint4(ca.x, 0u, 0u, ca.y), Ga, xa, lane, ncand, C, TC);
            if (b + 64 < qn) drain_compact<2>(a, R, sbase, n, lb, pb, make_uint4(cb.x, 0u, 0u, cb.y), Gb, xb, lane, ncand, C, TC);
            continue;
        }
        if constexpr (kH16 == 1) {  // deferring drain over 16-B heads
            const uint4 ca = a.dents16[qa];
            const uint4 cb = a.dents16[qb];
            uint64_t Ga, Gb;
            uint32_t xa, xb;
            window_from_regs(a, R, sbase, pa, true, Ga, xa);
            window_from_regs(a, R, sbase, pb, true, Gb, xb);
            drain_compact<1>(a, R, sbase, n, la, pa, ca, Ga, xa, lane, ncand, C, TC);
            if (b + 64 < qn) drain_compact<1>(a, R, sbase, n, lb, pb, cb, Gb, xb, lane, ncand, C, TC);
            continue;
        }
        const uint2 ca = a.dents8[qa];
        const uint2 cb = a.dents8[qb];
        uint64_t Ga, Gb;
        uint32_t xa, xb;
        window_from_regs(a, R, sbase, pa, true, Ga, xa);
        window_from_regs(a, R, sbase, pb, true, Gb, xb);
        if constexpr (kDefer) {  // compact heads tested here, full-head buckets to tail_kernel
            drain_compact<0>(a, R, sbase, n, la, pa, make_uint4(ca.x, 0u, 0u, ca.y), Ga, xa, lane, ncand, C, TC);
            if (b + 64 < qn)
                drain_compact<0>(a, R, sbase, n, lb, pb, make_uint4(cb.x, 0u, 0u, cb.y), Gb, xb, lane, ncand, C, TC);
            continue;
        }
        const uint32_t ha = (uint32_t)(Ga >> shw), hb = (uint32_t)(Gb >> shw);
        Entry e0a{}, e0b{};
        if (la) {
            if (ca.y & kHead8Full) e0a = a.dents[qa];  // full entry: IUPAC/long primer or bucket tail
            else e0a = head8_entry(ca, ha, (uint32_t)a.W);
        }
        if (lb) {
            if (cb.y & kHead8Full) e0b = a.dents[qb];
            else e0b = head8_entry(cb, hb, (uint32_t)a.W);
        }
        heads_and_tails<1, kInline>(a, R, sbase, n, la, pa, e0a, Ga, xa, lane, ncand, C, TC);
        if (b + 64 < qn) heads_and_tails<1, kInline>(a, R, sbase, n, lb, pb, e0b, Gb, xb, lane, ncand, C, TC);
    }
}

// Bit 31-i set iff window i (bases [i, i+W) of the lane's 64-base ambiguity window,
// bit 63-j = base j is not A/C/G/T/U) is clean: every bad base is smeared over the W
// windows that contain it (OR of bad << t, t < W, by binary decomposition of W).
__device__ __forceinline__ uint32_t window_ok_mask(uint64_t bad, uint32_t W) {
    uint64_t acc = 0, pw = bad;
    uint32_t done = 0;
#pragma unroll
    for (int b = 0; b < 5; ++b) {
        if (W & (1u << b)) {
            acc |= pw << done;
            done += 1u << b;
        }
        pw |= pw << (1u << b);
    }
    return ~(uint32_t)(acc >> 32);
}

// Bits 31-i for i in [lo, hi), 0 <= lo, hi <= 32.
__device__ __forceinline__ uint32_t bit_range(int lo, int hi) {
    const uint32_t a = lo <= 0 ? 0xFFFFFFFFu : (lo >= 32 ? 0u : (0xFFFFFFFFu >> lo));
    const uint32_t b = hi <= 0 ? 0xFFFFFFFFu : (hi >= 32 ? 0u : (0xFFFFFFFFu >> hi));
    return a & ~b;
}

// Windows pb .. pb + 31 of a lane that lie in the span's [p_lo, p_hi).  Both differences in
// 64 bits, clamped before the narrowing: a lane deep in a record (pb >= 2^31) of a span that
// starts at 0 gave (int)p_lo - (int)pb > 0 in 32-bit arithmetic and masked every window.
__device__ __forceinline__ uint32_t span_bits(const SeqSpan& sp, uint32_t pb) {
    return bit_range((int)smax64((int64_t)sp.p_lo - (int64_t)pb, -1), (int)smin64((int64_t)sp.p_hi - (int64_t)pb, 32));
}

// W-mer at window i of a lane: top 2W bits of the 32-bit big-endian funnel at bit 2i of
// (d0, d1, d2), the lane's 48 bases; i is a compile-time constant after unrolling.
template <int I>
__device__ __forceinline__ uint32_t kmer_top(uint32_t d0, uint32_t d1, uint32_t d2) {
    constexpr int q = (2 * I) >> 5;
    constexpr int r = (2 * I) & 31;
    const uint32_t hi = q == 0 ? d0 : d1;
    const uint32_t lo = q == 0 ? d1 : d2;
    if constexpr (r == 0) return hi;
    else return __builtin_amdgcn_alignbit(hi, lo, 32 - r);
}

// Seed filter for the lane's 32 windows.  Level 1: the LDS prefilter (32 random
// ds_read_b32).  Level 2 (unless the LDS filter is the exact 4^W bitmap): the global
// presence bitmap, probed only for windows whose level-1 bit is set -- other lanes'
// requests go to word 0 and coalesce into one line.  All 32 level-2 loads are issued
// before the first result is consumed (one L2 round trip per super-step); the
// returned `issue_next` hook runs between issue and consumption so that younger loads
// (the next super-step's prefetch) do not gate the probe results.
template <int kMode, class F>
__device__ __forceinline__ uint32_t probe32(const ScanArgs& a, const uint32_t* __restrict__ lds, uint32_t d0,
                                            uint32_t d1, uint32_t d2, uint32_t shw, uint32_t okm, F&& issue_next) {
    // kMode 0: LDS exact; 1: LDS hashed + exact rank bitmap; 2: LDS hashed + hashed filter
    uint32_t lmask = 0;
    [&]<int... T>(std::integer_sequence<int, T...>) {
        ((
            [&] {
                const uint32_t x = kmer_top<T>(d0, d1, d2);  // key left-aligned
                uint32_t wi, bi;
                if constexpr (kMode == 0) {
                    wi = x >> (shw + 5u);
                    bi = (x >> shw) & 31u;
                } else {  // lds_bit: top 20 bits of the left-aligned key
                    wi = x >> (37 - kLdsFilterLog2);
                    bi = (x >> (32 - kLdsFilterLog2)) & 31u;
                }
                lmask |= __builtin_amdgcn_ubfe(lds[wi], bi, 1u) << (31 - T);
            }()),
         ...);
    }(std::make_integer_sequence<int, 32>{});
    lmask &= okm;
    if constexpr (kMode == 0) {
        issue_next();
        return lmask;
    } else {
        uint32_t gw[32];
        [&]<int... T>(std::integer_sequence<int, T...>) {
            ((
                [&] {
                    const uint32_t h = kmer_top<T>(d0, d1, d2) >> shw;
                    const uint32_t fi = kMode == 1 ? h : filter_index(h, a.filt_log2);
                    const bool on = (lmask >> (31 - T)) & 1u;
                    // kMode 1: the rank words' bits -- the same lines the drain reads next
                    // for the seeds that pass (a separate bits-only bitmap measured slower).
                    // Byte offset (h >> 5) * 8 straight from the funnel, masked to 0 by the
                    // sign-extended LDS bit: shift, and, bfe, and -- no select
                    if constexpr (kMode == 1) {
                        const uint32_t off = (kmer_top<T>(d0, d1, d2) >> (shw + 2u)) & ~7u;
                        const uint32_t sel = (uint32_t)__builtin_amdgcn_sbfe((int)lmask, 31 - T, 1);
                        gw[T] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(a.rk) + (off & sel));
                        (void)on; (void)fi;
                    } else {
                        gw[T] = a.filt[on ? (fi >> 5) : 0u];
                    }
                }()),
             ...);
        }(std::make_integer_sequence<int, 32>{});
        issue_next();
        uint32_t hits = 0;
        [&]<int... T>(std::integer_sequence<int, T...>) {
            ((
                [&] {
                    const uint32_t h = kmer_top<T>(d0, d1, d2) >> shw;
                    const uint32_t fi = kMode == 1 ? h : filter_index(h, a.filt_log2);
                    hits |= __builtin_amdgcn_ubfe(gw[T], fi & 31u, 1u) << (31 - T);
                }()),
             ...);
        }(std::make_integer_sequence<int, 32>{});
        return hits & lmask;
    }
}

// Level 1 only, kMode 1: the blocked LDS filter bits of the lane's 32 windows (bit 31-T):
// all kK bits of lds_block_mask set in the key's word.
// kGap: 0 contiguous, 1 gapped (shape in gap_at / gap_len), kGapW8 the W = 8 gapped shape.
template <int kK, int kGap = 0>
__device__ __forceinline__ uint32_t lds_probe32(const uint32_t* __restrict__ lds, uint32_t d0, uint32_t d1, uint32_t d2,
                                                uint32_t shw, uint32_t gap_at = 0u, uint32_t gap_len = 0u) {
    uint32_t lmask = 0;
    [&]<int... T>(std::integer_sequence<int, T...>) {
        ((
            [&] {
                uint32_t x = kmer_top<T>(d0, d1, d2);
                if constexpr (kGap == kGapW8) {
                    // the gapped key g = x's top 16 bits (bases 0..7) ++ x's bases 11..13: the word
                    // index (g's top 15 bits) is x's, and the second bit (g's bits 14..10, below
                    // the top 16) is x's bits 8..4; only the first bit needs g (bit 16 ++ 15..12)
                    constexpr uint32_t kShw = 32 - 2 * kSplitSeed;  // the W' = 11 key's low bits
                    static_assert(kLdsFilterLog2 - 5 <= 2 * (int)kGapW8At && kShw + 5 <= 2 * kGapW8At,
                                  "word index inside the ungapped bases, second bit below them");
                    const uint32_t wv = lds[x >> (37 - kLdsFilterLog2)];
                    // g's bits 16..12 are x's bit 16 and bits 9..6: ubfe reads only the offset's low
                    // five bits, so the bit-field insert of the two shifts is the whole index
                    // (three instructions where the masked assembly of g took four)
                    static_assert(kLdsFilterLog2 == 20 && kGapW8Len == 3, "b1 = x16 ++ x9..6");
                    const uint32_t b1 = ((x >> 6) & 15u) | ((x >> 12) & ~15u);
                    uint32_t on = __builtin_amdgcn_ubfe(wv, b1, 1u);
                    if constexpr (kK >= 2) on &= __builtin_amdgcn_ubfe(wv, (x >> (kShw - 2 * kGapW8Len)) & 31u, 1u);
                    static_assert(kK <= 2, "the W = 8 gapped form takes one or two bits per key");
                    lmask |= on << (31 - T);
                    return;
                }
                if constexpr (kGap != 0) x = gap_key(x, gap_at, gap_len);
                const uint32_t wv = lds[x >> (37 - kLdsFilterLog2)];
                uint32_t on = __builtin_amdgcn_ubfe(wv, (x >> (32 - kLdsFilterLog2)) & 31u, 1u);
                if constexpr (kK >= 2) on &= __builtin_amdgcn_ubfe(wv, (x >> shw) & 31u, 1u);
                if constexpr (kK >= 3) on &= __builtin_amdgcn_ubfe(wv, (((x >> shw) & 127u) * 37u) >> 2, 1u);
                lmask |= on << (31 - T);
            }()),
         ...);
    }(std::make_integer_sequence<int, 32>{});
    return lmask;
}

// 32-bit funnel of window i (0..31, run-time) of the lane: bases i..i+15, left-aligned.
__device__ __forceinline__ uint32_t kmer_dyn(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t i) {
    const uint32_t hi = i < 16 ? d0 : d1, lo = i < 16 ? d1 : d2;
    const uint32_t r = 2u * (i & 15u);
    return r ? __builtin_amdgcn_alignbit(hi, lo, 32u - r) : hi;
}

// The same over the lane's 64 bases (d3: bases 48..63), p in [0, 48).
__device__ __forceinline__ uint32_t kmer_dyn4(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, uint32_t p) {
    const uint32_t hi = p < 16 ? d0 : (p < 32 ? d1 : d2), lo = p < 16 ? d1 : (p < 32 ? d2 : d3);
    const uint32_t r = 2u * (p & 15u);
    return r ? __builtin_amdgcn_alignbit(hi, lo, 32u - r) : hi;
}

// Bucket-tail reference of a seed that passed the key groups (kRkf scan): no bucket field;
// tail_kernel finds the bucket from the seed window's key.
constexpr uint32_t kKeyRef = 0x80000000u;

// 16-B key reference (round 5; the key-group scans, when the genome's padded length is under
// 2^40 bases and it has fewer than 2^23 - 1 sequences): {seed position (40 bits), an
// exception flag, the sequence (23 bits), the 32-base window at the seed}.  The 32-B form also
// carried the window's exception bits and the bases left to the sequence's end; tail_kernel
// now takes the latter from seq_base / seq_len and re-reads the former from the genome only
// for a window that holds an exception base (the flag).  c4 writes and reads back ~16M
// references per run.
__device__ __forceinline__ uint4 ref16_make(uint64_t gp, uint32_t seq, uint64_t G, uint32_t ex) {
    return make_uint4((uint32_t)gp, (uint32_t)(gp >> 32) | (ex ? 0x100u : 0u) | (seq << 9), (uint32_t)G, (uint32_t)(G >> 32));
}

// 32-bit funnel of bases p..p+15 of a lane's 48 bases (A, B, C = bases 0-15, 16-31,
// 32-47), p in [0, 48); bases past 47 read as 0.
__device__ __forceinline__ uint32_t funnel3(uint32_t A, uint32_t B, uint32_t C, uint32_t p) {
    const uint32_t hi = p < 16u ? A : (p < 32u ? B : C);
    const uint32_t lo = p < 16u ? B : (p < 32u ? C : 0u);
    return (uint32_t)(((((uint64_t)hi << 32) | lo) << (2u * (p & 15u))) >> 32);
}

// Level-2 probe of the key groups (kRkf, Table::kgrp): presence of the window's key and, for
// the group's first three present keys with a compact head, primer-1 bases W..W+F-1 (see
// kKgrpKeys).  `pk`: the window's bases W..W+F-1 << 4 | the key's low 4 bits.  True = the
// seed goes on.
//
// I = 1 tables (kgrp_wild): two 24-bit fields {2-bit codes of bases W..W+F-1; at the even
// bits of the next 12, the bases that are not plain}.  The count covers the plain bases
// only, so it is a lower bound on primer-1 mismatches when every genome base of the window's
// first W + F is one of A/C/G/T/U (under I = 1 a genome IUPAC base may match anything, and
// it reads as 'A' in the 2-bit plane); bit 31 of pk marks a window where that fails, which
// then passes on presence alone.
// Gapped seed (kGap, split tables): the field holds the record's gap bases, then its gap_post
// bases after the seed's span (the low 2 gap_post bits); a window passes when its gap differs
// in 1..N positions, or has an invalid base (bit 31 of pk) -- with neither, the contiguous seed
// of the split finds the window -- and gap and post bases together differ in at most N.
// kGap = kGapW8: the W = 8 shape and N = 1 as constants.  kFix (I = 0 tables of W = 11, the
// c2 / c3 / split-contiguous shape): F = kFixF, no I = 1 fields, N = kFix - 1.
constexpr uint32_t kFixW = 11, kFixF = 6;
template <int kGap = 0, int kFix = 0>
__device__ __forceinline__ bool kgrp_pass(const ScanArgs& a, uint2 rw, uint32_t pk) {
    const uint32_t bit = pk & 15u;
    if (!((rw.x >> bit) & 1u)) return false;  // the key is absent
    if constexpr (kGap != 0) {
        constexpr bool kC = kGap == kGapW8;
        const uint32_t glen = kC ? kGapW8Len : a.gap_len, gpost = kC ? kGapW8Post : a.gap_post;
        const uint32_t F = kC ? kGapW8Len + kGapW8Post : a.kgrp_F, N = kC ? 1u : (uint32_t)a.N;
        const uint32_t j = (uint32_t)__popc(__builtin_amdgcn_ubfe(rw.x, 0u, bit));
        if (j >= kKgrpFields) return true;
        const uint32_t field = j == 0u ? (rw.x >> 16) : (j == 1u ? (rw.y & 0xFFFFu) : (rw.y >> 16));
        if (!(field & kKgrpFlag)) {
            if (!(field & kKgrpPair)) return true;
            // two records (gap_len <= 3): either record's gap differs in 1..N positions, or the
            // window's gap holds an invalid base
            if (pk >> 31) return true;
            const uint32_t gm = (1u << (2u * glen)) - 1u;
            const uint32_t g = (pk >> (4u + 2u * gpost)) & gm;
            const uint32_t x0 = g ^ ((field >> 6) & gm), x1 = g ^ (field & gm);
            const uint32_t m0 = (uint32_t)__popc((x0 | (x0 >> 1)) & 0x555u), m1 = (uint32_t)__popc((x1 | (x1 >> 1)) & 0x555u);
            return (m0 >= 1u && m0 <= N) || (m1 >= 1u && m1 <= N);
        }
        const uint32_t x = ((pk >> 4) ^ field) & ((1u << (2u * F)) - 1u);
        const uint32_t m = (x | (x >> 1)) & 0x55555555u;
        return (uint32_t)__popc(m) <= N && ((m >> (2u * gpost)) != 0u || (pk >> 31) != 0u);
    }
    if (!kFix && a.kgrp_wild) {
        if (pk >> 31) return true;
        const uint32_t j = (uint32_t)__popc(__builtin_amdgcn_ubfe(rw.x, 0u, bit));
        if (j >= kKgrpWildFields) return true;
        const uint64_t w64 = ((uint64_t)rw.y << 32) | rw.x;
        const uint32_t field = (uint32_t)(w64 >> (16u + 24u * j));
        const uint32_t x = ((pk >> 4) ^ field) & ((1u << (2u * a.kgrp_F)) - 1u);
        return (uint32_t)__popc((x | (x >> 1)) & 0x555u & ~(field >> 12)) <= (uint32_t)a.N;
    }
    const uint32_t F = kFix ? kFixF : a.kgrp_F, N = kFix ? (uint32_t)(kFix - 1) : (uint32_t)a.N;
    const uint32_t j = (uint32_t)__popc(__builtin_amdgcn_ubfe(rw.x, 0u, bit));
    if (j >= kKgrpFields) return true;
    const uint32_t field = j == 0u ? (rw.x >> 16) : (j == 1u ? (rw.y & 0xFFFFu) : (rw.y >> 16));
    if (!(field & kKgrpFlag)) {
        if (!(field & kKgrpPair)) return true;
        // two records: the window's bases W..W+2 (the top 3 of its F) against each record's
        const uint32_t g3 = (pk >> (4u + 2u * (F - 3u))) & 63u;
        const uint32_t x0 = g3 ^ ((field >> 6) & 63u), x1 = g3 ^ (field & 63u);
        return (uint32_t)__popc((x0 | (x0 >> 1)) & 0x15u) <= N || (uint32_t)__popc((x1 | (x1 >> 1)) & 0x15u) <= N;
    }
    const uint32_t x = ((pk >> 4) ^ field) & ((1u << (2u * F)) - 1u);
    return (uint32_t)__popc((x | (x >> 1)) & 0x55555555u) <= N;
}

// Level-2 probe of the wide I = 1 key groups (kgrp4, see kKgrp4Keys).  `pk`: the window's
// bases W..W+F-1 << 5 | the key's low 5 bits, bit 31 set when the window's first W + F bases
// are not all A/C/G/T/U (it then passes on presence alone).  True = the seed goes on (as a
// key reference).
// kFix: N = kFix - 1 as a constant.
template <int kFix = 0>
__device__ __forceinline__ bool kgrp_pass4(const ScanArgs& a, uint4 rw, uint32_t pk) {
    static_assert(kKgrp4F == 10 && kKgrp4Fields == 3, "field layout: three 32-bit fields");
    const uint32_t bit = pk & 31u;
    if (!((rw.x >> bit) & 1u)) return false;
    const uint32_t j = (uint32_t)__popc(__builtin_amdgcn_ubfe(rw.x, 0u, bit));
    if ((pk >> 31) || j >= kKgrp4Fields) return true;
    const uint32_t f = j == 0u ? rw.y : (j == 1u ? rw.z : rw.w);
    const uint32_t x = ((pk >> 5) ^ f) & ((1u << (2u * kKgrp4F)) - 1u);
    // the plain flags (bits 2F.., base W on top) spread to the low bit of each base's slot
    uint32_t pl = (f >> (2u * kKgrp4F)) & ((1u << kKgrp4F) - 1u);
    pl = (pl | (pl << 8)) & 0x00FF00FFu;
    pl = (pl | (pl << 4)) & 0x0F0F0F0Fu;
    pl = (pl | (pl << 2)) & 0x33333333u;
    pl = (pl | (pl << 1)) & 0x55555555u;
    return (uint32_t)__popc((x | (x >> 1)) & pl) <= (kFix ? (uint32_t)(kFix - 1) : (uint32_t)a.N);
}

// The span of super-step x (wave-uniform; every lane active) and the next span's first
// super-step.  Up to 63 spans (c3-c5: 24): one load per lane and a ballot -- a scan's first
// super-step had waited for a binary search of ~5 dependent loads (its first super-step took
// 15 us against ~6.2, per-super-step stamps); more spans: the binary search.
__device__ __forceinline__ void span_find(const ScanArgs& a, uint64_t x, int lane, SeqSpan& pf, uint64_t& pf_end) {
    if (a.n_spans < 64u) {
        SeqSpan my{};
        my.super0 = ~0ull;
        if ((uint32_t)lane <= a.n_spans) my = a.spans[lane];  // spans[n_spans]: the sentinel
        const int lo = __popcll(__ballot(my.super0 <= x)) - 1;
        pf.super0 = shfl64(my.super0, lo);
        pf.seq = (uint32_t)__shfl((int)my.seq, lo, 64);
        pf.p_lo = (uint32_t)__shfl((int)my.p_lo, lo, 64);
        pf.p_hi = (uint32_t)__shfl((int)my.p_hi, lo, 64);
        pf.p_al = (uint32_t)__shfl((int)my.p_al, lo, 64);
        pf_end = shfl64(my.super0, lo + 1);
        return;
    }
    uint32_t lo = 0, hi = a.n_spans;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.spans[mid].super0 <= x) lo = mid;
        else hi = mid;
    }
    pf = a.spans[lo];
    pf_end = a.spans[lo + 1].super0;
}

// Persistent scan: every wave walks global super-steps blockIdx*kWaves + w, + all waves,
// ...; a super-step is 2048 consecutive window positions of one sequence, 32 per lane.
// The next super-step's plane words are loaded before the current one is processed.
// Dynamic super-step order: with a static round-robin the last wave of the scan
// ended 15% after the mean (c3: 2.76 vs 2.36 ms, per-wave timers) -- super-steps differ in
// cost and a CU's younger waves get fewer issue slots.  Each XCD (blocks x, x+8, ...) owns
// a contiguous 1/8 of the super-steps in chunks of kSChunk; its waves take one chunk each,
// then claim further chunks from the XCD's counter one chunk ahead (the claim's latency
// hides behind the chunk's work; ~9 atomics per microsecond per counter on c3).
#ifndef MP_SCHUNK
#define MP_SCHUNK 8
#endif
constexpr uint32_t kSChunk = MP_SCHUNK;
// Short scans (under kSChunkShort super-steps per wave, e.g. one rank's eighth of c3) take
// chunks of 4: the last chunks then even out sooner (1/8 of c3: scan 0.354 ms static, 0.335
// in chunks of 8, 0.323 in chunks of 4; full c3 is best with 8).  Only scans under
// MP_SCHED_MIN super-steps per wave keep the static order.
constexpr uint32_t kSChunkShort = 128;
#ifndef MP_SCHUNK_SHORT
#define MP_SCHUNK_SHORT 4
#endif
#ifndef MP_SCHED_MIN
#define MP_SCHED_MIN 4u
#endif
// Claims are positions, not tickets: a wave adds the size it wants to its group's counter.
// The size shrinks with the group's remaining range (about the range left / twice the
// group's waves, from the wave's last claim: "guided"), and is halved for the two youngest
// waves of each SIMD.  Per-wave stamps (scripts/wave_times.py, ablation 40) on a 1/8 c3
// scan: a SIMD issues for its oldest wave first, so waves 12-15 of a block did 29
// super-steps at ~11 us each and waves 0-3 did 60 at ~5 us; with fixed chunks of 4 and one
// chunk claimed ahead the young waves ended 20 us after the old ones and the last wave 47 us
// after the first.
// Round 6: a block's first chunks are claimed, not assigned.  Thread 0 claims kW chunks for its
// waves with one atomic on the group's counter while the block stages its LDS (block_claim); the
// waves then claim on as before.  Round 5 gave each wave a static first chunk at lo + (its index
// in the group) x chunk: a block that started late (another kernel holding its CU) still owned
// that chunk, and the scan could not end before the late block had done it.  Now a late block
// takes only what is left, and its waves find nothing and leave when the group's range is gone.
// Start-up cost: one more returning atomic per block (32 per group counter), under the LDS
// staging; same-box step times unchanged (profiles/r06i_sched_ab.json).
__device__ __forceinline__ bool sched_dynamic(uint64_t n_supers, int kW) {
    return n_supers >= (uint64_t)gridDim.x * (uint32_t)kW * MP_SCHED_MIN;
}
__device__ __forceinline__ uint32_t sched_chunk(uint64_t n_supers, int kW, uint32_t short_chunk) {
    return n_supers < (uint64_t)gridDim.x * (uint32_t)kW * kSChunkShort ? short_chunk : kSChunk;
}
// thread 0 of the block: the group-relative position of the block's kW first chunks
__device__ __forceinline__ uint32_t block_claim(unsigned long long* counters, uint32_t sched_base, uint64_t n_supers,
                                                int kW, uint32_t short_chunk) {
    const uint32_t g = gridDim.x < 8u ? gridDim.x : 8u;
    unsigned int* ctr = reinterpret_cast<unsigned int*>(counters + sched_base + (blockIdx.x % g) * kStatStride);
    return atomicAdd(ctr, (uint32_t)kW * sched_chunk(n_supers, kW, short_chunk));
}

struct SuperSched {  // 32-bit state (super-step indices < 2^32): it lives beside the scan's registers
    uint32_t lo, hi, nw, end;  // XCD group range, waves of the group, end of the current chunk
    uint32_t S;                // where claimed positions count from (the group's lo)
    uint32_t pending, psize;   // lane 0: position claimed for the next chunk, and its size
    uint32_t stride;           // 0: dynamic; else the static round-robin stride
    uint32_t chunk;            // largest claim
    uint32_t young;            // the SIMD's two youngest waves (w >= kW / 2) claim half
    uint32_t hint;             // start of this wave's last chunk (the guided size's estimate)
    unsigned int* ctr;
    // first_pos: the block's claim (block_claim, shared through LDS; unused for static-order scans)
    __device__ __forceinline__ uint64_t first(unsigned long long* counters, uint32_t sched_base, uint64_t n_supers, int w,
                                              int kW, int lane, uint32_t short_chunk, uint32_t first_pos) {
        // short scans (under 64 super-steps per wave, e.g. c2) keep the static order: their
        // per-wave totals average out and the claims would only add latency
        const uint32_t waves = gridDim.x * (uint32_t)kW;
        if (!sched_dynamic(n_supers, kW)) {
            stride = waves;
            return (uint64_t)blockIdx.x * (uint64_t)kW + (uint64_t)w;
        }
        stride = 0;
        chunk = sched_chunk(n_supers, kW, short_chunk);
        const uint32_t g = gridDim.x < 8u ? gridDim.x : 8u;  // groups: one per XCD, fewer on small grids
        const uint32_t x = blockIdx.x % g;
        ctr = reinterpret_cast<unsigned int*>(counters + sched_base + x * kStatStride);
        lo = (uint32_t)(n_supers * x / g);
        hi = (uint32_t)(n_supers * (x + 1) / g);
        nw = ((gridDim.x - x + g - 1u) / g) * (uint32_t)kW;
        S = lo;
        young = (uint32_t)w >= (uint32_t)kW / 2u;
        // positions past the range: the sum saturates instead of wrapping (a very late block)
        const uint64_t st64 = (uint64_t)lo + first_pos + (uint64_t)w * chunk;
        const uint32_t st = st64 < hi ? (uint32_t)st64 : hi;
        end = min(st + chunk, hi);
        hint = st;
        claim(lane);
        return st < hi ? st : n_supers;
    }
    __device__ __forceinline__ void claim(int lane) {
        const uint32_t from = max(hint, S);
        const uint32_t left = hi > from ? hi - from : 0u;
        uint32_t sz = min(chunk, max(1u, left / (2u * nw)));
        if (young) sz = max(1u, sz >> 1);
        psize = sz;
        pending = 0;
        if (lane == 0) pending = atomicAdd(ctr, sz);
    }
    __device__ __forceinline__ uint64_t next(uint64_t ss, uint64_t n_supers, int lane) {
        if (stride) return ss + stride;
        if (ss + 1 < end) return ss + 1;
        // lane 0 holds the claimed position; next() runs at the top of the super-step loop
        // with every lane active, so the first active lane is lane 0 and the broadcast is a
        // readfirstlane (the scheduler state then stays in scalar registers)
        uint32_t st = S + (uint32_t)__builtin_amdgcn_readfirstlane((int)pending);
        if (st >= hi) {
            end = 0;
            return n_supers;
        }
        end = min(st + psize, hi);
        hint = st;
        claim(lane);
        return st;
    }
};

// kRkf: 0 the rank queue and drain; 1 the key groups (kgrp, u64 per 16 keys); 2 the wide I = 1 key
// groups (kgrp4, uint4 per 32 keys: presence and three ten-base fields).  1 and 2 leave the seeds
// that pass as key references for tail_kernel.
template <int kMode, bool kInline, int kK = 1, bool kDefer = false, int kH16 = 0, int kRkf = 0,
          int kGap = 0, int kFix = 0>
__global__ __launch_bounds__(kBlock) void scan_kernel(ScanArgs a) {
    static_assert(kGap == 0 || (kMode == 1 && kRkf), "gapped seeds take the key-group path");
    // kFix: W = 11 and N = kFix - 1 as constants; for kRkf 1 (I = 0 key groups) also F = 6
    static_assert(kFix == 0 || (kMode == 1 && kRkf != 0 && kGap == 0), "kFix: the key-group scans");
    // the gapped seed's shape: compile-time for kGapW8 (c5), else the table's
    constexpr bool kGC = kGap == kGapW8;
    const uint32_t g_at = kGC ? kGapW8At : a.gap_at, g_len = kGC ? kGapW8Len : a.gap_len;
    const uint32_t g_post = kGC ? kGapW8Post : a.gap_post;
    __shared__ uint32_t s_lf[kLdsFilterWords];
    // the per-wave lists: the key-group forms (kRkf) use only the offset list rq.q (680 B per
    // wave of the 2,040): 21 KB of the CU's LDS stay free beside the scan block, for a later
    // step's bucket-tail or order blocks to run on the same CU
    constexpr uint32_t kWlBytes = kRkf ? (uint32_t)((kSeedQR * sizeof(uint16_t) + 15u) & ~15u) : (uint32_t)sizeof(WaveLds);
    __shared__ __attribute__((aligned(16))) uint8_t s_wl_raw[kWaves * kWlBytes];

    zero_sort_counts(a);
    const uint64_t n_supers = a.spans[a.n_spans].super0;
    __shared__ uint32_t s_first;  // the block's first chunks (block_claim), issued before the staging loads
    if (threadIdx.x == 0 && sched_dynamic(n_supers, kWaves))
        s_first = block_claim(a.counters, a.sched_base, n_supers, kWaves, a.sched_short);
    // stage the seed prefilter in LDS (once per persistent workgroup): all eight 16-B loads of
    // a thread in flight before the first LDS store (one L2 round trip, not eight)
    {
        constexpr int kStage = (int)(kLdsFilterWords / 4 / kBlock);  // eight uint4 per thread (128 KiB)
        static_assert(kLdsFilterWords / 4 == kStage * kBlock, "whole uint4 rows per thread");
        const uint4* src = reinterpret_cast<const uint4*>(a.lfilt);
        uint4 v[kStage];
#pragma unroll
        for (int k = 0; k < kStage; ++k) v[k] = src[threadIdx.x + k * kBlock];
#pragma unroll
        for (int k = 0; k < kStage; ++k) reinterpret_cast<uint4*>(s_lf)[threadIdx.x + k * kBlock] = v[k];
    }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const uint64_t stride = (uint64_t)gridDim.x * kWaves;
    const uint32_t W = kFix ? kFixW : (uint32_t)a.W;
    const uint32_t shw = 32u - 2u * W;
    WaveLds& L = *reinterpret_cast<WaveLds*>(s_wl_raw + (uint32_t)w * kWlBytes);
    uint32_t ncand = 0;
    SurvChunk C{0, kChunkNone, 0u};
    // the wave's first kStaticRefs bucket-tail slots are its own, [gwave * kStaticRefs, + kStaticRefs):
    // when every wave took its first chunk with an atomic, the 4,096 reservations of a scan's
    // first super-steps queued on one address (~88 per us) and the first two super-steps of a
    // wave took 34 and 21 us against ~6.5 (per-super-step stamps, ablation 42).  Expressed as
    // a chunk of kTC slots of which kTC - kStaticRefs are used.
    constexpr uint32_t kTC = kRkf == 2 ? kRefChunk : (kRkf ? kRefChunk1 : 64u);
    static_assert(kTC >= kStaticRefs, "static slots within one chunk");
    // (Inline-tail scans rarely leave a reference: theirs start with no chunk.)
    SurvChunk TC{0, kChunkNone, 0u};
    if constexpr (!kInline)
        TC = SurvChunk{((uint64_t)blockIdx.x * kWaves + (uint64_t)(threadIdx.x >> 6)) * kStaticRefs - (kTC - kStaticRefs),
                       kTC - kStaticRefs, 0u};

    SuperSched sch;
    uint64_t ss = sch.first(a.counters, a.sched_base, n_supers, w, kWaves, lane, a.sched_short, s_first);
    // span of the super-step being prefetched, cached in registers (wave-uniform): the
    // common path of the prefetch issues only the four plane loads, no waits
    SeqSpan pf{};
    pf.super0 = 1;
    uint64_t pf_end = 0, pf_sbase = 0;
    uint32_t pf_n = 0;
    auto locate = [&](uint64_t x) {  // wave-uniform x, every lane active
        if (x >= pf.super0 && x < pf_end) return;
        span_find(a, x, lane, pf, pf_end);
        pf_sbase = a.seq_base[pf.seq];
        pf_n = (uint32_t)a.seq_len[pf.seq];
    };
    // The prefetch keeps the two raw ambiguity words; they are joined where the super-step
    // starts.  Joining them at the prefetch (round 5) put a vmcnt wait for the ambiguity load
    // -- and, counters being in order, for every level-2 probe issued before it -- right
    // after the issue: the "prefetch" of that plane was a synchronous HBM round trip per
    // super-step.
    auto words = [&](uint64_t x, uint64_t& w0, uint64_t& w1, uint64_t& v0, uint64_t& v1) {
        const uint64_t j = pf_sbase + pf.p_al + (x - pf.super0) * kSuper + (uint64_t)lane * kLanePos;
        w0 = a.g2[j >> 5];
        w1 = a.g2[(j >> 5) + 1];
        v0 = a.ginv[j >> 6];  // branch-free: both loads always issue
        v1 = a.ginv[(j >> 6) + 1];
    };
    uint64_t nw0 = 0, nw1 = 0, nv0 = 0, nv1 = 0;
    // The next super-step's words, issued after this step's level-2 probes.  They are issued
    // on every path -- a scan's last super-step reloads its own words, a dense super-step's
    // later rounds the same addresses -- so that they are the youngest loads wherever the
    // probes are consumed: the compiler then waits vmcnt(2) there, and the HBM round trip
    // runs under the rest of the super-step.  (A conditional issue merges with a path that
    // has no such loads, and the merged wait is vmcnt(0).)
    auto prefetch = [&](uint64_t nx, uint64_t cur) {
        const uint64_t x = nx < n_supers ? nx : cur;
        locate(x);
        words(x, nw0, nw1, nv0, nv1);
    };
    if (ss < n_supers) {
        locate(ss);
        words(ss, nw0, nw1, nv0, nv1);
    }
    while (ss < n_supers) {
        const SeqSpan sp = pf;
        const uint64_t sbase = pf_sbase;
        const uint32_t n = pf_n;
        SuperRegs R;
        R.w0 = nw0;
        R.w1 = nw1;
        R.base = sp.p_al + (uint32_t)(ss - sp.super0) * kSuper;
        R.seq = sp.seq;
        R.owned = (a.g_lo == 0 || sbase + R.base >= a.g_lo + 65536u) && sbase + R.base + kSuper <= a.g_hi;
        const uint32_t pb = R.base + (uint32_t)lane * kLanePos;
        R.iv = inv_join(nv0, nv1, (uint32_t)((sbase + pb) & 32u));
        const uint32_t d0 = (uint32_t)(R.w0 >> 32), d1 = (uint32_t)R.w0, d2 = (uint32_t)(R.w1 >> 32);
        // a gapped seed's windows: both of its pieces clean
        const uint32_t okm = (kGap ? window_ok_mask(R.iv, g_at) &
                                         window_ok_mask(R.iv << (g_at + g_len), (kGC ? kSplitSeed : W) - g_at)
                                   : window_ok_mask(R.iv, W)) &
                             span_bits(sp, pb);
        const uint64_t nx = sch.next(ss, n_supers, lane);
        (void)stride;
        if constexpr (kMode == 1) {
            // level 2, wave-compacted: the wave's LDS-positive windows go into the LDS list
            // {key, offset} (the queue's arrays), then every lane probes one list entry per
            // pass -- full lanes, all passes' rank-word loads in flight together -- and the
            // seeds are compacted back into the same arrays as {offset, rank}
            const uint32_t rem = lds_probe32<kK, kGap>(s_lf, d0, d1, d2, shw, g_at, g_len) & okm;
            // I = 1 key groups: windows whose first W + F bases are not all A/C/G/T/U; gapped
            // seeds: windows with an invalid base in the gap
            const uint32_t fbad = kGap ? ~window_ok_mask(R.iv << g_at, g_len)
                                       : (kRkf == 2 ? ~window_ok_mask(R.iv, W + kKgrp4F)
                                                    : ((kRkf && !kFix && a.kgrp_wild) ? ~window_ok_mask(R.iv, W + a.kgrp_F) : 0u));
            const uint32_t c = (uint32_t)__popc(rem);
            const uint32_t incl = wave_incl_scan(c, lane);
            const uint32_t tot = rl32(incl, 63);
            uint32_t r0 = 0;
            do {  // rounds of kSeedQR positives (one round unless the super-step is dense)
                {
                    uint32_t m = rem, qi = incl - c;
                    while (m) {
                        const uint32_t i = (uint32_t)__clz(m);
                        m &= ~(0x80000000u >> i);
                        if (qi - r0 < kSeedQR) {
                            if constexpr (kRkf) {  // the offset only: the probe shuffles the window from its lane
                                L.rq.q[qi - r0] = (uint16_t)(((uint32_t)lane * kLanePos + i) |
                                                             (((fbad << i) >> 31) << 15));
                            } else {
                                L.rq.r[qi - r0] = kmer_dyn(d0, d1, d2, i) >> shw;
                                L.rq.q[qi - r0] = (uint16_t)((uint32_t)lane * kLanePos + i);
                            }
                        }
                        ++qi;
                    }
                }
                wave_sync();
                const uint32_t nr = min(tot - r0, kSeedQR);
                constexpr int kP = (kSeedQR + 63) / 64;
                uint32_t pk[kP], po[kP];
                std::conditional_t<kRkf == 2, uint4, uint2> rw[kP];
#pragma unroll
                for (int q = 0; q < kP; ++q) {
                    const uint32_t e = (uint32_t)q * 64u + (uint32_t)lane;
                    pk[q] = 0;
                    po[q] = 0;
                    rw[q] = {};
                    if ((uint32_t)q * 64u < nr) {
                        const bool v = e < nr;
                        if constexpr (kRkf) {
                            // bases [i, i + W + F) of window i of lane src: three shuffles of the
                            // lane's 48 bases; pk = the F filter bases << 4 | the key's low 4 bits
                            const uint32_t qe = v ? (uint32_t)L.rq.q[e] : 0u;
                            po[q] = qe & 0x7FFu;
                            const int sa = (int)((po[q] >> 5) << 2);
                            const uint32_t A = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)d0);
                            const uint32_t B = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)d1);
                            const uint32_t C = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)d2);
                            const uint32_t i = po[q] & 31u;
                            const uint32_t key = (kGap ? gap_key(funnel3(A, B, C, i), g_at, g_len)
                                                       : funnel3(A, B, C, i)) >> shw;
                            // the field's bases: after the key, or a gapped seed's gap and the
                            // bases after its span (2 gap_len bases after the gap's start)
                            uint32_t fb;
                            if constexpr (kRkf == 2) {  // kKgrp4F bases: a fourth shuffle (bases 48..63)
                                const uint32_t D = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)(uint32_t)R.w1);
                                const uint32_t p = i + W;
                                const uint32_t hi = p < 16u ? A : (p < 32u ? B : C), lo = p < 16u ? B : (p < 32u ? C : D);
                                const uint32_t r = 2u * (p & 15u);
                                fb = (r ? __builtin_amdgcn_alignbit(hi, lo, 32u - r) : hi) >> (32u - 2u * kKgrp4F);
                                pk[q] = (fb << 5) | (key & (kKgrp4Keys - 1u)) | ((qe >> 15) << 31);
                                rw[q] = a.kgrp4[v ? (key >> kKgrp4Log2) : 0u];
                            } else if constexpr (kGap != 0) {
                                const uint32_t f = funnel3(A, B, C, i + g_at);
                                fb = ((f >> (32u - 2u * g_len)) << (2u * g_post)) |
                                     (g_post ? (f << (4u * g_len)) >> (32u - 2u * g_post) : 0u);
                            } else {
                                fb = funnel3(A, B, C, i + W) >> (32u - 2u * (kFix ? kFixF : a.kgrp_F));
                            }
                            if constexpr (kRkf != 2) {
                                pk[q] = (fb << 4) | (key & 15u) | ((qe >> 15) << 31);
                                rw[q] = a.kgrp[v ? (key >> 4) : 0u];
                            }
                        } else {
                            pk[q] = v ? L.rq.r[e] : 0u;
                            po[q] = v ? (uint32_t)L.rq.q[e] : 0u;
                            rw[q] = a.rk[v ? (pk[q] >> 5) : 0u];
                        }
                    }
                }
                prefetch(nx, ss);  // after this round's probes (every round: see prefetch)
                wave_sync();  // every list entry is in registers before the seeds overwrite it
                if constexpr (kRkf != 0) {
                    // the few seeds that pass the key groups (c3: 4% of seeds) leave as key
                    // references for tail_kernel, with their window, exception bits and bases
                    // left: compacted into the list, then one pass of window shuffles per 64
                    uint32_t qn = 0;
#pragma unroll
                    for (int q = 0; q < kP; ++q) {
                        if ((uint32_t)q * 64u < nr) {
                            const uint32_t e = (uint32_t)q * 64u + (uint32_t)lane;
                            bool hit;
                            if constexpr (kRkf == 2) hit = kgrp_pass4<kFix>(a, rw[q], pk[q]) && e < nr;
                            else hit = e < nr && kgrp_pass<kGap, kFix>(a, rw[q], pk[q]);
                            const uint64_t hm = __ballot(hit);
                            if (hit) L.rq.q[qn + (uint32_t)__popcll(hm & ((1ull << lane) - 1ull))] = (uint16_t)po[q];
                            qn += (uint32_t)__popcll(hm);
                        }
                    }
                    wave_sync();
                    for (uint32_t b = 0; b < qn; b += 64) {
                        const uint32_t e = b + (uint32_t)lane;
                        const bool on = e < qn;
                        const uint32_t p = R.base + (on ? ((uint32_t)L.rq.q[e] & 0x7FFu) : 0u);
                        uint64_t G;
                        uint32_t x;
                        window_from_regs(a, R, sbase, p, true, G, x);
                        const uint64_t gp = sbase + p;
                        if (a.ref16)  // wave-uniform
                            append_chunked<1, kTC>(&a.counters[a.tail_ctr], a.tails, a.tails_cap, on,
                                                   ref16_make(gp, R.seq, G, x), lane, TC, uint4{}, a.tail_static);
                        else
                            append_chunked<2, kTC>(&a.counters[a.tail_ctr], a.tails, a.tails_cap, on,
                                                   make_uint4((uint32_t)gp, (uint32_t)(gp >> 32), kKeyRef, R.seq), lane, TC,
                                                   make_uint4((uint32_t)G, (uint32_t)(G >> 32), x, n - p), a.tail_static);
                    }
                    wave_sync();  // the next round rewrites the list
                    r0 += kSeedQR;
                    continue;
                }
                uint32_t qn = 0;
#pragma unroll
                for (int q = 0; q < kP; ++q) {
                    if ((uint32_t)q * 64u < nr) {
                        const uint32_t e = (uint32_t)q * 64u + (uint32_t)lane;
                        bool hit;
                        uint32_t rank;
                        {
                            const uint32_t bq = pk[q] & 31u;
                            hit = e < nr && ((rw[q].x >> bq) & 1u);
                            rank = rw[q].y + (uint32_t)__popc(rw[q].x & ((1u << bq) - 1u));
                        }
                        const uint64_t hm = __ballot(hit);
                        if (hit) {
                            const uint32_t at = qn + (uint32_t)__popcll(hm & ((1ull << lane) - 1ull));
                            L.rq.q[at] = (uint16_t)(po[q] & 0x7FFu);
                            L.rq.r[at] = rank;
                        }
                        qn += (uint32_t)__popcll(hm);
                    }
                }
                wave_sync();
                if (qn) drain_ranked<kInline, kDefer, kH16>(a, R, sbase, n, qn, lane, ncand, L, C, TC);
                wave_sync();
                r0 += kSeedQR;
            } while (r0 < tot);
            ss = nx;
            continue;
        }
        uint32_t hits = probe32<kMode>(a, s_lf, d0, d1, d2, shw, okm, [&] {
            prefetch(nx, ss);  // the next super-step's words (issued after this step's probes)
        });
        // publish this super-step's seed hits: per-lane masks + prefix of their counts
        const uint32_t c = (uint32_t)__popc(hits);
        const uint32_t incl = wave_incl_scan(c, lane);
        const uint32_t total = rl32(incl, 63);
        // queue this super-step's seed offsets (lane-major = window order) and drain them
        for (uint32_t rb = 0; rb < total; rb += kSeedQ) {
            uint32_t m = hits, q = incl - c;
            while (m) {
                const uint32_t i = (uint32_t)__clz(m);
                m &= ~(0x80000000u >> i);
                if (q - rb < kSeedQ) L.q[q - rb] = (uint16_t)((uint32_t)lane * kLanePos + i);
                ++q;
            }
            wave_sync();
            drain_seeds<kMode, kInline>(a, R, sbase, n, min(total - rb, kSeedQ), lane, ncand, L, C, TC);
            wave_sync();
        }
        ss = nx;
    }
    close_chunked(a.surv, a.surv_cap, lane, C);
    if (a.ref16) close_chunked<1, kTC>(a.tails, a.tails_cap, lane, TC);
    else close_chunked<2, kTC>(a.tails, a.tails_cap, lane, TC);
    // candidate statistics
    add_stats(a, ncand, lane == 0 ? C.total : 0u, lane);
}

// Dense seeds (W <= kDenseMaxW, e.g. W=8: ~95% of windows hit one of 62k keys, 3.2 records
// each).  A per-32-key bucket index {inline-bucket bits, first oct | any-escape flag} plus
// the group's escape bits (12 B per group, 24 KiB at W=8) is staged in LDS.  Every lane takes its own 32 windows in four static
// batches of eight: for each seed window of a batch the index gives the bucket's oct (the
// 16-bit filter words of up to eight records, primer-1 bases W..W+F-1 each), all eight oct
// loads are issued together, then each word is tested against the window's bases W..W+F-1
// from the lane's own registers -- two words per 32-bit XOR / mismatch-mask / popcount.
// Only words that pass (and "always" words) reach the full 32-B Entry test (fp_reject,
// exact); buckets of more than eight records (escape bit) are walked through binfo.  One
// L2 request per seed window, no seed queue, no shuffles, no per-seed loop.
constexpr int kDenseBlock = kBlock;
#ifndef MP_DENSE_BATCH
#define MP_DENSE_BATCH 8
#endif
constexpr int kDB = MP_DENSE_BATCH;  // windows whose oct loads are in flight together
constexpr int kDenseWaves = kDenseBlock / 64;

// Full test of filter-passing slots: bit 8t+j of pm (window t of the batch base tb, slot j
// of its oct oi[t]) -> fp_reject on the Entry, survivors appended.
__device__ __forceinline__ void dense_full_tests(const ScanArgs& a, uint64_t pm, const uint2* s_grp, uint32_t ob,
                                                 uint32_t tb, uint32_t pb, uint64_t w0, uint64_t w1, uint64_t iv,
                                                 uint64_t sbase, uint32_t n, bool owned, uint32_t seq, int lane,
                                                 SurvChunk& C, uint32_t& ncand) {
    const uint64_t* exc = a.has_u ? a.gexc : a.ginv;
    while (__any(pm != 0)) {
        bool surv = false, exact = false;
        uint32_t k = 0, rec = 0;
        if (pm) {
            const uint32_t bit = (uint32_t)__builtin_ctzll(pm);
            pm &= pm - 1;
            const uint32_t t = bit >> 3, j = bit & 7u;
            const uint32_t wi = tb + t;  // window offset in the lane's 32
            uint32_t o = ob;             // escape walk: the oct itself
            if (s_grp) {                 // batch: the window's oct from the LDS index again
                const uint32_t h = (uint32_t)((wi ? (w0 << (2 * wi)) | (w1 >> (64 - 2 * wi)) : w0) >> (64 - 2 * a.W));
                const uint2 L = s_grp[h >> 5];
                o = (L.y & 0x7FFFFFFFu) + (uint32_t)__popc(L.x & ((1u << (h & 31u)) - 1u));
            }
            const Entry e = a.dents_pad[(uint64_t)o * kDenseOct + j];  // l1 = 0: a spare slot
            const uint32_t pos = pb + wi;
            k = pos - e.hash_off;
            rec = e.rec;
            bool act = e.l1 != 0 && pos >= e.hash_off && (uint64_t)k + e.l1 <= n;
            if (!owned) act = act && sbase + k >= a.g_lo && sbase + k < a.g_hi;
            if (act) {
                uint64_t Gk = wi ? (w0 << (2 * wi)) | (w1 >> (64 - 2 * wi)) : w0;
                uint32_t xk = (uint32_t)((iv << wi) >> 32);
                if (a.has_u || e.hash_off) {  // U in the genome, or a record seeded inside its primer
                    Gk = ext2(a.g2, sbase + k);
                    xk = (uint32_t)(ext1(exc, sbase + k) >> 32);
                }
                surv = !fp_reject(a, Gk, xk, e.l1, e.code, e.pmask, exact);
#ifndef MP_DENSE_SLOT_STATS
                ++ncand;
#endif
            }
        }
        const uint64_t gk = sbase + k;
        append_chunked(&a.counters[2], a.surv, a.surv_cap, surv,
                       make_uint4((uint32_t)gk, (uint32_t)(gk >> 32), rec | (exact ? 0x80000000u : 0u), seq), lane,
                       C);
    }
}

// Filter pass bits of one oct (slot 2j in the low half of word j, 2j+1 in the high half;
// bit j of the result = slot j) against the window's bases W..W+F-1 in both halves of gg:
// set where at most N of the F bases differ.  Per word: one mismatch bit per base (the low
// bit of its 2-bit slot), the lowest set bit cleared N times by a packed 16-bit decrement,
// then a packed minimum with 1 leaves 1 in each half that still holds a mismatch -- seven
// VALU per two records, where a popcount and compare per half took twelve.
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_min1(uint32_t v) {  // per 16-bit half: min(half, 1)
    uint32_t r;
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(v), "v"(0x00010001u));
    return r;
}
template <int kN>  // N when 0..2 (straight-line), -1: the run-time N
__device__ __forceinline__ uint32_t oct_pass8(const uint4 q, uint32_t gg, uint32_t fmask, int N) {
    const uint32_t wv[4] = {q.x, q.y, q.z, q.w};
    uint32_t nz = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t x = gg ^ wv[j];
        u16x2 d = __builtin_bit_cast(u16x2, (x | (x >> 1)) & fmask);
        if constexpr (kN >= 0) {
#pragma unroll
            for (int t = 0; t < kN; ++t) d &= d - (u16x2)(1);
        } else {
            for (int t = 0; t < N; ++t) d &= d - (u16x2)(1);
        }
        nz |= pk_min1(__builtin_bit_cast(uint32_t, d)) << (2 * j);
    }
    const uint32_t p = ~nz;
    return (p & 0x55u) | ((p >> 15) & 0xAAu);
}
// Spare slots of an oct (kDensePad set in the word's half).
__device__ __forceinline__ uint32_t oct_spares(const uint4 q) {
    const uint32_t m = kDensePad | (kDensePad << 16);
    return (uint32_t)__popc((q.x & m) | ((q.y & m) << 1) | ((q.z & m) << 2) | ((q.w & m) << 3));
}

// kSum: the per-key summary's form (Table::dsum_mode: 0 none, 1 N = 0, 2 N = 1), a template
// parameter so the window's two LDS reads (group word, summary) issue together with one wait
// and no branch between them.
template <int kN, int kSum>
__global__ __launch_bounds__(kDenseBlock) void dense_kernel(ScanArgs a) {
    extern __shared__ uint2 s_grp[];
    const uint32_t W = (uint32_t)a.W;
    const uint32_t ngrp = max(1u, (1u << (2 * W)) / 32);
    uint32_t* s_esc = reinterpret_cast<uint32_t*>(s_grp + ngrp);
    uint32_t* s_sum = s_esc + ngrp;  // dsum_mode: 16-bit summary per key, two per word
    zero_sort_counts(a);
    const uint64_t n_supers = a.spans[a.n_spans].super0;
    __shared__ uint32_t s_first;  // the block's first chunks (block_claim, as scan_kernel's)
    if (threadIdx.x == 0 && sched_dynamic(n_supers, kDenseWaves))
        s_first = block_claim(a.counters, a.sched_base, n_supers, kDenseWaves, a.sched_short);
    for (uint32_t i = threadIdx.x; i < ngrp; i += kDenseBlock) {
        s_grp[i] = a.dgrp[i];
        s_esc[i] = a.dgesc[i];
    }
    if (kSum) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(a.dsum);
        for (uint32_t i = threadIdx.x; i < (1u << (2 * W)) / 2; i += kDenseBlock) s_sum[i] = src[i];
    }
    __syncthreads();
    const uint32_t sumF = a.dense_F, sumFB = sumF / 2;

    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const uint64_t stride = (uint64_t)gridDim.x * kDenseWaves;
    const uint32_t shw = 32u - 2u * W;
    const uint32_t fmask = a.dense_M;
    const uint32_t N = (uint32_t)a.N;
    const uint4* __restrict__ octs = reinterpret_cast<const uint4*>(a.dfilt);
    uint32_t ncand = 0;
    SurvChunk C{0, kChunkNone, 0u};

    SuperSched sch;
    uint64_t ss = sch.first(a.counters, a.sched_base, n_supers, w, kDenseWaves, lane, a.sched_short, s_first);
    SeqSpan pf{};
    pf.super0 = 1;
    uint64_t pf_end = 0, pf_sbase = 0;
    uint32_t pf_n = 0;
    auto locate = [&](uint64_t x) {  // wave-uniform x, every lane active
        if (x >= pf.super0 && x < pf_end) return;
        span_find(a, x, lane, pf, pf_end);
        pf_sbase = a.seq_base[pf.seq];
        pf_n = (uint32_t)a.seq_len[pf.seq];
    };
    auto words = [&](uint64_t x, uint64_t& w0, uint64_t& w1, uint64_t& v0, uint64_t& v1) {  // as scan_kernel's
        const uint64_t j = pf_sbase + pf.p_al + (x - pf.super0) * kSuper + (uint64_t)lane * kLanePos;
        w0 = a.g2[j >> 5];
        w1 = a.g2[(j >> 5) + 1];
        v0 = a.ginv[j >> 6];
        v1 = a.ginv[(j >> 6) + 1];
    };
    uint64_t nw0 = 0, nw1 = 0, nv0 = 0, nv1 = 0;
    if (ss < n_supers) {
        locate(ss);
        words(ss, nw0, nw1, nv0, nv1);
    }
    while (ss < n_supers) {
        const SeqSpan sp = pf;
        const uint64_t sbase = pf_sbase;
        const uint32_t n = pf_n;
        const uint64_t w0 = nw0, w1 = nw1;
        const uint32_t base = sp.p_al + (uint32_t)(ss - sp.super0) * kSuper;
        const bool owned = (a.g_lo == 0 || sbase + base >= a.g_lo + 65536u) && sbase + base + kSuper <= a.g_hi;
        const uint32_t pb = base + (uint32_t)lane * kLanePos;
        const uint64_t iv = inv_join(nv0, nv1, (uint32_t)((sbase + pb) & 32u));
        const uint32_t d0 = (uint32_t)(w0 >> 32), d1 = (uint32_t)w0, d2 = (uint32_t)(w1 >> 32);
        const uint32_t okm = window_ok_mask(iv, W) &
                             span_bits(sp, pb);
        // I=1: a window with a non-A/C/G/T/U base among its first 16 sends all its records
        // to the full test (a genome IUPAC base may match where the 2-bit compare says
        // otherwise; under I=0 such a base reads as 'A' and can only hide a mismatch, and U
        // compares as T under I=1)
        const uint32_t slowm = a.I ? ~window_ok_mask(iv, 16u) : 0u;
        const uint64_t nx = sch.next(ss, n_supers, lane);
        (void)stride;
        if (nx < n_supers) {  // next super-step's words, in flight during this one
            locate(nx);
            words(nx, nw0, nw1, nv0, nv1);
        }
        uint32_t escm = 0;
#pragma unroll 1
        for (uint32_t TB = 0; TB < 32; TB += kDB) {  // batches of kDB windows
            // window t's 16-base funnel: bases t..t+15 of the lane, from (d0, d1) for t < 16
            const uint32_t dh = TB < 16 ? d0 : d1, dl = TB < 16 ? d1 : d2;
            uint4 q[kDB];
            uint32_t live = 0;
#pragma unroll
            for (int T = 0; T < kDB; ++T) {
                const uint32_t r = 2u * ((TB + (uint32_t)T) & 15u);
                const uint32_t h = (r ? __builtin_amdgcn_alignbit(dh, dl, 32u - r) : dh) >> shw;
                const uint2 L = s_grp[h >> 5];
                const uint32_t smw = kSum ? s_sum[h >> 1] : 0u;  // issued beside the group word
                const uint32_t bq = h & 31u;
                const uint32_t wb = 31u - (TB + (uint32_t)T);
                const bool ok = (okm >> wb) & 1u;
                // bitwise, not short-circuit: no branch may sink the summary read below the
                // group word's wait
                uint32_t inlb = (okm >> wb) & (L.x >> bq) & 1u;
                if constexpr (kSum != 0) {  // the key's summary: no record can pass -> no oct load
                    const uint32_t sm = smw >> ((h & 1u) << 4);
                    const uint32_t key = r ? __builtin_amdgcn_alignbit(dh, dl, 32u - r) : dh;
                    const uint32_t gf = (key << (2 * W)) >> (32u - 2u * sumF);  // bases W..W+F-1
                    const uint32_t sb = kSum == 1
                                            ? sm >> dsum_hash4(gf)
                                            : (sm >> dsum_hash3(gf >> (2u * sumFB))) |
                                                  (sm >> (8u + dsum_hash3(gf & ((1u << (2u * sumFB)) - 1u))));
                    inlb &= sb | (slowm >> wb);
                }
                const bool inl = inlb != 0u;
                if ((int32_t)L.y < 0 && ok)  // the group holds a key of more than eight records
                    escm |= ((s_esc[h >> 5] >> bq) & 1u) << wb;
                live |= (uint32_t)inl << T;
                q[T] = octs[inl ? (L.y & 0x7FFFFFFFu) + (uint32_t)__popc(L.x & ((1u << bq) - 1u)) : 0u];
            }
            uint64_t pm = 0;
#pragma unroll
            for (int T = 0; T < kDB; ++T) {
                // window bases W..W+F-1 (F <= 7, W + F <= 16: inside the window's funnel),
                // in both 16-bit halves
                const uint32_t r = 2u * ((TB + (uint32_t)T) & 15u);
                const uint32_t key = r ? __builtin_amdgcn_alignbit(dh, dl, 32u - r) : dh;
                const uint32_t gwin = (key << (2 * W)) >> 16;
                const uint32_t gg = gwin | (gwin << 16);
                const bool lv = (live >> T) & 1u;
                const bool sl = (slowm >> (31u - (TB + (uint32_t)T))) & 1u;
                const uint32_t pbits = oct_pass8<kN>(q[T], gg, fmask, (int)N);
                pm |= (uint64_t)(lv ? (sl ? 0xFFu : pbits) : 0u) << (8 * T);
#ifdef MP_DENSE_SLOT_STATS  // timing only: every filled slot of every loaded oct counted
                ncand += lv ? 8u - oct_spares(q[T]) : 0u;
#endif
            }
            if (__any(pm != 0)) dense_full_tests(a, pm, s_grp, 0u, TB, pb, w0, w1, iv, sbase, n, owned, sp.seq, lane, C, ncand);
        }
        // buckets of more than eight records (rare): walked oct by oct through binfo
        while (__any(escm != 0)) {
            uint32_t wi = 0, first = 0, cnt = 0;
            if (escm) {
                wi = (uint32_t)__clz(escm);
                escm &= ~(0x80000000u >> wi);
                const uint32_t h = (uint32_t)((wi ? (w0 << (2 * wi)) | (w1 >> (64 - 2 * wi)) : w0) >> (64 - 2 * W));
                const uint2 rw = a.rk[h >> 5];
                const uint2 bi = a.binfo[rw.y + (uint32_t)__popc(rw.x & ((1u << (h & 31u)) - 1u))];
                first = bi.x;
                cnt = bi.y;
            }
            const bool sl = (slowm >> (31 - wi)) & 1u;
            const uint32_t tb = wi;  // full tests index windows from tb: one window per pass
            for (uint32_t c0 = 0; __any(c0 < cnt); c0 += kDenseOct) {
                uint32_t ob = 0;
                uint64_t pm = 0;
                if (c0 < cnt) {
                    ob = (first + c0) / kDenseOct;
                    const uint4 qq = octs[ob];
                    const uint32_t gwin = (uint32_t)(((wi ? (w0 << (2 * wi)) | (w1 >> (64 - 2 * wi)) : w0) << (2 * W)) >> 48);
                    const uint32_t gg = gwin | (gwin << 16);
                    const uint32_t wv[4] = {qq.x, qq.y, qq.z, qq.w};
#pragma unroll
                    for (int h2 = 0; h2 < 4; ++h2) {
                        const uint32_t x = gg ^ wv[h2];
                        const uint32_t d = (x | (x >> 1)) & fmask;
                        const bool p0 = (uint32_t)__popc(d & 0xFFFFu) <= N || (wv[h2] & kDenseAlways);
                        const bool p1 = (uint32_t)__popc(d >> 16) <= N || ((wv[h2] >> 16) & kDenseAlways);
                        const uint32_t pad0 = (wv[h2] >> 1) & 1u, pad1 = (wv[h2] >> 17) & 1u;
                        pm |= ((uint64_t)((p0 || sl) && !pad0) << (2 * h2)) | ((uint64_t)((p1 || sl) && !pad1) << (2 * h2 + 1));
#ifdef MP_DENSE_SLOT_STATS
                        ncand += (1u - pad0) + (1u - pad1);
#endif
                    }
                }
                if (__any(pm != 0)) dense_full_tests(a, pm, nullptr, ob, tb, pb, w0, w1, iv, sbase, n, owned, sp.seq, lane, C, ncand);
            }
        }
        ss = nx;
    }
    close_chunked(a.surv, a.surv_cap, lane, C);
    add_stats(a, ncand, lane == 0 ? C.total : 0u, lane);
}

// Bucket tails: one lane per reference left by the scan (a seed whose key names more
// than one record).  The lane walks the bucket's other records in order -- each is the
// same (seed position, record) candidate the reference's loop over sts_table[h] tests
// (engine.py:480-489) -- and appends fingerprint survivors to the survivor list.
// Survivors of a tail_kernel block collect in LDS and leave in batches with one
// returning atomic: one per wave-iteration would serialise on the single list counter
// (returning atomics on one address: ~88 per microsecond, MI355X_MICROARCH.md).
// 1024-thread blocks, two per CU: each block's survivors leave with one returning atomic on
// the survivor counter per flush, and those serialise at one address (~11 ns each), so
// 512 blocks where 2,048 smaller ones spent ~20 us on them at the kernel's end.
#ifndef MP_TAIL_BLOCK
#define MP_TAIL_BLOCK 1024
#endif
constexpr uint32_t kTailBlock = MP_TAIL_BLOCK;
#ifndef MP_TAIL_BUF
#define MP_TAIL_BUF 4096
#endif
constexpr uint32_t kTailBuf = MP_TAIL_BUF;
static_assert(kKeyRef == 0x80000000u, "key references: bucket field 2^31 (ents indices are below)");
__device__ __forceinline__ void tail_flush(const ScanArgs& a, uint4* buf, uint32_t& n_sh,
                                           unsigned long long& base_sh) {
    __syncthreads();
    const uint32_t cnt = min(n_sh, kTailBuf);
    if (threadIdx.x == 0 && cnt) base_sh = atomicAdd(&a.counters[2], (unsigned long long)cnt);
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < cnt; t += blockDim.x)
        if (base_sh + t < a.surv_cap) a.surv[base_sh + t] = buf[t];
    __syncthreads();
    if (threadIdx.x == 0) n_sh = 0;
    __syncthreads();
}

// The seed key of a 16-B key reference v (ref16_make: the window at the seed in v.z, v.w).
template <bool kGap>
__device__ __forceinline__ uint32_t ref16_key(const ScanArgs& a, const uint4& v) {
    const uint32_t W = (uint32_t)a.W;
    return kGap ? gap_key(v.w, a.gap_at, a.gap_len) >> (32u - 2u * W) : v.w >> (32u - 2u * W);
}

// kGap: the references of a gapped seed scan (split tables): the key is the gapped one, and a
// window whose gap matches the record exactly is left to the contiguous seed's scan.
// One reference per thread.  (Round 4 measured two and four per thread with their head loads
// in flight together: c4's ~16M key references took 0.33-0.37 ms either way, bound by the
// references' own traffic, and c3's / c5's tails took 17 us longer in that form.)
#ifndef MP_TAIL_BPC
#define MP_TAIL_BPC 2
#endif
constexpr uint32_t kTailBPC = MP_TAIL_BPC;  // blocks per CU
// At most this many passes of 1,024 references between two checks of the block's survivor
// buffer (round 5; a check is two barriers, and a barrier waits for the block's slowest wave:
// c4's tail spent 67 of its 312 us in the buffer and its barriers, ablation 82).  c4 tail, one
// check per 1 / 2 / 4 / 8 / 16 passes: 0.315 / 0.298 / 0.283 / 0.271 / 0.264 ms.
#ifndef MP_TAIL_CHECK
#define MP_TAIL_CHECK 16
#endif
constexpr uint32_t kTailCheck = MP_TAIL_CHECK;
#ifndef MP_TAIL_PREFETCH
#define MP_TAIL_PREFETCH 1
#endif
constexpr bool kTailPrefetch = MP_TAIL_PREFETCH != 0;  // the next pass's 16-B reference and rank word in flight
// kH12: the table has wide key groups (kgrp4), whose key references read the 8-B IUPAC heads
// kRef16: the references are in the 16-B form (ScanArgs::ref16).
template <bool kGap = false, bool kH12 = false, bool kRef16 = false>
__global__ __launch_bounds__(kTailBlock) void tail_kernel(ScanArgs a) {
    __shared__ uint4 s_buf[kTailBuf];
    __shared__ uint32_t s_n;
    __shared__ unsigned long long s_base;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint64_t n_refs = umin64(a.tail_static + a.counters[a.tail_ctr], a.tails_cap);
    const uint64_t* exc = a.has_u ? a.gexc : a.ginv;
    uint32_t ncand = 0, nsurv = 0;
    // key references of a table with wide key groups: the 8-B IUPAC heads (kgrp_pass4); a run-time
    // choice here cost c3's tail 17 us
    const uint2* kref_heads = kH12 ? a.dents12 : a.dents8;
    const uint64_t stride = (uint64_t)gridDim.x * kTailBlock;
    uint32_t it = 0, next_check = 0, period = 1, fill0 = 0;  // buffer checks (block-uniform)
    // 16-B references: the next pass's reference is loaded at the top of this pass, so its
    // latency hides behind this pass's dependent loads (rank word, head, entries)
    // and the reference's rank word is loaded at the end of the pass before (one dependent
    // load fewer on each pass's chain)
    uint4 vnext = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u);
    uint2 rwnext = make_uint2(0u, 0u);
    if (kRef16 && kTailPrefetch && (uint64_t)blockIdx.x * kTailBlock + threadIdx.x < n_refs) {
        vnext = a.tails[(uint64_t)blockIdx.x * kTailBlock + threadIdx.x];
        if (!(vnext.x == 0xFFFFFFFFu && vnext.y == 0xFFFFFFFFu)) rwnext = a.rk[ref16_key<kGap>(a, vnext) >> 5];
    }
    for (uint64_t b = (uint64_t)blockIdx.x * kTailBlock; b < n_refs; b += stride, ++it) {  // block-uniform
        const uint64_t i = b + threadIdx.x;
        uint4 v = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u), w = make_uint4(0u, 0u, 0u, 0u);
        uint2 rwpre = make_uint2(0u, 0u);  // the rank word of v, loaded the pass before
        if (kRef16) {
            // 16-B key reference (ref16_make) -> the 32-B form's fields: the bases left from the
            // sequence tables, the window's exception bits from the genome when flagged
            if constexpr (kTailPrefetch) {
                v = vnext;
                rwpre = rwnext;
                vnext = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u);
                if (i + stride < n_refs) vnext = a.tails[i + stride];
            } else if (i < n_refs) {
                v = a.tails[i];
            }
            if (!(v.x == 0xFFFFFFFFu && v.y == 0xFFFFFFFFu)) {
                const uint64_t gp = (uint64_t)v.x | ((uint64_t)(v.y & 0xFFu) << 32);
                const uint32_t seq = v.y >> 9;
                w.x = v.z;
                w.y = v.w;
                w.z = (v.y & 0x100u) ? (uint32_t)(ext1(exc, gp) >> 32) : 0u;
                w.w = (uint32_t)(a.seq_len[seq] - (gp - a.seq_base[seq]));
                v = make_uint4(v.x, v.y & 0xFFu, kKeyRef, seq);
            }
        } else if (i < n_refs) {
            v = a.tails[2 * i];
            w = a.tails[2 * i + 1];
        }
        if (!(v.x == 0xFFFFFFFFu && v.y == 0xFFFFFFFFu)) {
            const uint64_t gp = (uint64_t)v.x | ((uint64_t)v.y << 32);
            const uint64_t Gs = (uint64_t)w.x | ((uint64_t)w.y << 32);  // window at the seed
            const uint32_t rem = w.w;                                    // bases from the seed to the end
            uint32_t first = v.z;
            Entry e;
            if (v.z == kKeyRef) {  // a seed that passed the key groups: its bucket by key rank
                const uint32_t W = (uint32_t)a.W;
                const uint32_t h = kGap ? gap_key((uint32_t)(Gs >> 32), a.gap_at, a.gap_len) >> (32u - 2u * W)
                                        : (uint32_t)(Gs >> (64u - 2u * W));
                const uint2 rw = (kRef16 && kTailPrefetch) ? rwpre : a.rk[h >> 5];
                const uint2 c = kref_heads[rw.y + (uint32_t)__popc(rw.x & ((1u << (h & 31u)) - 1u))];
                if (c.y & kHead8Full) {
                    first = c.x;  // the bucket's first entry
                    if (c.y & kHead8Filt) {  // none of the bucket's records within N on bases W..W+F-1: done
                        const uint32_t cnt = ((c.y >> 28) & 3u) + 1u;
                        const uint32_t F = head8_filt_bases(cnt);
                        const uint32_t fm = (1u << (2u * F)) - 1u;
                        const uint32_t gf = (uint32_t)((Gs << (2u * W)) >> (64u - 2u * F));
                        const uint32_t xf = w.z & (0xFFFFFFFFu >> W) & ~(0xFFFFFFFFu >> (W + F));
                        bool any = xf != 0u;
                        for (uint32_t j = 0; j < cnt; ++j) {
                            const uint32_t xj = gf ^ ((c.y >> (2u * F * j)) & fm);
                            any = any || __popc((xj | (xj >> 1)) & 0x55555555u) <= a.N;
                        }
                        if (!any) first = 0xFFFFFFFFu;
                    }
                    if (first != 0xFFFFFFFFu) e = a.ents[first];
                    else e.count = 0;
                } else {
                    if constexpr (kH12) e = head12_entry(c, h, W);
                    else e = head8_entry(c, h, W);
                }
            } else {
                e = a.ents[first];                                       // its count = tail length
            }
            const uint32_t cnt = e.count;
            for (uint32_t j = 0; j < cnt; ++j) {
                if (j) e = a.ents[first + j];
                const uint64_t gk = gp - e.hash_off;
                if ((uint32_t)e.l1 > rem + e.hash_off || gk < a.g_lo || gk >= a.g_hi) continue;  // k + l1 > n / not owned
                uint64_t G = Gs;
                uint32_t ex = w.z;
                if (e.hash_off) {  // seed inside the primer: bounds and window from the genome
                    const uint64_t sbase = a.seq_base[v.w];
                    if (gp - sbase < e.hash_off) continue;  // k < 0
                    G = ext2(a.g2, gk);
                    ex = (uint32_t)(ext1(exc, gk) >> 32);
                }
                if constexpr (kGap) {  // a window whose gap matches exactly is the contiguous seed's
                    const uint64_t gm = sp_lt((int)(a.gap_at + a.gap_len)) & ~sp_lt((int)a.gap_at);
                    const uint64_t xg = G ^ e.code;
                    const uint32_t inv = a.has_u ? (uint32_t)(ext1(a.ginv, gk) >> 32) : ex;  // A/C/G/T/U are valid
                    const uint32_t im = (0xFFFFFFFFu >> a.gap_at) & ~(0xFFFFFFFFu >> (a.gap_at + a.gap_len));
                    if (((xg | (xg >> 1)) & gm) == 0 && (inv & im) == 0) continue;
                }
                ++ncand;
                bool exact = false;
                if (fp_reject(a, G, ex, e.l1, e.code, e.pmask, exact)) continue;
                ++nsurv;
                const uint4 sv = make_uint4((uint32_t)gk, (uint32_t)(gk >> 32), e.rec | (exact ? 0x80000000u : 0u), v.w);
                const uint32_t at = atomicAdd(&s_n, 1u);
                if (at < kTailBuf) {
                    s_buf[at] = sv;
                } else {  // block buffer full (a burst of survivors): straight to the list
                    const unsigned long long g = atomicAdd(&a.counters[2], 1ull);
                    if (g < a.surv_cap) a.surv[g] = sv;
                }
            }
        }
        if (kRef16 && kTailPrefetch && !(vnext.x == 0xFFFFFFFFu && vnext.y == 0xFFFFFFFFu))
            rwnext = a.rk[ref16_key<kGap>(a, vnext) >> 5];
        // The buffer's fill is read by every thread between two barriers at a check, and the
        // waves run free between checks.  The next check comes after as many passes as the
        // buffer's free half holds at the survivor rate since the last one (1..kTailCheck): c4's
        // ~130 survivors per pass check every 16 passes; a denser table checks every pass, as
        // before round 5, instead of spilling a burst to one global atomic per survivor.
        if (it == next_check) {  // block-uniform
            __syncthreads();
            const uint32_t f = s_n;
            const uint32_t rate = (f - fill0 + period - 1u) / period;
            if (f >= kTailBuf / 4u) tail_flush(a, s_buf, s_n, s_base);  // barriers inside, s_n = 0 after
            else __syncthreads();  // every thread has read s_n before the next pass appends
            fill0 = f >= kTailBuf / 4u ? 0u : f;
            period = max(1u, min(kTailCheck, (kTailBuf / 2u) / max(rate, 1u)));
            next_check = it + period;
        }
    }
    tail_flush(a, s_buf, s_n, s_base);
    add_stats(a, ncand, nsurv, lane);
}

// One wave per fingerprint survivor: exact primer-1 compare unless the fingerprint was
// already exact, then the amplicon pair-check with lanes over the offsets.
// Persistent: each wave strides over the survivor list (empty slots skipped) and stages
// its hits in LDS.
// One 1024-thread block per CU: the LDS stages (9.2 KB per wave) allow 16 waves per CU in
// any block shape, and the block's hits leave with one returning atomic on the hit counter
// (256 per launch instead of 1,024 with 4-wave blocks; c4 pair 0.743 -> 0.714 ms).
constexpr int kPairWaves = 16;
constexpr int kPairBlock = kPairWaves * 64;
// kI, kN, kX >= 0: the compare rule's I, N and X as constants (the common configurations;
// -1: the run's).  The generic form spilled 103 SGPRs into VGPR lanes: its exec-mask saves
// for every rule branch and the rule's scalars did not fit.
template <int kI = -1, int kN = -1, int kX = -1>
__global__ __launch_bounds__(kPairBlock, 1) void pair_kernel(ScanArgs a_) {
    ScanArgs a = a_;
    if constexpr (kI >= 0) a.I = kI;
    if constexpr (kN >= 0) a.N = kN;
    if constexpr (kX >= 0) a.X = kX;
    const uint64_t n_surv = umin64(a.counters[2], a.surv_cap);  // written by the scan / tail kernels
    __shared__ HitStage s_st[kPairWaves];
    __shared__ uint64_t s_pst[kPairWaves][kPSlots * MP_PBATCH];
    const int lane = threadIdx.x & 63;
    HitStage& S = s_st[threadIdx.x >> 6];
    if (lane == 0) S.n = 0;
    wave_sync_lds();
    // survivors per wave batch: up to MP_PBATCH, fewer when the list is short, so that
    // every resident wave gets work (a batch is checked one survivor at a time)
    const uint64_t waves = (uint64_t)gridDim.x * kPairWaves;
    // Dynamic batches: survivors cost very different amounts (primer-1 failures leave in
    // the prologue), so a static split left the slowest wave ~1.7x the mean.  Each XCD
    // (blocks x, x+8, ...) owns 1/8 of the batches: its waves take one batch each, then
    // pull the rest from the XCD's own counter (8 counters 256 B apart, ~1.3k atomics each).
    {
        // at least MP_PAIR_MINB survivors per batch (c2, 30k survivors: minimum 4, 16, 32, 64
        // -> 0.049, 0.047, 0.050, 0.057 ms); at most 32 while there are fewer than 128 per
        // wave (batches of 32 halve their try loop over two lane groups: c3 pair 0.111 ->
        // 0.099 ms; c4, 650 per wave, is faster with 64: 0.80 vs 0.83 ms)
        const uint64_t per_wave = (n_surv + waves - 1) / waves;
        const uint32_t db = (uint32_t)umax64(MP_PAIR_MINB, umin64(per_wave < 128 ? 32 : MP_PDYN_BATCH, per_wave));
        const uint64_t nbat = (n_surv + db - 1) / db;
        const uint32_t g = gridDim.x < 8u ? gridDim.x : 8u;  // groups: one per XCD, fewer on small grids
        const uint32_t x = blockIdx.x % g;
        // the group's survivor batches [lo_b, lo_b + ns)
        const uint64_t lo_b = nbat * x / g, ns = nbat * (x + 1) / g - lo_b;
        const uint64_t nw_x = (uint64_t)((gridDim.x - x + g - 1u) / g) * kPairWaves;  // waves of this group
        uint64_t li = (uint64_t)(blockIdx.x / g) * kPairWaves + (threadIdx.x >> 6);
        uint64_t* pst = s_pst[threadIdx.x >> 6];
        // (Round 6: the next batch's claim issued as a batch starts measured slower -- c4 pair
        // 0.345-0.349 -> 0.366 ms, c3 0.075 -> 0.083 ms, profiles/r06d_pair_claim_ab.json: the
        // returning atomic queues behind the XCD's other claims, and vmcnt retires in order, so
        // every wait of the batch's own loads waited for it.)
        while (li < ns) {  // check a batch, then claim the next
            const uint64_t i = (lo_b + li) * db + (uint64_t)lane;
            uint4 v = kEmptySurv;
            if ((uint32_t)lane < db && i < n_surv) v = a.surv[i];
            pair_check_lanes(a, v, db, lane, S, pst);
            unsigned long long c = 0;
            if (lane == 0) c = atomicAdd(&a.counters[kPairQBase + x * kStatStride], 1ull);
            li = nw_x + (uint64_t)__shfl((long long)c, 0, 64);
        }
    }
    // the block's stages leave with one returning atomic: one per wave at the end of the
    // kernel would serialise ~4k atomics on the hit counter (~88 per microsecond)
    __syncthreads();
    __shared__ unsigned long long s_base;
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int q = 0; q < kPairWaves; ++q) tot += s_st[q].n;
        s_base = tot ? atomicAdd(&a.counters[kHitBase + hit_region() * kStatStride], (unsigned long long)tot) : 0ull;
    }
    __syncthreads();
    const int w = threadIdx.x >> 6;
    uint64_t off = s_base;
    for (int q = 0; q < w; ++q) off += s_st[q].n;
    write_hits(a, S, off, lane);
}

// The run's last kernel in order mode 2 (finish_fold: the counters into the device-mapped
// pinned words the host polls, then zeroed for the next run).
__global__ __launch_bounds__(1024) void finish_kernel(unsigned long long* __restrict__ counters, uint32_t n_words,
                                                      unsigned long long* __restrict__ h_out,
                                                      unsigned long long* __restrict__ rcount) {
    finish_fold(counters, n_words, h_out, rcount);
}

__global__ void decode_kernel(const uint64_t* __restrict__ hi, const uint64_t* __restrict__ lo, uint64_t n,
                              const uint64_t* __restrict__ seq_base, const uint64_t* __restrict__ seq_len,
                              uint32_t n_seq, const uint2* __restrict__ rank_rec, mp_hit* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t gk = hi[i];
    const uint64_t l = lo[i];
    uint32_t a = 0, b = n_seq;  // last sequence with base <= gk
    while (b - a > 1) {
        const uint32_t mid = (a + b) >> 1;
        if (seq_base[mid] <= gk) a = mid;
        else b = mid;
    }
    const uint64_t k = gk - seq_base[a];
    const uint2 rr = rank_rec[l >> 32];
    const uint32_t rec = rr.x;
    const int32_t d = try_offset((uint32_t)l);
    const uint64_t len = seq_len[a];
    const uint64_t size = rr.y;
    const uint64_t e = size > len - k ? len - k : size;
    mp_hit h;
    h.pos1 = k;
    h.pos2 = (uint64_t)((int64_t)(k + e) - 1 + d);
    h.seq = a;
    h.rec = rec;
    out[i] = h;
}

// Per-stage events (tail, pair, order timings) only with stage timing on: each event
// recorded between two kernels cost ~6 us of idle GPU (c2 step trace: 6 us gaps between
// kernels with them, none without).  The scan kernel's own pair of events always stays.
#define MID_EVENT(x)                  \
    do {                              \
        if (s->stage_timing) MP_HIP_CHECK(x); \
    } while (0)

static void free_search(Search* s) {
    if (!s) return;
    if (s->pending) {  // a run still owns the buffers: let it drain before they are freed
        if (!s->pend_empty && s->evd) (void)hipEventSynchronize(s->evd);
        s->pending = false;
        if (s->genome && s->genome->n_pending) --s->genome->n_pending;
    }
    hipFree(s->keys); hipFree(s->tmp_hi); hipFree(s->tmp_lo); hipFree(s->out); hipFree(s->sort_tmp);
    hipFree(s->counters); hipFree(s->spans); hipFree(s->bucket);
    hipFree(s->surv);
    hipFree(s->tails);
    hipFree(s->slots);
    if (s->ev0) hipEventDestroy(s->ev0);
    if (s->ev1) hipEventDestroy(s->ev1);
    if (s->ev2) hipEventDestroy(s->ev2);
    if (s->ev3) hipEventDestroy(s->ev3);
    if (s->evt) hipEventDestroy(s->evt);
    if (s->evd) hipEventDestroy(s->evd);
    if (s->h_cnt) hipHostFree(s->h_cnt);
    if (s->h_put) hipHostFree(s->h_put);
    if (s->put_ev) {
        for (uint32_t i = 0; i < kPutRing; ++i)
            if (s->put_ev[i]) hipEventDestroy(s->put_ev[i]);
        delete[] s->put_ev;
    }
    if (s->put_done) hipEventDestroy(s->put_done);
    delete s;
}

static int alloc_hits(Search* s, uint64_t cap) {
    cap = (cap + kHitRegions - 1) / kHitRegions * kHitRegions;  // whole regions
    hipFree(s->keys); hipFree(s->tmp_hi); hipFree(s->tmp_lo); hipFree(s->out);
    s->keys = s->tmp_hi = s->tmp_lo = nullptr;
    s->out = nullptr;
    s->cap = 0;
    MP_HIP_CHECK(hipMalloc(&s->keys, cap * 16));
    MP_HIP_CHECK(hipMalloc(&s->tmp_hi, cap * 8));
    MP_HIP_CHECK(hipMalloc(&s->tmp_lo, cap * 8));
    MP_HIP_CHECK(hipMalloc(&s->out, cap * sizeof(mp_hit)));
    s->cap = cap;
    return MP_OK;
}

static int alloc_surv(Search* s, uint64_t cap) {
    hipFree(s->surv);
    s->surv = nullptr;
    s->surv_cap = 0;
    MP_HIP_CHECK(hipMalloc(&s->surv, cap * sizeof(uint4)));
    s->surv_cap = cap;
    return MP_OK;
}

static int alloc_tails(Search* s, uint64_t cap) {
    hipFree(s->tails);
    s->tails = nullptr;
    s->tails_cap = 0;
    MP_HIP_CHECK(hipMalloc(&s->tails, cap * 2 * sizeof(uint4)));
    s->tails_cap = cap;
    return MP_OK;
}

// dense_kernel's dynamic LDS for table t: the per-32-key index and escape words, plus the
// per-key summary when the table has one.
static size_t dense_lds_of(const Table* t) {
    size_t b = (sizeof(uint2) + sizeof(uint32_t)) *
               std::max<size_t>(1, ((size_t)1 << (2 * std::min<int>(t->prm.wordsize, kDenseMaxW))) / 32);
    if (t->dsum_mode) b += sizeof(uint16_t) * ((size_t)1 << (2 * t->prm.wordsize));
    return b;
}

// (the tail list's first 64 slots per scan wave are static: 262,144 on a full-chip grid, per
// half of a split run)
constexpr uint64_t kDefaultHitCap = 1 << 16, kDefaultSurvCap = 1 << 20, kDefaultTailCap = 1 << 20;

}  // namespace mp

using namespace mp;

MP_EXPORT int mp_search_set_stage_timing(void* search, int32_t on) {
    Search* s = (Search*)search;
    if (!s) return fail(MP_E_ARG, "mp_search_set_stage_timing: null search");
    s->stage_timing = on != 0;
    return MP_OK;
}

MP_EXPORT int mp_search_set_options(void* search, const mp_search_options* opt) {
    Search* s = (Search*)search;
    if (!s || !opt) return fail(MP_E_ARG, "mp_search_set_options: null pointer");
    if (s->pending) return fail(MP_E_STATE, "mp_search_set_options: a run is enqueued");
    if (opt->tails < MP_TAILS_AUTO || opt->tails > MP_TAILS_KERNEL || opt->sort < MP_SORT_AUTO ||
        opt->sort > MP_SORT_SCATTER || opt->sort_bucket_bits < 0 || opt->sort_bucket_bits > 16 ||
        opt->pair_blocks_per_cu < 0 || opt->generic_forms < 0 ||
        opt->generic_forms > (int32_t)(MP_GENERIC_FIX | MP_GENERIC_GAP | MP_GENERIC_PAIR) || opt->ref32 < 0 ||
        opt->ref32 > 1 || opt->sched_short < 0 || opt->sched_short > 64 || opt->crowd_grid < 0 || opt->scan_grid < 0)
        return fail(MP_E_ARG, "mp_search_set_options: option out of range");
    MP_HIP_CHECK(hipSetDevice(s->genome->device));
    s->opt = *opt;
    s->order_mode = opt->sort == MP_SORT_SCATTER ? 1 : 0;
    int rc = alloc_hits(s, opt->hit_cap ? opt->hit_cap : kDefaultHitCap);
    if (!rc) rc = alloc_surv(s, opt->surv_cap ? opt->surv_cap : kDefaultSurvCap);
    if (!rc) rc = alloc_tails(s, opt->tail_cap ? opt->tail_cap : kDefaultTailCap);
    return rc;
}

MP_EXPORT int mp_search_create(void* table, void* genome, void** out) {
    if (!table || !genome || !out) return fail(MP_E_ARG, "mp_search_create: null pointer");
    *out = nullptr;
    Table* t = (Table*)table;
    Genome* g = (Genome*)genome;
    if (t->device != g->device) return fail(MP_E_ARG, "mp_search_create: table and genome on different devices");
    Search* s = new Search();
    s->table = t;
    s->genome = g;
    int rc = MP_OK;
    do {
        if (hipSetDevice(g->device) != hipSuccess) { rc = fail(MP_E_HIP, "hipSetDevice failed"); break; }
        if (hipMalloc(&s->counters, kCounterBytes) != hipSuccess) { rc = fail(MP_E_NOMEM, "counter allocation failed"); break; }
        if (hipDeviceGetAttribute(&s->n_cu, hipDeviceAttributeMultiprocessorCount, g->device) != hipSuccess ||
            s->n_cu <= 0)
            s->n_cu = 256;
        int occ = 0;  // persistent pair check: every resident block slot once
        s->pair_per_cu = (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, pair_kernel<>, kPairBlock, 0) == hipSuccess && occ > 0)
                             ? (uint32_t)occ : 1u;
        s->dense_lds = dense_lds_of(t);
        if (t->split_rest) s->dense_lds = std::max(s->dense_lds, dense_lds_of(t->split_rest));
        if (s->dense_lds > 64 * 1024)
            for (const void* k : {(const void*)dense_kernel<0, 0>, (const void*)dense_kernel<0, 1>,
                                  (const void*)dense_kernel<1, 0>, (const void*)dense_kernel<1, 2>,
                                  (const void*)dense_kernel<2, 0>, (const void*)dense_kernel<-1, 0>})
                (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)s->dense_lds);
        occ = 0;
        s->dense_per_cu = (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, dense_kernel<1, 2>, kDenseBlock, s->dense_lds) ==
                               hipSuccess && occ > 0) ? (uint32_t)occ : 1u;
        if (hipEventCreate(&s->ev0) != hipSuccess || hipEventCreate(&s->ev1) != hipSuccess ||
            hipEventCreate(&s->ev2) != hipSuccess || hipEventCreate(&s->ev3) != hipSuccess ||
            hipEventCreate(&s->evt) != hipSuccess ||
            hipEventCreateWithFlags(&s->evd, hipEventDisableTiming) != hipSuccess) {
            rc = fail(MP_E_HIP, "event creation failed");
            break;
        }
        // device-mapped pinned words: finish_kernel writes the run's counters straight into them
        if (hipHostMalloc((void**)&s->h_cnt, kHostWords * sizeof(unsigned long long), hipHostMallocMapped) != hipSuccess ||
            hipHostGetDevicePointer((void**)&s->d_hcnt, (void*)s->h_cnt, 0) != hipSuccess) {
            rc = fail(MP_E_NOMEM, "pinned counter allocation failed");
            break;
        }
        std::memset((void*)s->h_cnt, 0, kHostWords * sizeof(unsigned long long));
        if (hipMemset(s->counters, 0, kCounterBytes) != hipSuccess) { rc = fail(MP_E_HIP, "counter reset failed"); break; }
        rc = alloc_hits(s, kDefaultHitCap);
        if (!rc) rc = alloc_surv(s, kDefaultSurvCap);
        if (!rc) rc = alloc_tails(s, kDefaultTailCap);
        if (!rc) rc = alloc_sort_buckets(s);
    } while (0);
    if (rc) {
        free_search(s);
        return rc;
    }
    *out = s;
    return MP_OK;
}

namespace mp {

static_assert(sizeof(ScanArgs) <= sizeof(Search::pend_args), "ScanArgs fits the pending-run slot");

// The list pointers, capacities and hit-order fields of a run in order mode `mode`.
static int set_lists(Search* s, ScanArgs& a, int mode) {
    a.hit_hi = s->keys;
    a.hit_lo = s->keys + s->cap;
    a.counters = s->counters;
    a.cap = s->cap;
    a.cap_r = s->cap / kHitRegions;
    a.surv = s->surv;
    a.surv_cap = s->surv_cap;
    a.tails = s->tails;
    a.tails_cap = s->tails_cap;
    a.sort_cnt = nullptr;
    a.sort_keys = nullptr;
    a.sort_slots = nullptr;
    a.sort_nb = a.sort_shift = a.sort_try_bits = a.sort_low_bits = a.slot_cap = 0;
    if (mode < 2) {  // after a hit-list regrowth too: the plan follows the capacity
        const SortPlan P = sort_plan(s);
        a.sort_cnt = sort_bucket_counts(s);
        a.sort_keys = s->tmp_lo;
        a.sort_nb = P.nb;
        a.sort_shift = P.shift;
        a.sort_try_bits = P.try_bits;
        a.sort_low_bits = P.low_bits;
        if (mode == 0) {
            const int rc = alloc_sort_slots(s, P);
            if (rc) return rc;
            a.sort_slots = s->slots;
            a.slot_cap = P.slot_cap;
        }
    }
    return MP_OK;
}

// Every kernel of one run, back to back on the stream with no host wait: scan -> fingerprint
// survivors (+ bucket-tail references -> tail survivors) -> pair check -> hit keys and bucket
// counts -> hit order (modes 0 and 1: bucket offsets, then the sort) ->
// finish_kernel (counters into the mapped host words, then zeroed) -> the completion event.
// The scan-side fields of table t (its seeds, filters and heads); the record side (recs,
// ranks, primer planes) stays the searched table's.
static void scan_fields(ScanArgs& a, const Table* t, const Search* s) {
    a.binfo = t->binfo; a.dfilt = t->dfilt; a.dgrp = t->dgrp; a.dgesc = t->dgesc; a.dents_pad = t->dents_pad; a.dense_M = t->dense_M;
    a.dsum = t->dsum; a.dsum_mode = t->dsum_mode; a.dense_F = t->dense_F;
    a.defer_full = t->defer_full && (!s->opt.no_defer || t->gap_len);
    a.kgrp = reinterpret_cast<const uint2*>(t->kgrp); a.kgrp_F = t->kgrp_F; a.kgrp_wild = t->kgrp_wild;
    a.kgrp4 = t->kgrp4;
    a.filt = t->filt; a.filt_log2 = t->filt_log2; a.rk = t->rk; a.dents = t->dents; a.dents8 = t->dents8; a.dents16 = t->dents16; a.dents12 = t->dents12; a.lfilt = t->lfilt;
    a.slots = t->slots; a.slot_log2 = t->slot_log2;
    a.ents = t->ents;
    a.W = t->prm.wordsize;
    a.gap_at = t->gap_at;
    a.gap_len = t->gap_len;
    a.gap_post = t->gap_post;
}

// The scan of table t takes the wide I = 1 key groups (kgrp4); its key references are opened by
// tail_kernel through the 8-B IUPAC heads.
static bool scan_uses_kgrp4(const Search* s, const Table* t, const ScanArgs& a) {
    const bool inl = (t->n_rec > t->n_keys + t->n_keys / 4 || s->opt.tails == MP_TAILS_INLINE) &&
                     s->opt.tails != MP_TAILS_KERNEL;
    const bool dense = (uint32_t)t->prm.wordsize <= kDenseMaxW && !s->opt.no_dense;
    return t->kgrp4 && a.I == 1 && !s->opt.no_rank_filter && t->filt_direct && !t->lds_exact && a.W >= 11 &&
           a.W <= 13 && a.defer_full && t->h12 && !t->gap_len && !inl && !dense;
}

// The scan kernel of table t (dense_kernel, or scan_kernel in the form the table and the
// handle's options select).  *tail: the run needs tail_kernel over this scan's references.
static void launch_fixed(int fix, uint32_t grid, hipStream_t st, const ScanArgs& a) {
    if (fix == 1) hipLaunchKernelGGL((scan_kernel<1, false, 2, true, 0, 1, 0, 1>), dim3(grid), dim3(kBlock), 0, st, a);
    else hipLaunchKernelGGL((scan_kernel<1, false, 2, true, 0, 1, 0, 2>), dim3(grid), dim3(kBlock), 0, st, a);
}

static void launch_fixed4(int fix, uint32_t grid, hipStream_t st, const ScanArgs& a) {
    if (fix == 1) hipLaunchKernelGGL((scan_kernel<1, false, 2, true, 0, 2, 0, 1>), dim3(grid), dim3(kBlock), 0, st, a);
    else if (fix == 2) hipLaunchKernelGGL((scan_kernel<1, false, 2, true, 0, 2, 0, 2>), dim3(grid), dim3(kBlock), 0, st, a);
    else hipLaunchKernelGGL((scan_kernel<1, false, 2, true, 0, 2, 0, 3>), dim3(grid), dim3(kBlock), 0, st, a);
}

// Workgroups of a scan over `tiles` super-steps: one per CU (persistent), at most
// mp_search_options.scan_grid, at most one per kWaves super-steps.
static uint32_t scan_grid_of(const Search* s, uint64_t tiles) {
    uint64_t cap = (uint64_t)s->n_cu * kBlocksPerCU;
    if (s->opt.scan_grid > 0) cap = std::min<uint64_t>(cap, (uint64_t)s->opt.scan_grid);
    return (uint32_t)std::min<uint64_t>((tiles + kWaves - 1) / kWaves, cap);
}

// *ref16: the run's key references are in the 16-B form (the key-group scans; a0.ref16 says
// whether the genome allows it), as the tail pass must read them.
static int launch_scan(Search* s, const Table* t, const ScanArgs& a0, uint64_t tiles, hipStream_t st, bool* tail,
                       uint32_t* ref16) {
    ScanArgs a = a0;
    const uint32_t grid = scan_grid_of(s, tiles);
    *tail = false;
    *ref16 = 0;
    if (t->gap_len) {  // gapped seed: the key-group path, every passing seed deferred to tail_kernel
        *ref16 = a.ref16;  // always a key-group form: 16-B references when the genome allows them
        if (!(t->filt_direct && !t->lds_exact && t->kgrp_F >= 2 && a.W >= 11 && a.W <= 13 && a.defer_full))
            return fail(MP_E_STATE, "gapped seed table without key groups");
        // c5's shape (W = 8, N = 1) with its gap as constants; other W 7..9 shapes from the table
        const bool w8 = t->gap_at == kGapW8At && t->gap_len == kGapW8Len && t->gap_post == kGapW8Post && a.N == 1 &&
                        t->kgrp_F == kGapW8Len + kGapW8Post && a.W == (int)kSplitSeed &&
                        !(s->opt.generic_forms & MP_GENERIC_GAP);
        if (w8 && t->lds_k == 2) hipLaunchKernelGGL((scan_kernel<1, false, 2, true, false, true, kGapW8>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (w8) hipLaunchKernelGGL((scan_kernel<1, false, 1, true, false, true, kGapW8>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (t->lds_k == 2) hipLaunchKernelGGL((scan_kernel<1, false, 2, true, false, true, 1>), dim3(grid), dim3(kBlock), 0, st, a);
        else hipLaunchKernelGGL((scan_kernel<1, false, 1, true, false, true, 1>), dim3(grid), dim3(kBlock), 0, st, a);
        MP_HIP_CHECK(hipGetLastError());
        *tail = true;
        return MP_OK;
    }
    bool inl = t->n_rec > t->n_keys + t->n_keys / 4;  // bucket tails inline vs tail_kernel
    if (s->opt.tails == MP_TAILS_INLINE) inl = true;
    if (s->opt.tails == MP_TAILS_KERNEL) inl = false;
    // W <= kDenseMaxW: dense_kernel (bucket index in LDS, filter-word octs)
    const bool dense = (uint32_t)t->prm.wordsize <= kDenseMaxW && !s->opt.no_dense;
    // level-2 filter of the filtered rank groups: I = 0 (the 2-bit mismatch count is then a
    // lower bound), compact 8-B heads (not h16)
    // (I = 1: the field form with the non-plain bases marked, kgrp_wild)
    const bool rkf = t->kgrp_F >= 2 && (a.I == 0 ? !t->h16 && !t->kgrp_wild : t->kgrp_wild != 0) &&
                     !s->opt.no_rank_filter && t->filt_direct && !t->lds_exact && a.W >= 11 && a.W <= 13;
    // I = 1 tables whose 8-B fields are too short (c4): the wide key groups
    const bool rkf4 = scan_uses_kgrp4(s, t, a);
    // the I = 0 key-group scan with its shape as constants (kFix: W = 11, F = 6, N <= 1)
    const int fix = (a.W == (int)kFixW && a.I == 0 && !t->kgrp_wild && t->kgrp_F == kFixF && a.N <= 1 &&
                     !(s->opt.generic_forms & MP_GENERIC_FIX)) ? a.N + 1 : 0;
    const int fix4 = (a.W == (int)kFixW && a.N <= 2 && !(s->opt.generic_forms & MP_GENERIC_FIX)) ? a.N + 1 : 0;
    // the forms below that leave key references (kRkf 1 and 2), in the 16-B form: the wide key
    // groups' (rkf4) forms whatever defer_full says, the I = 0 / wild key groups' only when the
    // dispatch below takes them, which needs defer_full -- a table with many full heads runs a
    // kRkf = 0 form, whose 32-B references the 16-B tail pass would misread (round 6: that
    // mismatch was the illegal address of the first 16-B attempts)
    const bool keyref = !dense && !inl && !t->lds_exact && (rkf4 || (rkf && a.defer_full)) &&
                        (t->lds_k == 1 || t->lds_k == 2);
    // (a.ref16, the copy's: a split table's caller passes &pa[i].ref16 as `ref16`, the same
    // object as a0, which the `*ref16 = 0` above has already cleared -- round 6 found the split
    // seeds' scans writing 32-B references for that reason alone)
    a.ref16 = keyref ? a.ref16 : 0u;
    *ref16 = a.ref16;
    if (dense) {
        const uint32_t dgrid = (uint32_t)std::min<uint64_t>((tiles + kDenseWaves - 1) / kDenseWaves,
                                                            (uint64_t)s->n_cu * (uint64_t)s->dense_per_cu);
        const size_t lds = dense_lds_of(t);
        // the summary exists only for N <= 1 (mp_table.hip): N = 0 form 1, N = 1 form 2
        if (a.N == 0 && a.dsum_mode == 1) hipLaunchKernelGGL((dense_kernel<0, 1>), dim3(dgrid), dim3(kDenseBlock), lds, st, a);
        else if (a.N == 0) hipLaunchKernelGGL((dense_kernel<0, 0>), dim3(dgrid), dim3(kDenseBlock), lds, st, a);
        else if (a.N == 1 && a.dsum_mode == 2) hipLaunchKernelGGL((dense_kernel<1, 2>), dim3(dgrid), dim3(kDenseBlock), lds, st, a);
        else if (a.N == 1) hipLaunchKernelGGL((dense_kernel<1, 0>), dim3(dgrid), dim3(kDenseBlock), lds, st, a);
        else if (a.N == 2) hipLaunchKernelGGL((dense_kernel<2, 0>), dim3(dgrid), dim3(kDenseBlock), lds, st, a);
        else hipLaunchKernelGGL((dense_kernel<-1, 0>), dim3(dgrid), dim3(kDenseBlock), lds, st, a);
    } else if (inl) {
        if (t->lds_exact) hipLaunchKernelGGL((scan_kernel<0, true>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (t->filt_direct && t->lds_k == 2) hipLaunchKernelGGL((scan_kernel<1, true, 2>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (t->filt_direct) hipLaunchKernelGGL((scan_kernel<1, true, 1>), dim3(grid), dim3(kBlock), 0, st, a);
        else hipLaunchKernelGGL((scan_kernel<2, true>), dim3(grid), dim3(kBlock), 0, st, a);
    } else {
        if (t->lds_exact) hipLaunchKernelGGL((scan_kernel<0, false>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (rkf4 && t->lds_k == 2 && fix4)  // c4: W = 11, N <= 2 as constants
            launch_fixed4(fix4, grid, st, a);
        else if (rkf4 && t->lds_k == 2)
            hipLaunchKernelGGL((scan_kernel<1, false, 2, true, 0, 2>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (rkf4 && t->lds_k == 1)
            hipLaunchKernelGGL((scan_kernel<1, false, 1, true, 0, 2>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (t->filt_direct && t->lds_k == 2 && a.defer_full && rkf && fix)  // c2 / c3: W = 11, I = 0, N <= 1
            launch_fixed(fix, grid, st, a);
        else if (t->filt_direct && t->lds_k == 2 && a.defer_full && rkf)
            hipLaunchKernelGGL((scan_kernel<1, false, 2, true, false, true>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (t->filt_direct && t->lds_k == 3 && a.defer_full && rkf)  // MP_LDS_K=3 (A/B)
            hipLaunchKernelGGL((scan_kernel<1, false, 3, true, false, true>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (t->filt_direct && t->lds_k == 3 && a.defer_full && t->h12)
            hipLaunchKernelGGL((scan_kernel<1, false, 3, true, 2>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (t->filt_direct && t->lds_k == 3 && a.defer_full && t->h16)
            hipLaunchKernelGGL((scan_kernel<1, false, 3, true, 1>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (t->filt_direct && t->lds_k == 2 && a.defer_full && t->h12)
            hipLaunchKernelGGL((scan_kernel<1, false, 2, true, 2>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (t->filt_direct && t->lds_k == 2 && a.defer_full && t->h16)
            hipLaunchKernelGGL((scan_kernel<1, false, 2, true, 1>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (t->filt_direct && t->lds_k == 2 && a.defer_full)
            hipLaunchKernelGGL((scan_kernel<1, false, 2, true>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (t->filt_direct && t->lds_k == 1 && a.defer_full && rkf)
            hipLaunchKernelGGL((scan_kernel<1, false, 1, true, false, true>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (t->filt_direct && a.defer_full && t->h12)
            hipLaunchKernelGGL((scan_kernel<1, false, 1, true, 2>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (t->filt_direct && a.defer_full && t->h16)
            hipLaunchKernelGGL((scan_kernel<1, false, 1, true, 1>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (t->filt_direct && t->lds_k == 2) hipLaunchKernelGGL((scan_kernel<1, false, 2>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (t->filt_direct && a.defer_full)
            hipLaunchKernelGGL((scan_kernel<1, false, 1, true>), dim3(grid), dim3(kBlock), 0, st, a);
        else if (t->filt_direct) hipLaunchKernelGGL((scan_kernel<1, false, 1>), dim3(grid), dim3(kBlock), 0, st, a);
        else hipLaunchKernelGGL((scan_kernel<2, false>), dim3(grid), dim3(kBlock), 0, st, a);
    }
    MP_HIP_CHECK(hipGetLastError());
    *tail = !dense && !inl && (t->max_bucket > 1 || a.defer_full);  // defer_full: single-record full heads too
    return MP_OK;
}

// Split seeds in use for this handle (kSplitSeed): the table has them and the options leave
// the dense path alone (no_dense or no_split keep the unsplit table's scan).
static bool use_split(const Search* s) {
    return s->table->split_a && !s->opt.no_dense && !s->opt.no_split;
}

// Every kernel of one run, back to back on the stream with no host wait: scan -> fingerprint
// survivors (+ bucket-tail references -> tail survivors) -> pair check -> hit keys and bucket
// counts -> hit order (modes 0 and 1: bucket offsets, then the sort) ->
// finish_kernel (counters into the mapped host words, then zeroed) -> the completion event.
// A split table scans its seeds one after another (the contiguous seed, the gapped seed, the
// rest's dense scan), each appending to the one survivor list; the two seed scans keep their
// bucket-tail references in the two halves of the tail list (counters 4 and 5).
// The bucket-tail pass: the gapped seed's form, or the wide key groups' IUPAC heads.
static void launch_tail(const Search* s, bool gap, bool h12, hipStream_t st, const ScanArgs& a) {
    const dim3 g((uint32_t)s->n_cu * kTailBPC), b(kTailBlock);
    if (a.ref16) {
        if (gap) hipLaunchKernelGGL((tail_kernel<true, false, true>), g, b, 0, st, a);
        else if (h12) hipLaunchKernelGGL((tail_kernel<false, true, true>), g, b, 0, st, a);
        else hipLaunchKernelGGL((tail_kernel<false, false, true>), g, b, 0, st, a);
    } else {
        if (gap) hipLaunchKernelGGL((tail_kernel<true, false>), g, b, 0, st, a);
        else if (h12) hipLaunchKernelGGL((tail_kernel<false, true>), g, b, 0, st, a);
        else hipLaunchKernelGGL((tail_kernel<false, false>), g, b, 0, st, a);
    }
}

static int enqueue_kernels(Search* s, const ScanArgs& a, uint64_t tiles, hipStream_t st, int mode) {
    Table* t = s->table;
    if (s->dirty) {  // an abandoned run may have left counts behind
        MP_HIP_CHECK(hipMemsetAsync(s->counters, 0, kCounterBytes, st));
        s->dirty = false;
    }
    const bool timed = s->scan_timing || s->stage_timing;  // stage times start from the scan's end event
    if (timed) MP_HIP_CHECK(hipEventRecord(s->ev0, st));
    if (!use_split(s)) {
        bool tail = false;
        ScanArgs ta = a;
        const int rc = launch_scan(s, t, a, tiles, st, &tail, &ta.ref16);
        if (rc) return rc;
        if (timed) MP_HIP_CHECK(hipEventRecord(s->evt, st));
        if (tail) {
            launch_tail(s, false, t->kgrp4 != nullptr, st, ta);
            MP_HIP_CHECK(hipGetLastError());
        }
    } else {
        const Table* sub[3] = {t->split_a, t->split_b, t->split_rest};
        ScanArgs pa[3];
        bool tail[3] = {false, false, false};
        const uint64_t half = s->tails_cap / 2;
        for (int i = 0; i < 3; ++i) {
            if (!sub[i]) continue;
            pa[i] = a;
            scan_fields(pa[i], sub[i], s);
            pa[i].tails = s->tails + (i == 1 ? 2 * half : 0);
            pa[i].tails_cap = half;
            pa[i].tail_ctr = i == 1 ? 5u : 4u;
            pa[i].sched_base = i == 0 ? (uint32_t)kSchedBase : (uint32_t)(kSchedSplit + (i - 1) * 8 * kStatStride);
            const int rc = launch_scan(s, sub[i], pa[i], tiles, st, &tail[i], &pa[i].ref16);
            if (rc) return rc;
        }
        if (timed) MP_HIP_CHECK(hipEventRecord(s->evt, st));
        for (int i = 0; i < 3; ++i) {
            if (!sub[i] || !tail[i]) continue;
            launch_tail(s, sub[i]->gap_len != 0, false, st, pa[i]);
            MP_HIP_CHECK(hipGetLastError());
        }
    }
    MID_EVENT(hipEventRecord(s->ev1, st));
    const uint32_t pair_per_cu = s->opt.pair_blocks_per_cu ? std::min(s->pair_per_cu, (uint32_t)s->opt.pair_blocks_per_cu)
                                                           : s->pair_per_cu;
    const dim3 pg((uint32_t)s->n_cu * pair_per_cu);
    const bool pgen = (s->opt.generic_forms & MP_GENERIC_PAIR) != 0;
    if (!pgen && a.I == 0 && a.N == 0 && a.X == 1) hipLaunchKernelGGL((pair_kernel<0, 0, 1>), pg, dim3(kPairBlock), 0, st, a);
    else if (!pgen && a.I == 0 && a.N == 1 && a.X == 1) hipLaunchKernelGGL((pair_kernel<0, 1, 1>), pg, dim3(kPairBlock), 0, st, a);
    else if (!pgen && a.I == 1 && a.N == 2 && a.X == 1) hipLaunchKernelGGL((pair_kernel<1, 2, 1>), pg, dim3(kPairBlock), 0, st, a);
    else hipLaunchKernelGGL(pair_kernel<>, pg, dim3(kPairBlock), 0, st, a);
    MP_HIP_CHECK(hipGetLastError());
    MID_EVENT(hipEventRecord(s->ev2, st));
    if (mode < 2) {  // hit order on the device count: no host round trip before it; its offsets
                     // launch also finishes the run (counters to the host words, then zeroed)
        const int rc = sort_hits_device(s, st, mode, true);
        if (rc) return rc;
    } else {
        hipLaunchKernelGGL(finish_kernel, dim3(1), dim3(1024), 0, st, s->counters, (uint32_t)(kCounterBytes / 8), s->d_hcnt,
                           sort_region_counts(s));
        MP_HIP_CHECK(hipGetLastError());
    }
    MID_EVENT(hipEventRecord(s->ev3, st));
    MP_HIP_CHECK(hipEventRecord(s->evd, st));
    return MP_OK;
}

// The order mode of the next run: keys over 64 bits (or a forced rocPRIM sort) take 2; the
// handle's sticky mode otherwise, except that mode 0's bucket slots (kSlotCap keys per
// bucket) are skipped once the planned mean bucket at the hit capacity is past kSlotCap / 4:
// such runs would overflow a slot and redo their order in mode 1 anyway.
static int run_order_mode(const Search* s) {
    if (!sort_hits_device_ok(s)) return 2;
    int m = s->order_mode;
    if (m == 0) {
        const SortPlan P = sort_plan(s);
        if (s->cap / P.nb > kSlotCap / 4) m = 1;
    }
    return m;
}

// Wait for the enqueued run and read its counters (written by finish_kernel).
static int wait_counts(Search* s, unsigned long long* cnt) {
    MP_HIP_CHECK(poll_event(s->evd));
    std::memcpy(cnt, (const void*)s->h_cnt, kHostWords * sizeof(unsigned long long));
    return MP_OK;
}

// The run's order again, synchronously, one mode up (a bucket overflowed in `from`); raises
// the handle's sticky mode.  The linear keys (tmp_lo; hi/lo for rocPRIM) are intact.
// The sticky mode rises only when a device order overflowed (raise): a run that took mode 2
// because its key was wider than 64 bits leaves the handle's mode alone, so a later genome
// whose key fits goes back to the device order.
static int redo_order(Search* s, hipStream_t st, int from, uint64_t nh, bool raise) {
    Genome* g = s->genome;
    Table* t = s->table;
    for (int mode = from + 1; mode <= 2; ++mode) {
        if (raise) s->order_mode = std::max(s->order_mode, mode);
        if (mode == 1) {
            // the bucket counts and keys are intact; the offsets again (no finish: the host
            // words hold this run's counters), then scatter and sort; an overflow shows in
            // the host word
            s->h_cnt[kSortOverflow] = 0;
            const int rc = sort_hits_device(s, st, 1, false);
            if (rc) return rc;
            MP_HIP_CHECK(hipStreamSynchronize(st));
            if (!s->h_cnt[kSortOverflow]) break;
            continue;
        }
        const uint64_t* hi = nullptr;
        const uint64_t* lo = nullptr;
        const int rc = sort_hits(s, nh, st, &hi, &lo);
        if (rc) return rc;
        if (nh) {
            const uint32_t blocks = (uint32_t)((nh + 255) / 256);
            hipLaunchKernelGGL(decode_kernel, dim3(blocks), dim3(256), 0, st, hi, lo, nh,
                               g->d_base, g->d_len, g->n_seq, t->rank_rec, s->out);
            MP_HIP_CHECK(hipGetLastError());
        }
        MP_HIP_CHECK(hipStreamSynchronize(st));
    }
    return MP_OK;
}

static int search_complete(Search* s, uint64_t* n_hits) {
    hipStream_t st = s->pend_st;
    ScanArgs& a = *reinterpret_cast<ScanArgs*>(s->pend_args);
    const int mode0 = s->pend_mode;
    int mode = mode0;
    unsigned long long cnt[kHostWords];
    int rc = wait_counts(s, cnt);
    if (rc) return rc;
    if (s->scan_timing || s->stage_timing) MP_HIP_CHECK(hipEventElapsedTime(&s->scan_ms, s->ev0, s->evt));
    else s->scan_ms = -1.f;
    MID_EVENT(hipEventElapsedTime(&s->tail_ms, s->evt, s->ev1));
    // A list that overflowed is grown and the whole run enqueued again (rare: the first runs of
    // a handle); kernels never write past a capacity.
    // (the hit list overflows when one of its regions does: cnt[kHitMaxRegion] > cap / kHitRegions)
    // (a split run's two seed scans each hold half the tail list: counters 4 and 5)
    // (each list, or half, starts with a.tail_static static slots)
    auto tails_need = [&]() {
        return use_split(s) ? 2 * (a.tail_static + std::max(cnt[4], cnt[5])) : a.tail_static + cnt[4];
    };
    for (int attempt = 0;
         cnt[2] > s->surv_cap || tails_need() > s->tails_cap || cnt[kHitMaxRegion] > s->cap / kHitRegions; ++attempt) {
        if (attempt == 3) return fail(MP_E_STATE, "mp_search_run: list overflow after growth");
        ++s->n_regrowths;
        if (tails_need() > s->tails_cap) rc = alloc_tails(s, tails_need() + tails_need() / 4 + 1024);
        if (!rc && cnt[2] > s->surv_cap) rc = alloc_surv(s, cnt[2] + cnt[2] / 2 + 1024);
        if (!rc && cnt[kHitMaxRegion] > s->cap / kHitRegions) {
            const uint64_t mx = cnt[kHitMaxRegion];
            rc = alloc_hits(s, kHitRegions * (mx + mx / 4 + 1024));
        }
        mode = run_order_mode(s);
        if (!rc) rc = set_lists(s, a, mode);
        if (!rc) rc = enqueue_kernels(s, a, s->pend_tiles, st, mode);
        if (!rc) rc = wait_counts(s, cnt);
        if (rc) return rc;
        if (s->scan_timing || s->stage_timing) MP_HIP_CHECK(hipEventElapsedTime(&s->scan_ms, s->ev0, s->evt));
        MID_EVENT(hipEventElapsedTime(&s->tail_ms, s->evt, s->ev1));
    }
    (void)mode0;
    MID_EVENT(hipEventElapsedTime(&s->pair_ms, s->ev1, s->ev2));
    MID_EVENT(hipEventElapsedTime(&s->order_ms, s->ev2, s->ev3));
    s->n_candidates = cnt[1];
    s->n_survivors = cnt[3];
    const uint64_t nh = cnt[0];
    if (mode == 2 || cnt[kSortOverflow]) {  // the device order did not hold this run's keys
        rc = redo_order(s, st, mode == 2 ? 1 : mode, nh, cnt[kSortOverflow] != 0);
        if (rc) return rc;
    }
    if (!s->stage_timing) s->tail_ms = s->pair_ms = s->order_ms = -1.f;  // not measured
    s->n_hits = nh;
    if (n_hits) *n_hits = nh;
    return MP_OK;
}

}  // namespace mp

MP_EXPORT int mp_search_set_scan_timing(void* search, int32_t on) {
    Search* s = (Search*)search;
    if (!s) return fail(MP_E_ARG, "mp_search_set_scan_timing: null search");
    s->scan_timing = on != 0;
    return MP_OK;
}

MP_EXPORT int mp_search_enqueue(void* search, const mp_range* range, void* stream) {
    Search* s = (Search*)search;
    if (!s) return fail(MP_E_ARG, "mp_search_enqueue: null search");
    if (s->pending) return fail(MP_E_STATE, "mp_search_enqueue: the previous run was not completed (mp_search_complete)");
    Table* t = s->table;
    Genome* g = s->genome;
    if (!g->sealed) return fail(MP_E_STATE, "mp_search_run: genome not sealed (call mp_genome_seal)");
    hipStream_t st = (hipStream_t)stream;
    MP_HIP_CHECK(hipSetDevice(g->device));
    if (s->put_wait) {  // a put of the last run's hits may still be reading them (any stream)
        MP_HIP_CHECK(hipStreamWaitEvent(st, s->put_done, 0));
        s->put_wait = false;
    }
    mp_range r{0, g->n_seq, 0, 0};
    if (range) r = *range;
    if (r.seq_begin > r.seq_end || r.seq_end > g->n_seq)
        return fail(MP_E_ARG, "mp_search_run: bad sequence range");
    const uint32_t W = (uint32_t)t->prm.wordsize;

    // owned (seq, k) range in global coordinates
    const uint64_t g_lo = (r.seq_begin < g->n_seq) ? g->base[r.seq_begin] + r.k_begin : g->total;
    const uint64_t g_hi = (r.seq_end < g->n_seq) ? g->base[r.seq_end] + r.k_end : g->total;

    // window positions to scan: k in the owned range, extended by max hash offset
    std::vector<SeqSpan> spans;
    uint64_t tiles = 0, windows = 0;
    const uint32_t last = std::min<uint32_t>(r.seq_end, g->n_seq ? g->n_seq - 1 : 0);
    for (uint32_t q = r.seq_begin; q <= last && q < g->n_seq; ++q) {
        const uint64_t n = g->len[q];
        if (n <= W) continue;  // engine.py:458: no window in a sequence of length <= W
        uint64_t klo = (q == r.seq_begin) ? r.k_begin : 0;
        uint64_t khi = (q == r.seq_end) ? r.k_end : n;
        if (q > r.seq_end || (q == r.seq_end && r.k_end == 0)) continue;
        khi = std::min<uint64_t>(khi, n);
        if (klo >= khi) continue;
        const uint64_t plo = klo;
        const uint64_t phi = std::min<uint64_t>(khi + t->max_hash_off, n - W + 1);
        if (plo >= phi) continue;
        SeqSpan sp;
        sp.super0 = tiles;
        sp.seq = q;
        sp.p_lo = (uint32_t)plo;
        sp.p_hi = (uint32_t)phi;
        sp.p_al = (uint32_t)(plo & ~(uint64_t)(kLanePos - 1));
        spans.push_back(sp);
        tiles += (phi - sp.p_al + kSuper - 1) / kSuper;
        windows += phi - plo;
    }
    // windows: counted here, on the host, from the spans the kernel walks
    s->n_windows = windows;
    s->n_candidates = 0;
    s->n_hits = 0;
    s->scan_ms = s->tail_ms = 0.f;
    s->pend_st = st;
    s->pend_tiles = tiles;
    s->pend_empty = tiles == 0;
    s->pending = true;
    ++g->n_pending;
    if (!tiles) return MP_OK;
    const uint32_t n_real_spans = (uint32_t)spans.size();
    {
        SeqSpan sentinel{};
        sentinel.super0 = tiles;
        spans.push_back(sentinel);
    }
    int rc = MP_OK;
    do {
        if (spans.size() > s->spans_cap) {
            hipFree(s->spans);
            s->spans = nullptr;
            s->spans_cap = 0;
            s->last_spans.clear();
            if (hipMalloc(&s->spans, spans.size() * sizeof(SeqSpan)) != hipSuccess) {
                rc = fail(MP_E_NOMEM, "mp_search_run: span allocation failed");
                break;
            }
            s->spans_cap = spans.size();
        }
        // the same range again (a repeated search, a benchmark step): the device copy is current
        if (spans.size() != s->last_spans.size() ||
            memcmp(spans.data(), s->last_spans.data(), spans.size() * sizeof(SeqSpan)) != 0) {
            s->last_spans.clear();
            if (hipMemcpyAsync(s->spans, spans.data(), spans.size() * sizeof(SeqSpan), hipMemcpyHostToDevice, st) !=
                    hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess) {  // the pageable source must outlive the copy
                rc = fail(MP_E_HIP, "mp_search_run: span upload failed");
                break;
            }
            s->last_spans = spans;
        }
        ScanArgs& a = *reinterpret_cast<ScanArgs*>(s->pend_args);
        a = ScanArgs{};
        a.g2 = g->g2; a.gexc = g->gexc; a.ginv = g->ginv; a.gwild = g->gwild; a.gpair = g->gpair;
        a.xr_start = g->xr_start; a.xr_char = g->xr_char; a.xr_dir = g->xr_dir; a.n_xr = g->n_xr;
        a.has_u = g->has_u ? 1 : 0;
        a.seq_base = g->d_base; a.seq_len = g->d_len;
        a.spans = s->spans; a.n_spans = n_real_spans;
        scan_fields(a, t, s);
        a.tail_ctr = 4;
        a.sched_base = kSchedBase;
        a.recs = t->recs; a.rank = t->rank;
        a.planes = t->planes; a.pchars = t->pchars; a.prec = t->prec;
        a.M = t->prm.margin; a.N = t->prm.mismatches;
        a.X = t->prm.three_prime_match; a.I = t->prm.iupac_mode;
        a.g_lo = g_lo; a.g_hi = g_hi;
        a.sched_short = s->opt.sched_short ? (uint32_t)s->opt.sched_short : (uint32_t)MP_SCHUNK_SHORT;
        // the scan grid's static bucket-tail slots (launch_scan's grid; a dense scan has none,
        // and its run launches no tail pass)
        a.tail_static = (uint64_t)scan_grid_of(s, tiles) * kWaves * kStaticRefs;
        // 16-B key references need the position in 40 bits and the sequence in 23 (ref16_make)
        a.ref16 = (g->total < (1ull << 40) && g->n_seq + 1u < (1u << 23) && !s->opt.ref32) ? 1u : 0u;
        // keys over 64 bits, or a forced rocPRIM sort: mode 2
        const int mode = run_order_mode(s);
        s->pend_mode = mode;
        rc = set_lists(s, a, mode);
        if (!rc) rc = enqueue_kernels(s, a, tiles, st, mode);
    } while (0);
    if (rc) {
        s->pending = false;
        --g->n_pending;
        s->dirty = true;
    }
    return rc;
}

MP_EXPORT int mp_search_complete(void* search, uint64_t* n_hits) {
    Search* s = (Search*)search;
    if (!s) return fail(MP_E_ARG, "mp_search_complete: null search");
    if (!s->pending) return fail(MP_E_STATE, "mp_search_complete: no run enqueued (mp_search_enqueue)");
    // the run is no longer pending whatever happens below (a failed call must not leave the
    // handle and its genome locked in MP_E_STATE); a failure marks the counters dirty
    if (n_hits) *n_hits = 0;
    s->pending = false;
    if (s->genome->n_pending) --s->genome->n_pending;
    if (s->pend_empty) return MP_OK;
    if (hipSetDevice(s->genome->device) != hipSuccess) {
        s->dirty = true;
        MP_HIP_CHECK(hipSetDevice(s->genome->device));
    }
    const int rc = search_complete(s, n_hits);
    if (rc) s->dirty = true;
    return rc;
}

MP_EXPORT int mp_search_run(void* search, const mp_range* range, void* stream, uint64_t* n_hits) {
    const int rc = mp_search_enqueue(search, range, stream);
    if (rc) return rc;
    return mp_search_complete(search, n_hits);
}

MP_EXPORT int mp_search_fetch(void* search, mp_hit* out, uint64_t cap, void* stream) {
    Search* s = (Search*)search;
    if (!s || (s->n_hits && !out)) return fail(MP_E_ARG, "mp_search_fetch: null pointer");
    if (s->pending) return fail(MP_E_STATE, "mp_search_fetch: a run is enqueued (mp_search_complete first)");
    if (cap < s->n_hits) return fail(MP_E_CAP, "mp_search_fetch: output buffer too small");
    if (!s->n_hits) return MP_OK;
    MP_HIP_CHECK(hipSetDevice(s->genome->device));
    MP_HIP_CHECK(hipMemcpyAsync(out, s->out, s->n_hits * sizeof(mp_hit), hipMemcpyDeviceToHost,
                                (hipStream_t)stream));
    MP_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
    return MP_OK;
}

MP_EXPORT int mp_search_fetch_device(void* search, mp_hit* dev_out, uint64_t cap, void* stream) {
    Search* s = (Search*)search;
    if (!s || (s->n_hits && !dev_out)) return fail(MP_E_ARG, "mp_search_fetch_device: null pointer");
    if (s->pending) return fail(MP_E_STATE, "mp_search_fetch_device: a run is enqueued (mp_search_complete first)");
    if (cap < s->n_hits) return fail(MP_E_CAP, "mp_search_fetch_device: output buffer too small");
    if (!s->n_hits) return MP_OK;
    MP_HIP_CHECK(hipSetDevice(s->genome->device));
    MP_HIP_CHECK(hipMemcpyAsync(dev_out, s->out, s->n_hits * sizeof(mp_hit), hipMemcpyDeviceToDevice,
                                (hipStream_t)stream));
    return MP_OK;
}

MP_EXPORT int mp_search_device_hits(void* search, const mp_hit** dev_hits) {
    Search* s = (Search*)search;
    if (!s || !dev_hits) return fail(MP_E_ARG, "mp_search_device_hits: null pointer");
    if (s->pending) return fail(MP_E_STATE, "mp_search_device_hits: a run is enqueued (mp_search_complete first)");
    *dev_hits = s->out;
    return MP_OK;
}

MP_EXPORT int mp_search_last_stats(void* search, float* scan_ms, uint64_t* n_windows, uint64_t* n_candidates) {
    Search* s = (Search*)search;
    if (!s) return fail(MP_E_ARG, "mp_search_last_stats: null search");
    if (s->pending) return fail(MP_E_STATE, "mp_search_last_stats: a run is enqueued (mp_search_complete first)");
    if (scan_ms) *scan_ms = s->scan_ms;
    if (n_windows) *n_windows = s->n_windows;
    if (n_candidates) *n_candidates = s->n_candidates;
    return MP_OK;
}

MP_EXPORT int mp_search_dev_bytes(void* search, uint64_t* dev_bytes) {
    Search* s = (Search*)search;
    if (!s || !dev_bytes) return fail(MP_E_ARG, "mp_search_dev_bytes: null pointer");
    *dev_bytes = s->cap * (16 + 8 + 8 + sizeof(mp_hit)) + s->surv_cap * sizeof(uint4) + s->tails_cap * 2 * sizeof(uint4) +
                 s->spans_cap * sizeof(SeqSpan) + s->slots_bytes + s->sort_tmp_bytes + kCounterBytes;
    return MP_OK;
}

MP_EXPORT int mp_search_regrowths(void* search, uint64_t* n_regrowths) {
    Search* s = (Search*)search;
    if (!s || !n_regrowths) return fail(MP_E_ARG, "mp_search_regrowths: null pointer");
    *n_regrowths = s->n_regrowths;
    return MP_OK;
}

MP_EXPORT int mp_search_survivors(void* search, uint64_t* n_survivors) {
    Search* s = (Search*)search;
    if (!s || !n_survivors) return fail(MP_E_ARG, "mp_search_survivors: null pointer");
    if (s->pending) return fail(MP_E_STATE, "mp_search_survivors: a run is enqueued (mp_search_complete first)");
    *n_survivors = s->n_survivors;
    return MP_OK;
}

MP_EXPORT int mp_search_timing(void* search, float* scan_ms, float* tail_ms, float* pair_ms, float* order_ms) {
    Search* s = (Search*)search;
    if (!s) return fail(MP_E_ARG, "mp_search_timing: null search");
    if (s->pending) return fail(MP_E_STATE, "mp_search_timing: a run is enqueued (mp_search_complete first)");
    if (scan_ms) *scan_ms = s->scan_ms;
    if (tail_ms) *tail_ms = s->tail_ms;
    if (pair_ms) *pair_ms = s->pair_ms;
    if (order_ms) *order_ms = s->order_ms;
    return MP_OK;
}

MP_EXPORT void mp_search_destroy(void* search) { free_search((Search*)search); }
