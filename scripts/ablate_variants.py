"""Timing-only variants of scan_kernel, kept out of the product source.

Each variant is a list of (anchor, insertion) edits applied to a temporary copy of
merpcr_amd/csrc/mp_search.hip: the insertion goes right before the anchor (which must
occur exactly once).  Hit counts of a variant are meaningless; only its scan time is.

  1   level 1 alone (genome stream, W-mers, validity smear, LDS prefilter)
  5   the genome stream, validity smear and scheduler alone (no LDS probe): the part of a
      scan pass two seed scans could share (the c5 single-pass question)
  2   level 1 and the positives' offset list
  3   level 1, the list and the level-2 loads (consumed, nothing more)
  6   the key-group scans without their key-reference writes (the field filter and compaction
      kept): what the references themselves cost in the scan
  30  no super-step loop (launch, LDS staging, statistics)
  31  no LDS staging and no loop
  40  per-wave wall-clock stamps (entry, LDS staged, loop end, exit) of scan_kernel, read back
      with mp_debug_wave_times (a function only this variant exports)
  42  variant 40 plus the end time of each of a wave's first 32 key-group super-steps
      (mp_debug_ss_times: 8192 waves x 32 stamps; 0 = not reached)
  50  pair_kernel without the lane-parallel try loop
  51  pair_kernel without any try (prologue, primer-1 compare and staging only)
  52  pair_kernel counting its per-survivor (non-lane-parallel) survivors by reason, read back
      with mp_debug_pair_counts (a function only this variant exports)
  54  pair_kernel without the primer-1 compare (every fingerprint survivor kept)
  55  pair_kernel's lane-parallel tries computed but never staged (no hits written)
  70  end-of-scan stealing across XCD groups (round 4, DESIGN 4.1: +20 us on 1/8 c3): a wave whose
      group is claimed out re-points its scheduler at the next group that still has more than
      one super-step per wave left and claims single super-steps there
  71  the key-group field filter of kgrp_pass in branch-free form (round 4, DESIGN 4.2: every
      form computed and selected; 1/8 c3 scan 0.342 -> 0.348 ms)
  90  64 v_nop per lane per super-step added to scan_kernel (~+8% of c3's VALU instructions):
      does issue bind the scan?  91: 128 (~+17%)
  80  tail_kernel reading its references (and the sequence tables / exception word they need)
      and nothing more
  81  tail_kernel up to the key's rank word and bucket head (no entries, no fingerprint test)
  82  tail_kernel with survivors counted, not stored: no LDS buffer, no barriers, no flushes
  7   level 2 without level 1's LDS reads: each window's level-1 bit is a hash of its W-mer
      (1/8 of windows pass, about the prefilter's 12% on c3), so the key-group probes, the field
      test and the references run as in the product on a like number of positives
  8   variant 5 with the static round-robin order (no claims): the genome stream alone
  9   variant 7 with 1/16 of windows passing level 1; 10: with 1/4 (the scan's sensitivity to
      the level-1 positive rate)
  57  pair_kernel with every survivor's record index folded into the first 1,024 records (their
      128-B record lines then stay in L2): the bound on what record-line locality could save
  58  pair_kernel's genome loads (the primer-2 stretch and the primer-1 window) non-temporal, so
      that they do not push the record lines out of L2
  11  a level 1.5 in the L1 for the I = 0 key groups, emulated: each level-1 positive first
      loads a word of a 32 KiB region (the first 32 KiB of the prefilter's global copy, which
      every CU reads, so it can stay in the CU's L1) by a hash of its key, then only 5/8 of the
      positives (by another hash) issue their key-group probe -- what a 32 KiB Bloom filter of
      the keys would pass; 12: the same loads, every positive probed (their cost alone)
  60  scan_kernel's genome-plane loads non-temporal (the stream kept out of L2's working set:
      the c4 level-2 tables, rank words + 16-B heads, are ~4.1 MB against a 4 MB L2)
"""
import os
import shutil

_L1 = "            const uint32_t c = (uint32_t)__popc(rem);\n"
_L2 = "                constexpr int kP = (kSeedQR + 63) / 64;\n"
_L3 = "                if constexpr (kRkf != 0) {\n                    // the few seeds that pass the key groups"
_LOOP = ("    while (ss < n_supers) {\n        const SeqSpan sp = pf;\n        const uint64_t sbase = pf_sbase;\n"
         "        const uint32_t n = pf_n;\n        SuperRegs R;")
_STAGE = "    {\n        constexpr int kStage = (int)(kLdsFilterWords / 4 / kBlock);  // eight uint4 per thread (128 KiB)\n"
_PROBE = "            const uint32_t rem = lds_probe32<kK, kGap>(s_lf, d0, d1, d2, shw, g_at, g_len) & okm;\n"

_LP = "    if (__any(lp)) {\n"
_TODO = "    uint64_t todo = __ballot(keep && !lp);\n"

_P1 = "    if (keep && !(v.z >> 31)) keep = primer_ok(a, gk, r.l1, r.p1_pl, r.p1_ch, true, pr->p1q);\n"
_LPHIT = "            stage_try_hit(a, S, lane, hit, sgk, srk, t - slo);\n"
_T_ENTRY = "    zero_sort_counts(a);\n    // stage the seed prefilter in LDS (once per persistent workgroup)"
_T_STAGED = "    const int lane = threadIdx.x & 63;\n    const int w = threadIdx.x >> 6;\n    const uint64_t stride = (uint64_t)gridDim.x * kWaves;"
_T_END = "    close_chunked(a.surv, a.surv_cap, lane, C);\n    if (a.ref16) close_chunked<1, kTC>"
_T_TAIL = "MP_EXPORT int mp_search_set_stage_timing(void* search, int32_t on) {"
_WORDS = ("        w0 = a.g2[j >> 5];\n        w1 = a.g2[(j >> 5) + 1];\n        v0 = a.ginv[j >> 6];  // branch-free: both loads always issue\n"
          "        v1 = a.ginv[(j >> 6) + 1];\n")
_WORDS_NT = ("        w0 = __builtin_nontemporal_load(&a.g2[j >> 5]);\n        w1 = __builtin_nontemporal_load(&a.g2[(j >> 5) + 1]);\n"
             "        v0 = __builtin_nontemporal_load(&a.ginv[j >> 6]);\n"
             "        v1 = __builtin_nontemporal_load(&a.ginv[(j >> 6) + 1]);\n")
_T_GLOBAL = ("}  // namespace mp\n\nusing namespace mp;\n\nMP_EXPORT int mp_search_set_stage_timing")

_STEAL = """    __device__ __forceinline__ bool steal(uint64_t n_supers) {  // ablation 70
        if (gridDim.x < 8u) return false;
        const uint32_t kW = blockDim.x >> 6;
        const uint32_t home = blockIdx.x & 7u;
        uint32_t x = lo;
        for (uint32_t t = 1; t < 8u; ++t) {
            const uint32_t nx = (x + 1u) & 7u;
            if (nx == home) return false;
            ctr += ((int)nx - (int)x) * (int)(2 * kStatStride);
            x = nx;
            const uint32_t h = (uint32_t)((n_supers * (x + 1)) >> 3);
            const uint32_t s0 = min((uint32_t)((n_supers * x) >> 3) + ((gridDim.x - x + 7u) >> 3) * kW * chunk, h);
            uint32_t cur = 0;
            if ((threadIdx.x & 63) == 0) cur = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            cur = (uint32_t)__builtin_amdgcn_readfirstlane((int)cur);
            const uint32_t own = ((gridDim.x - x + 7u) >> 3) * kW;
            if (s0 + cur + own < h) {
                lo = x;
                hi = h;
                S = s0;
                hint = h;
                young = 0;
                return true;
            }
        }
        return false;
    }
"""

_KGRP_BF = """    if (!kGap && !a.kgrp_wild) {  // ablation 71: every field form computed and selected
        const uint32_t present = (rw.x >> bit) & 1u;
        const uint32_t j = (uint32_t)__popc(__builtin_amdgcn_ubfe(rw.x, 0u, bit));
        const uint64_t w64 = ((uint64_t)rw.y << 32) | rw.x;
        const uint32_t field = (uint32_t)(w64 >> (16u + 16u * min(j, kKgrpFields - 1u))) & 0xFFFFu;
        const uint32_t x = ((pk >> 4) ^ field) & ((1u << (2u * a.kgrp_F)) - 1u);
        const uint32_t s_ok = (uint32_t)__popc((x | (x >> 1)) & 0x55555555u) <= (uint32_t)a.N;
        const uint32_t g3 = (pk >> (4u + 2u * (a.kgrp_F - 3u))) & 63u;
        const uint32_t x0 = g3 ^ ((field >> 6) & 63u), x1 = g3 ^ (field & 63u);
        const uint32_t p_ok = ((uint32_t)__popc((x0 | (x0 >> 1)) & 0x15u) <= (uint32_t)a.N) |
                              ((uint32_t)__popc((x1 | (x1 >> 1)) & 0x15u) <= (uint32_t)a.N);
        const uint32_t flag = (field >> 15) & 1u, pair = (field >> 14) & 1u;
        const uint32_t ok = (uint32_t)(j >= kKgrpFields) | (flag & s_ok) | ((flag ^ 1u) & ((pair ^ 1u) | p_ok));
        return (present & ok) != 0u;
    }
"""

VARIANTS = {
    1: [(_L1, "            if constexpr (kMode == 1) {  // ablation 1\n"
              "                ncand += (uint32_t)__popc(rem);\n"
              "                prefetch(nx, ss);\n"
              "                ss = nx;\n                continue;\n            }\n")],
    2: [(_L2, "                prefetch(nx, ss);\n"
              "                ncand += (uint32_t)L.rq.r[lane] & 1u;  // ablation 2\n"
              "                wave_sync();\n                r0 += kSeedQR;\n                continue;\n")],
    3: [(_L3, "                for (int q = 0; q < kP; ++q) ncand += rw[q].x & 1u;  // ablation 3\n"
              "                r0 += kSeedQR;\n                continue;\n")],
    5: [(_PROBE, "            if constexpr (kMode == 1) {  // ablation 5\n"
                 "                ncand += (uint32_t)__popc(okm ^ d0 ^ d1 ^ d2);\n"
                 "                prefetch(nx, ss);\n"
                 "                ss = nx;\n                continue;\n            }\n")],
    30: [(_LOOP, "    ss = n_supers;  // ablation 30\n")],
    31: [(_LOOP, "    ss = n_supers;  // ablation 31\n"), (_STAGE, "    if (false)  // ablation 31\n")],
    40: [(_T_ENTRY, "    const uint64_t wt0 = wall_clock64();  // ablation 40\n"),
         (_T_STAGED, "    const uint64_t wt1 = wall_clock64();  // ablation 40\n"),
         (_T_END, "    const uint64_t wt2 = wall_clock64();  // ablation 40\n"),
         ("        const uint64_t nx = sch.next(ss, n_supers, lane);\n        (void)stride;\n        if constexpr (kMode == 1) {",
          "        ++n_ss;  // ablation 40\n"),
         ("    SuperSched sch;\n    uint64_t ss = sch.first(a.counters, a.sched_base, n_supers, w, kWaves, lane, a.sched_short, s_first);",
          "    uint32_t n_ss = 0;  // ablation 40\n"),
         ("    // candidate statistics\n    add_stats(a, ncand, lane == 0 ? C.total : 0u, lane);\n}\n",
          "    if ((threadIdx.x & 63) == 0 && blockIdx.x * kWaves + (threadIdx.x >> 6) < 8192)  // ablation 40\n"
          "        g_wave_times[blockIdx.x * kWaves + (threadIdx.x >> 6)] = make_ulonglong4(wt0, wt1, wt2, n_ss);\n"),
         ("struct SuperSched {", "__device__ ulonglong4 g_wave_times[8192];  // ablation 40\n"),
         (_T_TAIL, "MP_EXPORT int mp_debug_wave_times(ulonglong4* out, uint32_t n) {  // ablation 40\n"
                   "    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_times), n * sizeof(ulonglong4)) == hipSuccess ? 0 : -1;\n}\n\n")],
    6: [("                        if (a.ref16)  // wave-uniform\n",
          "                        if (e < 0xFFFFFFFFu) continue;  // ablation 6\n")],
    80: [("        if (!(v.x == 0xFFFFFFFFu && v.y == 0xFFFFFFFFu)) {\n            const uint64_t gp = (uint64_t)v.x | ((uint64_t)v.y << 32);",
          "        ncand += (v.x != 0xFFFFFFFFu) ? ((w.w ^ w.z) & 1u) : 0u;  // ablation 80\n        v.x = v.y = 0xFFFFFFFFu;\n")],
    81: [("                if (c.y & kHead8Full) {\n                    first = c.x;  // the bucket's first entry",
          "                ncand += c.y & 1u;  // ablation 81\n                e.count = 0;\n                if (false)\n")],
    82: [("                const uint32_t at = atomicAdd(&s_n, 1u);\n", "                ncand += sv.x & 1u;  // ablation 82\n                continue;\n"),
         ("        if (it == next_check) {  // block-uniform\n", "        if (false)  // ablation 82\n")],
    90: [("        const uint32_t okm = (kGap ? window_ok_mask(R.iv, g_at) &",
          "        asm volatile(\".rept 64\\n v_nop\\n .endr\");  // ablation 90\n")],
    91: [("        const uint32_t okm = (kGap ? window_ok_mask(R.iv, g_at) &",
          "        asm volatile(\".rept 128\\n v_nop\\n .endr\");  // ablation 91\n")],
    42: None,  # variant 40 plus per-super-step stamps (below)
    70: [("        end = min(st + chunk, hi);\n        hint = st;\n        claim(lane);\n", "        lo = x;  // ablation 70\n"),
         ("        if (st >= hi) {\n            end = 0;\n            return n_supers;\n",
          "        while (st >= hi) {  // ablation 70\n            if (!steal(n_supers)) break;\n            claim(lane);\n"
          "            st = S + (uint32_t)__builtin_amdgcn_readfirstlane((int)pending);\n        }\n"),
         ("};\n\n// kRkf: 0 the rank queue", _STEAL)],
    71: [("    if (!((rw.x >> bit) & 1u)) return false;  // the key is absent\n    if constexpr (kGap != 0) {", _KGRP_BF)],
    7: [("                if constexpr (kGap != 0) x = gap_key(x, gap_at, gap_len);\n                const uint32_t wv = lds[x >> (37 - kLdsFilterLog2)];\n",
         "                if constexpr (kGap != 0) x = gap_key(x, gap_at, gap_len);\n"
         "                const uint32_t wv = ((x ^ (x >> 13)) & 7u) == 0u ? ~0u : 0u;  // ablation 7\n", "replace")],
    55: [(_LPHIT, "            if (hit && t < -1000000) // ablation 55\n")],
    54: [(_P1, "    if (false)  // ablation 54\n")],
    58: [("                    q0 = gq[2 * (e0 + t)];\n                    q1 = gq[2 * (e0 + t) + 1];\n",
          "                    {  // ablation 58\n"
          "                        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));\n"
          "                        const u64x2* gv = reinterpret_cast<const u64x2*>(a.gpair);\n"
          "                        const u64x2 t0 = __builtin_nontemporal_load(&gv[2 * (e0 + t)]);\n"
          "                        const u64x2 t1 = __builtin_nontemporal_load(&gv[2 * (e0 + t) + 1]);\n"
          "                        q0 = make_ulonglong2(t0.x, t0.y);\n"
          "                        q1 = make_ulonglong2(t1.x, t1.y);\n"
          "                    }\n", "replace"),
         ("        const uint64_t G = ext2p(a.gpair, gpos + c);  // the interleaved planes: one line, not three\n"
          "        const uint32_t ex = (uint32_t)(ext1p<2>(a.gpair, gpos + c) >> 32);\n",
          "        const uint64_t gj = gpos + c, w2 = gj >> 5, e2 = gj >> 6;  // ablation 58\n"
          "        const uint32_t s2 = (uint32_t)(gj & 31) * 2, s1 = (uint32_t)(gj & 63);\n"
          "        const uint64_t ga = __builtin_nontemporal_load(&a.gpair[((w2 >> 1) << 2) | (w2 & 1)]);\n"
          "        const uint64_t gb = __builtin_nontemporal_load(&a.gpair[(((w2 + 1) >> 1) << 2) | ((w2 + 1) & 1)]);\n"
          "        const uint64_t xa = __builtin_nontemporal_load(&a.gpair[(e2 << 2) | 2]);\n"
          "        const uint64_t xb = __builtin_nontemporal_load(&a.gpair[((e2 + 1) << 2) | 2]);\n"
          "        const uint64_t G = s2 ? (ga << s2) | (gb >> (64 - s2)) : ga;\n"
          "        const uint32_t ex = (uint32_t)((s1 ? (xa << s1) | (xb >> (64 - s1)) : xa) >> 32);\n", "replace")],
    57: [("    const uint32_t rec = v.z & 0x7FFFFFFFu;\n", "    const uint32_t rec = v.z & 0x3FFu;  // ablation 57\n", "replace")],
}


VARIANTS[9] = [(VARIANTS[7][0][0], VARIANTS[7][0][1].replace("& 7u", "& 15u").replace("ablation 7", "ablation 9"), "replace")]
VARIANTS[10] = [(VARIANTS[7][0][0], VARIANTS[7][0][1].replace("& 7u", "& 3u").replace("ablation 7", "ablation 10"), "replace")]

VARIANTS[8] = VARIANTS[5] + [
    ("        if (!sched_dynamic(n_supers, kW)) {\n            stride = waves;", "        if (true) {  // ablation 8\n            stride = waves;", "replace"),
]

def _l15(pass_rule):
    return [
        ("                uint32_t pk[kP], po[kP];\n",
         "                uint32_t pk[kP], po[kP];\n                uint32_t kq[kP], l1w[kP];  // ablation 11/12\n", "replace"),
        ("                                rw[q] = a.kgrp[v ? (key >> 4) : 0u];\n",
         "                                kq[q] = v ? key : 0xFFFFFFFFu;  // ablation 11/12\n"
         "                                l1w[q] = a.lfilt[v ? ((key * 0x9E3779B1u) >> 19) : 0u];\n", "replace"),
        ("                prefetch(nx, ss);  // after this round's probes (every round: see prefetch)\n",
         "                if constexpr (kRkf == 1) {  // ablation 11/12: the key-group probes after the L1 words\n"
         "#pragma unroll\n"
         "                    for (int q = 0; q < kP; ++q) {\n"
         "                        if ((uint32_t)q * 64u < nr) {\n"
         "                            const uint32_t key = kq[q];\n"
         "                            const bool v2 = key != 0xFFFFFFFFu && l1w[q] != 0xDEADBEEFu && " + pass_rule + ";\n"
         "                            rw[q] = a.kgrp[v2 ? (key >> 4) : 0u];\n"
         "                        }\n"
         "                    }\n"
         "                }\n"),
    ]


VARIANTS[11] = _l15("(((key * 0x85EBCA6Bu) >> 29) < 5u)")
VARIANTS[12] = _l15("true")

VARIANTS[42] = VARIANTS[40] + [
    ("            ss = nx;\n            continue;\n        }\n        uint32_t hits = probe32",
     "            if ((threadIdx.x & 63) == 0 && n_ss <= 32 && blockIdx.x * kWaves + (threadIdx.x >> 6) < 8192)  // ablation 42\n"
     "                g_ss_times[(blockIdx.x * kWaves + (threadIdx.x >> 6)) * 32 + n_ss - 1] = wall_clock64();\n"),
    ("struct SuperSched {", "__device__ unsigned long long g_ss_times[8192 * 32];  // ablation 42\n"),
    (_T_TAIL, "MP_EXPORT int mp_debug_ss_times(unsigned long long* out) {  // ablation 42\n"
              "    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ss_times), 8192 * 32 * 8) == hipSuccess ? 0 : -1;\n}\n\n"),
]


def make_source_dir(variant: int, csrc: str, root: str) -> str:
    """A copy of csrc at root/pkg/csrc (with the include directory at root/include, where
    the sources' relative includes expect it) with the variant's edits applied to
    mp_search.hip; returns the csrc copy."""
    if os.path.exists(root):
        shutil.rmtree(root)
    dst = os.path.join(root, "pkg", "csrc")
    shutil.copytree(csrc, dst)
    shutil.copytree(os.path.join(os.path.dirname(os.path.dirname(csrc)), "include"), os.path.join(root, "include"))
    p = os.path.join(dst, "mp_search.hip")
    s = open(p).read()
    for edit in VARIANTS[variant]:
        anchor, ins = edit[0], edit[1]
        if s.count(anchor) != 1:
            raise RuntimeError(f"ablation {variant}: anchor not unique in mp_search.hip: {anchor[:60]!r}")
        s = s.replace(anchor, ins if len(edit) > 2 and edit[2] == "replace" else ins + anchor)
    open(p, "w").write(s)
    return dst
