"""Timing-only variants of scan_kernel, kept out of the product source.

Each variant is a list of (anchor, insertion) edits applied to a temporary copy of
merpcr_amd/csrc/mp_search.hip: the insertion goes right before the anchor (which must
occur exactly once).  Hit counts of a variant are meaningless; only its scan time is.

  1   level 1 alone (genome stream, W-mers, validity smear, LDS prefilter)
  2   level 1 and the positives' offset list
  3   level 1, the list and the level-2 loads (consumed, nothing more)
  30  no super-step loop (launch, LDS staging, statistics)
  31  no LDS staging and no loop
  50  pair_kernel without the lane-parallel try loop
  51  pair_kernel without any try (prologue, primer-1 compare and staging only)
"""
import os
import shutil

_L1 = "            const uint32_t c = (uint32_t)__popc(rem);\n"
_L2 = "                constexpr int kP = (kSeedQR + 63) / 64;\n"
_L3 = "                if constexpr (kRkf) {\n                    // the few seeds that pass the key groups"
_LOOP = ("    while (ss < n_supers) {\n        const SeqSpan sp = pf;\n        const uint64_t sbase = pf_sbase;\n"
         "        const uint32_t n = pf_n;\n        SuperRegs R;")
_STAGE = ("    for (uint32_t i = threadIdx.x; i < kLdsFilterWords / 4; i += kBlock)\n"
          "        reinterpret_cast<uint4*>(s_lf)[i] = reinterpret_cast<const uint4*>(a.lfilt)[i];\n")

_LP = "    if (__any(lp)) {\n"
_TODO = "    uint64_t todo = __ballot(keep && !lp);\n"

VARIANTS = {
    1: [(_L1, "            if constexpr (kMode == 1) {  // ablation 1\n"
              "                ncand += (uint32_t)__popc(rem);\n"
              "                if (nx < n_supers) { locate(nx); words(nx, nw0, nw1, niv); }\n"
              "                ss = nx;\n                continue;\n            }\n")],
    2: [(_L2, "                if (first) { first = false; if (nx < n_supers) { locate(nx); words(nx, nw0, nw1, niv); } }\n"
              "                ncand += (uint32_t)L.rq.r[lane] & 1u;  // ablation 2\n"
              "                wave_sync();\n                r0 += kSeedQR;\n                continue;\n")],
    3: [(_L3, "                for (int q = 0; q < kP; ++q) ncand += rw[q].x & 1u;  // ablation 3\n"
              "                r0 += kSeedQR;\n                continue;\n")],
    30: [(_LOOP, "    ss = n_supers;  // ablation 30\n")],
    31: [(_LOOP, "    ss = n_supers;  // ablation 31\n"), (_STAGE, "    if (false)  // ablation 31\n")],
    50: [(_LP, "    if (false)  // ablation 50\n")],
    51: [(_LP, "    if (false)  // ablation 51\n"), (_TODO, "    keep = false;  // ablation 51\n")],
}


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
    for anchor, ins in VARIANTS[variant]:
        if s.count(anchor) != 1:
            raise RuntimeError(f"ablation {variant}: anchor not unique in mp_search.hip: {anchor[:60]!r}")
        s = s.replace(anchor, ins + anchor)
    open(p, "w").write(s)
    return dst
