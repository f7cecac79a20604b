"""Rebuild the A/B variant libraries from the current sources (run after every product
change, before a GPU call that loads them through MERPCR_LIB):
  libmerpcr_hip_ablate<DEFINES>.so for each NAME=VAL[+NAME=VAL] argument."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from merpcr_amd import _build  # noqa: E402

for v in sys.argv[1:]:
    defs = tuple(v.split("+"))
    tag = "".join(ch if ch.isalnum() else "_" for ch in v)
    print(_build.build_native(defines=defs, lib=os.path.join(_build.LIBDIR, f"libmerpcr_hip_ablate{tag}.so")))
