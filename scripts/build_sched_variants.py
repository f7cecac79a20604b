"""Build libmerpcr_hip_sched<X>.so: the product sources with mp_search.hip compiled under an
alternative AMDGPU machine-scheduler setting (a timing A/B; the kernels' semantics are the
product's).  usage: python scripts/build_sched_variants.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from merpcr_amd import _build  # noqa: E402

VARIANTS = {
    "ilp": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
    "memclause": ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"],
    "bias0": ["-mllvm", "-amdgpu-schedule-metric-bias=0"],
}
base = list(_build.SOURCE_FLAGS.get("mp_search.hip", []))
for name, extra in VARIANTS.items():
    _build.SOURCE_FLAGS = {"mp_search.hip": base + extra}
    out = _build.build_native(lib=os.path.join(_build.LIBDIR, f"libmerpcr_hip_sched{name}.so"), tag=f"_sched{name}",
                              force=True)
    print(out)
