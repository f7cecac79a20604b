"""Build libmerpcr_hip.so in-tree with hipcc for gfx950 (no JIT cache, no torch)."""

from __future__ import annotations

import concurrent.futures
import os
import shutil
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "_lib")
LIB = os.path.join(LIBDIR, "libmerpcr_hip.so")
SOURCES = ["mp_table.hip", "mp_genome.hip", "mp_search.hip", "mp_sort.hip", "mp_order.hip", "mp_multi.hip", "mp_fasta.hip",
           "mp_fasta_dev.hip", "mp_format.hip", "mp_sts.hip"]
HEADERS = ["mp_internal.h", "mp_text.h", os.path.join("..", "..", "include", "merpcr_hip.h")]
ARCH = os.environ.get("MERPCR_OFFLOAD_ARCH", "gfx950")
# Per-source flags.  mp_search.hip aggregates its atomics by hand (lane 0 of a wave); the
# compiler's atomic optimizer would add a readfirstlane of the returned value, i.e. a wait
# for every older load right at the atomic -- in the pipelined scan that is the super-step
# claim, which must not wait for the level-2 probes in flight.
SOURCE_FLAGS = {"mp_search.hip": ["-mllvm", "-amdgpu-atomic-optimizer-strategy=None"]}


def source_digest(src_dir: str = CSRC) -> str:
    """16 hex digits of sha256 over the library's sources and headers: the build a bench line
    or a profile was taken with (profiles/*_pmc.json record it; bench.py matches on it)."""
    import hashlib
    h = hashlib.sha256()
    for f in SOURCES + HEADERS:
        with open(os.path.normpath(os.path.join(src_dir, f)), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the MI355X engine needs ROCm's hipcc to build")


def _flags():
    return ["--offload-arch=" + ARCH, "-O3", "-std=c++20", "-fPIC", "-fvisibility=hidden",
            "-Wall", "-Wno-unused-result", "-I", os.path.join(ROOT, "include")]


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_native(force: bool = False, verbose: bool = False, defines=(), lib: str = LIB, src_dir: str = CSRC,
                 tag: str = "") -> str:
    """Compile the sources and link `lib`; `defines` and a `src_dir` copy (timing-only
    variants, scripts/ablate.py) get their own objects, named by `tag`."""
    os.makedirs(LIBDIR, exist_ok=True)
    cc = hipcc()
    tag = tag + "".join("_" + d.replace("=", "") for d in defines)
    hdrs = [os.path.normpath(os.path.join(src_dir, h)) for h in HEADERS]
    objs = []
    jobs = []
    for src in SOURCES:
        sp = os.path.join(src_dir, src)
        op = os.path.join(LIBDIR, src.replace(".hip", tag + ".o"))
        objs.append(op)
        if force or _stale(op, [sp] + hdrs):
            jobs.append([cc] + _flags() + SOURCE_FLAGS.get(src, []) + ["-D" + d for d in defines] + ["-c", sp, "-o", op])
    if jobs:
        with concurrent.futures.ThreadPoolExecutor(max_workers=min(4, len(jobs))) as ex:
            for cmd, res in zip(jobs, ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), jobs)):
                if verbose or res.returncode:
                    print(" ".join(cmd))
                    print(res.stdout + res.stderr)
                if res.returncode:
                    raise RuntimeError(f"hipcc failed for {cmd[-3]}")
    if force or jobs or _stale(lib, objs):
        cmd = [cc, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib] + objs + [
            "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode:
            print(" ".join(cmd))
            print(res.stdout + res.stderr)
            raise RuntimeError("hipcc link failed")
    return lib


if __name__ == "__main__":
    import sys
    print(build_native(force="--force" in sys.argv, verbose="-v" in sys.argv))
