"""Basic-block instruction counts of one kernel in the gfx950 assembly of mp_search.hip
(hipcc -S, device only; no GPU needed): per block the instruction mix (VALU / SALU / LDS /
VMEM / SMEM / waitcnt / branch) and the loop it sits in.  usage:
  python scripts/isa_blocks.py [kernel-symbol-substring] [--asm file.s] [--show .LBBx_y]"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]
args = sys.argv[1:]
_vals = {args[i + 1] for i, a in enumerate(args[:-1]) if a in ("--asm", "--show")}
sym = next((a for a in args if not a.startswith("-") and a not in _vals), "scan_kernelILi1ELb0ELi2ELb1ELi0ELb1ELb0E")
asm = args[args.index("--asm") + 1] if "--asm" in args else "/tmp/_isa.s"
defs = [a for a in args if a.startswith("-D")]
if "--asm" not in args:
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC", "-I", ROOT + "/include",
                    "-mllvm", "-amdgpu-atomic-optimizer-strategy=None", "--cuda-device-only", "-S",
                    ROOT + "/merpcr_amd/csrc/mp_search.hip", "-o", asm] + defs, check=True, capture_output=True)
lines = open(asm).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(sym) + r"\S*:", l))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))


def kind(op):
    if op.startswith("s_waitcnt"):
        return "wait"
    if "branch" in op or op.startswith("s_cbranch"):
        return "br"
    if op.startswith(("s_load", "s_buffer")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    return "other"


show = args[args.index("--show") + 1] if "--show" in args else None
cur, loop, blocks = "entry", "", []
body = []
for l in lines[start:end]:
    m = re.match(r"^(\.LBB\S+):\s*(;.*)?$", l)
    if m:
        if body or cur == "entry":
            blocks.append((cur, loop, body))
        cur, body = m.group(1), []
        loop = (m.group(2) or "").replace(";", "").strip()
        continue
    t = l.strip()
    if t and not t.startswith((";", ".")):
        body.append(t)
blocks.append((cur, loop, body))
tot = 0
for name, lp, ins in blocks:
    k = {}
    for t in ins:
        kk = kind(t.split()[0])
        k[kk] = k.get(kk, 0) + 1
    tot += len(ins)
    if show is None:
        print(f"{name:14s} {len(ins):4d} {k}  [{lp[:40]}]")
    elif name == show:
        print("\n".join(ins))
print("total", tot)
