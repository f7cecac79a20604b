"""Register / spill / scratch table of the device kernels of one source (hipcc
-Rpass-analysis=kernel-resource-usage, device-only compile; no GPU needed).
usage: python scripts/kernel_regs.py [source.hip] [-D...] [--filter substr] [--save base.json] [--diff base.json]"""
import json
import re
import subprocess
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]
args = sys.argv[1:]
src = next((a for a in args if a.endswith(".hip")), ROOT + "/merpcr_amd/csrc/mp_search.hip")
defs = [a for a in args if a.startswith("-D")]
flt = args[args.index("--filter") + 1] if "--filter" in args else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC", "-I", ROOT + "/include",
       "-mllvm", "-amdgpu-atomic-optimizer-strategy=None", "--cuda-device-only", "-c", src, "-o", "/tmp/_kr.o",
       "-Rpass-analysis=kernel-resource-usage"] + defs
res = subprocess.run(cmd, capture_output=True, text=True)
out, cur = {}, None
for l in res.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", l)
    if m:
        cur = m.group(1)
        out[cur] = {}
        continue
    m = re.search(r"remark:\s+(TotalSGPRs|VGPRs|ScratchSize \[bytes/lane\]|SGPRs Spill|VGPRs Spill|Occupancy \[waves/SIMD\]): (\d+)", l)
    if m and cur:
        out[cur][m.group(1).split()[0] + ("_spill" if "Spill" in m.group(1) else "")] = int(m.group(2))
if res.returncode:
    print(res.stderr[-3000:])
    sys.exit(1)
base = json.load(open(args[args.index("--diff") + 1])) if "--diff" in args else {}
for k, v in sorted(out.items()):
    if flt and flt not in k:
        continue
    d = "" if not base or base.get(k) == v else f"   (was {base.get(k)})"
    print(f"{k[:70]:70s} {v}{d}")
if "--save" in args:
    json.dump(out, open(args[args.index("--save") + 1], "w"))
