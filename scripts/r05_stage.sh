#!/bin/bash
# Per-stage budget of the scan forms of one config: timing-only variants of
# scripts/ablate_variants.py (built on the CPU side beforehand: scripts/ablate.py --build-only),
# each in its own process, under a kernel trace and then one PMC pass.
# usage: bash scripts/r05_stage.sh <tag> <config> <variants...>
set -o pipefail
TAG=$1; CFG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/stage_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/t$v" -o run --output-format csv -- \
      python3 "$R/scripts/ablate.py" --variants "$v" --config "$CFG" --steps 8 --no-build \
      > "$OUT/t$v.log" 2>&1 || { echo "trace $v failed rc=$?"; tail -5 "$OUT/t$v.log"; exit 1; }
  grep variant "$OUT/t$v.log" | tail -1
  timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES TCC_HIT_sum TCC_MISS_sum \
      --kernel-include-regex "scan_kernel|dense_kernel|tail_kernel" -d "$OUT/p$v" -o run --output-format csv -- \
      python3 "$R/scripts/ablate.py" --variants "$v" --config "$CFG" --steps 3 --no-build \
      > "$OUT/p$v.log" 2>&1 || { echo "pmc $v failed rc=$?"; tail -5 "$OUT/p$v.log"; exit 1; }
done
python3 "$R/scripts/pmc_forms.py" "$OUT"/t* "$OUT"/p* --match _kernel --json "$OUT/forms.json"
