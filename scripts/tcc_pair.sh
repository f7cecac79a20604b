#!/bin/bash
# L2 hit/miss and request counters for two ablation variants (one PMC pass each).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_tcc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for V in "$@"; do
  timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum -d "$OUT/$V" -o run --output-format csv \
      --kernel-include-regex scan_kernel -- python3 "$R/scripts/ablate.py" --variants $V --steps 2 > "$OUT/$V.log" 2>&1 \
      || { echo "pass $V failed rc=$?"; tail -5 "$OUT/$V.log"; exit 1; }
  echo "pass $V ok"
done
