#!/bin/bash
# Instruction-mix counters (two PMC passes) for each ablation variant given.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_sq
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for V in "$@"; do
  T=$(echo "$V" | tr -c 'A-Za-z0-9\n' '_')
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH \
      -d "$OUT/${T}_a" -o run --output-format csv --kernel-include-regex scan_kernel \
      -- python3 "$R/scripts/ablate.py" --variants $V --steps 2 > "$OUT/${T}_a.log" 2>&1 \
      || { echo "pass $V a failed rc=$?"; tail -5 "$OUT/${T}_a.log"; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES \
      -d "$OUT/${T}_b" -o run --output-format csv --kernel-include-regex scan_kernel \
      -- python3 "$R/scripts/ablate.py" --variants $V --steps 2 > "$OUT/${T}_b.log" 2>&1 \
      || { echo "pass $V b failed rc=$?"; tail -5 "$OUT/${T}_b.log"; exit 1; }
  echo "pass $V ok"
done
