#!/bin/bash
# PMC passes over pair_kernel (one counter set per pass), bench config given as args.
# usage: bash scripts/pmc_pair.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-c3}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_pair_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv --kernel-include-regex pair_kernel \
      -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 $BARGS > "$OUT/$name.log" 2>&1 \
      || { echo "pass $name failed rc=$?"; tail -5 "$OUT/$name.log"; exit 1; }
  echo "pass $name ok"
}
BARGS="$*"
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD
run sq2 SQ_WAIT_ANY SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH GRBM_GUI_ACTIVE
