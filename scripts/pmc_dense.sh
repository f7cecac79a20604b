#!/bin/bash
# PMC passes (one counter group per run) for one kernel of a bench config.
# usage: bash scripts/pmc_dense.sh <tag> <kernel-regex> [bench args...]
set -o pipefail
TAG=$1; KRE=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
Q="--no-cpu-baseline --no-e2e --steps 2 --warmup 1 $*"
run() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -d "$OUT/$name" -o run --output-format csv \
      -- python3 "$R/bench.py" $Q > "$OUT/$name.log" 2>&1 || { echo "pass $name failed rc=$?"; tail -5 "$OUT/$name.log"; exit 1; }
  echo "pass $name ok"
}

run req TCC_REQ_sum TCC_HIT_sum
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
run tcp TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
python3 "$R/scripts/pmc_summary.py" "$OUT" "$KRE"
