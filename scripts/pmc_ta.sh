#!/bin/bash
# TA / TCP stall counters of one kernel (one counter group per rocprofv3 run).
# usage: bash scripts/pmc_ta.sh <tag> <kernel-regex> [bench args...]
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
run ta1 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
run ta2 TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum
run tcp TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum
python3 "$R/scripts/pmc_summary.py" "$OUT" "$KRE"
