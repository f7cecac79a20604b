#!/bin/bash
# SQ issue / wait counters of one kernel (one rocprofv3 pass), beside scripts/pmc_ta.sh.
# usage: bash scripts/pmc_sq.sh <tag> <kernel-regex> [bench args...]
set -o pipefail
TAG=$1; KRE=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
Q="--no-cpu-baseline --no-e2e --no-pmc --no-ref-model --steps 2 --warmup 1 $*"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
    --kernel-include-regex "$KRE" -d "$OUT/sq" -o run --output-format csv \
    -- python3 "$R/bench.py" $Q > "$OUT/sq.log" 2>&1 || { echo "pass sq failed rc=$?"; tail -5 "$OUT/sq.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum \
    --kernel-include-regex "$KRE" -d "$OUT/tc" -o run --output-format csv \
    -- python3 "$R/bench.py" $Q > "$OUT/tc.log" 2>&1 || { echo "pass tc failed rc=$?"; tail -5 "$OUT/tc.log"; exit 1; }
python3 "$R/scripts/pmc_summary.py" "$OUT" "$KRE"
