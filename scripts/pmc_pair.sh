#!/bin/bash
# PMC passes of pair_kernel on a config (default c4), one counter set per pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=${1:-c4}
OUT=$R/gpurun_out/pmc_pair_$CFG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="--config $CFG --no-e2e --no-cpu-baseline --no-ref-model --steps 3 --warmup 1 --one-stream"
run() { local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --kernel-include-regex pair_kernel -d "$OUT/$name" -o run --output-format csv -- python3 "$R/bench.py" $B > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  echo "pass $name ok"; }
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY
run tcc --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
run ta --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
python3 "$R/scripts/pmc_table.py" "$OUT"
