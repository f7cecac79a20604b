#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_pair
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="--config c4 --no-e2e --no-cpu-baseline --no-ref-model --steps 3 --warmup 1 --one-stream"
run() { local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --kernel-include-regex pair_kernel -d "$OUT/$name" -o run --output-format csv -- python3 "$R/bench.py" $B > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  echo "pass $name ok"; }
run fetch --pmc FETCH_SIZE
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY
run tcc --pmc TCC_HIT_sum TCC_MISS_sum
