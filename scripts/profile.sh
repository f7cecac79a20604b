#!/bin/bash
# Kernel trace + PMC passes of bench.py on the GPU box (each counter set in its own run).
# usage: bash scripts/profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --steps 5 --warmup 1 $*"
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python3 "$R/bench.py" $ARGS \
      > "$OUT/$name.log" 2>&1 || { echo "pass $name failed rc=$?"; tail -5 "$OUT/$name.log"; exit 1; }
  echo "pass $name ok"
}
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE --kernel-include-regex scan_kernel
run write --pmc WRITE_SIZE --kernel-include-regex scan_kernel
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-include-regex scan_kernel
run tcc --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex scan_kernel
