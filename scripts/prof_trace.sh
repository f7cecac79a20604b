#!/bin/bash
# Trace-only refresh: the rocprofv3 --kernel-trace --stats pass of the bench command for every
# config (no PMC passes; use scripts/prof_all.sh when the scan kernels change).
# usage: bash scripts/prof_trace.sh <tag>   -> gpurun_out/prof_<tag>{,_c2,_c4,_c5}/trace
set -o pipefail
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
run() {  # name, bench-args
  local OUT=$R/gpurun_out/prof_$1; shift
  mkdir -p "$OUT"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
      -- python3 "$R/bench.py" "$@" > "$OUT/trace.log" 2>&1 \
      || { echo "trace $OUT failed rc=$?"; tail -5 "$OUT/trace.log"; exit 1; }
  echo "trace $OUT ok"; tail -1 "$OUT/trace.log"
}
run "$TAG" --e2e-file && \
run "${TAG}_c2" --config c2 --no-ref-model --cpu-budget 8 && \
run "${TAG}_c4" --config c4 --no-ref-model --cpu-budget 8 && \
run "${TAG}_c5" --config c5 --no-ref-model --cpu-budget 8
