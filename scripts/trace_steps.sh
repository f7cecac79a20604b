#!/bin/bash
# Kernel + copy timeline of a few bench steps (no counters): where a step's wall time goes
# between kernels.  usage: bash scripts/trace_steps.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-tl}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/trace_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT" -o run --output-format csv -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-ref-model --no-e2e --steps 5 --warmup 1 "$@" > "$OUT/bench.log" 2>&1 \
    || { echo "trace failed rc=$?"; tail -5 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-300
