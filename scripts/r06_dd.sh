#!/bin/bash
# Round 6: 16-B key references for the split seeds (the contiguous scan: launch_scan read the
# caller's cleared flag through an alias; then the gapped scan too): the GPU suite, then c5 / c3 A/B against the
# build with the contiguous fix only (libmerpcr_hip_base.so).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6dd_gputest.log 2>&1 \
    || { echo "gpu tests failed rc=$?"; tail -30 gpurun_out/r6dd_gputest.log; exit 1; }
tail -1 gpurun_out/r6dd_gputest.log
L=merpcr_amd/_lib
A="base|MERPCR_LIB=$L/libmerpcr_hip_base.so"
B="gap16|"
for cfg in "c5|--config c5 --steps 10 --warmup 3" "c3|--config c3 --steps 20 --warmup 5"; do
  IFS='|' read -r cn cargs <<< "$cfg"
  bash scripts/r05_ab.sh r6dd_$cn "${A}|$cargs" "${B}|$cargs" || exit 1
done
