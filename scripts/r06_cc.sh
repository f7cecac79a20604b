#!/bin/bash
# Round 6: the split seeds' contiguous scan with 16-B key references (launch_scan read the
# caller's cleared flag through an alias): the GPU suite, then c5 / c3 same-box A/B against the
# build before (libmerpcr_hip_base.so).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6cc_gputest.log 2>&1 \
    || { echo "gpu tests failed rc=$?"; tail -30 gpurun_out/r6cc_gputest.log; exit 1; }
tail -1 gpurun_out/r6cc_gputest.log
L=merpcr_amd/_lib
A="base|MERPCR_LIB=$L/libmerpcr_hip_base.so"
B="split16|"
for cfg in "c5|--config c5 --steps 10 --warmup 3" "c3|--config c3 --steps 20 --warmup 5"; do
  IFS='|' read -r cn cargs <<< "$cfg"
  bash scripts/r05_ab.sh r6cc_$cn "${A}|$cargs" "${B}|$cargs" || exit 1
done
