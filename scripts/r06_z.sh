#!/bin/bash
# Round 6: 16-B key references for the I = 0 key-group scans too (c3, c2; not the gapped seed),
# only where the dispatch takes a key-group form (defer_full):
# the GPU suite once, then same-box A/B against the final build (libmerpcr_hip_r6f.so).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6z_ref16_gputest.log 2>&1 \
    || { echo "gpu tests failed rc=$?"; tail -30 gpurun_out/r6z_ref16_gputest.log; exit 1; }
tail -1 gpurun_out/r6z_ref16_gputest.log
L=merpcr_amd/_lib
A="r6f|MERPCR_LIB=$L/libmerpcr_hip_r6f.so"
B="ref16|"
for cfg in "c3|--config c3 --steps 20 --warmup 5" "s8|--config c3 --shard-of 8 --steps 40 --warmup 5" "c2|--config c2 --steps 40 --warmup 5"; do
  IFS='|' read -r cn cargs <<< "$cfg"
  bash scripts/r05_ab.sh r6z_$cn "${A}|$cargs" "${B}|$cargs" || exit 1
done
