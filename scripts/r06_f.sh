#!/bin/bash
# Round 6: tail_kernel's 16-B references pipelined two deep (one round trip per pass), against
# the same build without it, and with 16-B key references for c3's and c5's scans too; then the
# whole GPU suite on the 16-B-everywhere library (which also has the two-deep tail).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=merpcr_amd/_lib
A="base|MERPCR_LIB=$L/libmerpcr_hip_ablateMP_TAIL_BLOCK_1024.so"
B="tail2|MERPCR_LIB=$L/libmerpcr_hip_ablateMP_R6TAIL_1.so"
C="ref16|MERPCR_LIB=$L/libmerpcr_hip_ablateMP_REF16_ALL_1.so"
for cfg in "c4|--config c4 --steps 10 --warmup 3" "c3|--config c3 --steps 20 --warmup 5" "s8|--config c3 --shard-of 8 --steps 40 --warmup 5" "c5|--config c5 --steps 10 --warmup 3"; do
  IFS='|' read -r cn cargs <<< "$cfg"
  bash scripts/r05_ab.sh r6f_$cn "${A}|$cargs" "${B}|$cargs" "${C}|$cargs" || exit 1
done
MERPCR_LIB=$L/libmerpcr_hip_ablateMP_REF16_ALL_1.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r6f_gputest.log 2>&1 \
    || { echo "gpu tests failed rc=$?"; tail -30 gpurun_out/r6f_gputest.log; exit 1; }
tail -3 gpurun_out/r6f_gputest.log
