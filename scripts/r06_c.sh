#!/bin/bash
# Round 6: can a later step's tail kernel share the CUs with the running scan?  Same-box A/B of
# the ABI-3 build (scan lists 2,040 B/wave), the key-group scan lists cut to 680 B/wave (21 KB of
# LDS free per CU), and that with 512- / 256-thread tail blocks of a 16 KiB buffer.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=merpcr_amd/_lib
A="abi3|MERPCR_LIB=$L/ab/libmerpcr_hip_abi3.so"
B="lds|MERPCR_LIB=$L/libmerpcr_hip_ablateMP_TAIL_BLOCK_1024.so"
C="t512|MERPCR_LIB=$L/libmerpcr_hip_ablateMP_TAIL_BLOCK_512_MP_TAIL_BUF_1024_MP_TAIL_BPC_4.so"
D="t256|MERPCR_LIB=$L/libmerpcr_hip_ablateMP_TAIL_BLOCK_256_MP_TAIL_BUF_1024_MP_TAIL_BPC_8.so"
for cfg in "c3|--config c3 --steps 20 --warmup 5" "c4|--config c4 --steps 10 --warmup 3" "s8|--config c3 --shard-of 8 --steps 30 --warmup 5"; do
  IFS='|' read -r cn cargs <<< "$cfg"
  bash scripts/r05_ab.sh r6c_$cn "${A}|$cargs" "${B}|$cargs" "${C}|$cargs" "${D}|$cargs" || exit 1
done
