#!/bin/bash
# Round 6: post-scan kernels beside the next scan block.  coex = the key-group scans held to 96
# VGPRs with dynamic LDS (scan_kernel_lean), 2-wave pair blocks, 256-thread tail blocks with a
# 16 KiB buffer, 16 KiB bucket_offsets tiles; against the product with dynamic scan LDS (dyn)
# and the final build before it (r6f), same box.  First the coex library's GPU parity subset.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
L=merpcr_amd/_lib
MERPCR_LIB=$L/libmerpcr_hip_coex.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 \
    -k "full_table_prefix or sharded or regrowth or dense_repeat" > gpurun_out/r6x_coex_tests.log 2>&1 \
    || { echo "coex tests failed rc=$?"; tail -20 gpurun_out/r6x_coex_tests.log; exit 1; }
tail -1 gpurun_out/r6x_coex_tests.log
A="r6f|MERPCR_LIB=$L/libmerpcr_hip_r6f.so"
B="dyn|"
C="coex|MERPCR_LIB=$L/libmerpcr_hip_coex.so"
for cfg in "s8|--config c3 --shard-of 8 --steps 40 --warmup 5" "c3|--config c3 --steps 20 --warmup 5" "c4|--config c4 --steps 10 --warmup 3" "c5|--config c5 --steps 10 --warmup 3" "c2|--config c2 --steps 40 --warmup 5"; do
  IFS='|' read -r cn cargs <<< "$cfg"
  bash scripts/r05_ab.sh r6x_$cn "${A}|$cargs" "${B}|$cargs" "${C}|$cargs" || exit 1
done
