#!/bin/bash
# Round 6: key-reference reservations of 128 slots for the 8-B key groups (MP_REF_CHUNK1=128)
# against 64, with 16-B references; c3 and 1/8 c3, same box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=merpcr_amd/_lib
A="base|MERPCR_LIB=$L/libmerpcr_hip_base.so"
B="rc128|MERPCR_LIB=$L/libmerpcr_hip_rc128.so"
for cfg in "c3|--config c3 --steps 20 --warmup 5" "s8|--config c3 --shard-of 8 --steps 40 --warmup 5"; do
  IFS='|' read -r cn cargs <<< "$cfg"
  bash scripts/r05_ab.sh r6aa_$cn "${A}|$cargs" "${B}|$cargs" || exit 1
done
