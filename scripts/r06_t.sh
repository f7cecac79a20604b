#!/bin/bash
# Round 6: pair_kernel without batch claims when a group's waves outnumber its batches, against
# the final build before it (merpcr_amd/_lib/ab/libmerpcr_hip_r6f.so), same box; then the
# unpipelined kernel durations of the new build at 1/8 and 1/64.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=merpcr_amd/_lib
A="base|MERPCR_LIB=$L/ab/libmerpcr_hip_r6f.so"
B="new|"
for cfg in "s8|--config c3 --shard-of 8 --steps 40 --warmup 5" "c3|--config c3 --steps 10 --warmup 3" "c4|--config c4 --steps 10 --warmup 3" "c2|--config c2 --steps 40 --warmup 5"; do
  IFS='|' read -r cn cargs <<< "$cfg"
  bash scripts/r05_ab.sh r6t_$cn "${A}|$cargs" "${B}|$cargs" || exit 1
done
bash scripts/r06_s.sh
