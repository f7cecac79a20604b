#!/bin/bash
# Round 6: the post-scan chain's shape at 1/8 of c3 -- bucket tails inline in the scan (no
# tail_kernel) and no full-head deferral -- against the default, same box; whole c3 beside.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
S8="--config c3 --shard-of 8 --steps 40 --warmup 5"
bash scripts/r05_ab.sh r6r_s8 "def||$S8" "inl||$S8 --opts tails=inline" "nodef||$S8 --opts defer=0" || exit 1
C3="--config c3 --steps 10 --warmup 3"
bash scripts/r05_ab.sh r6r_c3 "def||$C3" "inl||$C3 --opts tails=inline" "nodef||$C3 --opts defer=0" || exit 1
