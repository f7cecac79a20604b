#!/bin/bash
# Round 6: fewer scan workgroups than CUs (mp_search_options.scan_grid) so that the pipelined
# post-scan kernels of the step before find free CUs; 1/8 c3 and whole c3, same box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
S8="--config c3 --shard-of 8 --steps 40 --warmup 5"
bash scripts/r05_ab.sh r6p_s8 "g0||$S8" "g248||$S8 --opts scan_grid=248" "g240||$S8 --opts scan_grid=240" \
    "g224||$S8 --opts scan_grid=224" "g192||$S8 --opts scan_grid=192" || exit 1
C3="--config c3 --steps 10 --warmup 3"
bash scripts/r05_ab.sh r6p_c3 "g0||$C3" "g248||$C3 --opts scan_grid=248" "g240||$C3 --opts scan_grid=240" || exit 1
