#!/bin/bash
# Round 6: pipeline stream layouts, same box: the default (4 handles on 2 streams, 2 ahead)
# against one stream per handle (so a step's scan never queues behind an older step's chain).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for cfg in "s8|--config c3 --shard-of 8 --steps 40 --warmup 5" "c3|--config c3 --steps 10 --warmup 3" "c4|--config c4 --steps 10 --warmup 3"; do
  IFS='|' read -r cn cargs <<< "$cfg"
  bash scripts/r05_ab.sh r6n_$cn "d2||$cargs" "h4s4||$cargs --handles 4 --streams 4 --depth 2" \
      "h3s3||$cargs --handles 3 --streams 3 --depth 2" "h6s6d3||$cargs --handles 6 --streams 6 --depth 3" || exit 1
done
