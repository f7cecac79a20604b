#!/bin/bash
# Round 6: the host gap between a stream's chain and its next scan.  Same-box A/B of the
# default pipeline (2 handles on 2 streams, step i+1 enqueued before the host waits for step i)
# against 4 handles dealt onto 2 streams with 2 or 3 steps enqueued ahead.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for cfg in "s8|--config c3 --shard-of 8 --steps 40 --warmup 5" "c2|--config c2 --steps 40 --warmup 5" "c3|--config c3 --steps 20 --warmup 5" "c4|--config c4 --steps 10 --warmup 3"; do
  IFS='|' read -r cn cargs <<< "$cfg"
  bash scripts/r05_ab.sh r6e_$cn "h2||$cargs" "h4d2||$cargs --handles 4 --streams 2 --depth 2" \
      "h4d3||$cargs --handles 4 --streams 2 --depth 3" || exit 1
done
