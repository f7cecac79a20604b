#!/bin/bash
# Round 6: the deeper pipeline (4 handles, 2 streams, 2 steps ahead) against the default, with
# every handle primed before the warmup (a handle's first run uploads its spans and waits for its
# stream); product build with the block-claimed first chunks.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for cfg in "c3|--config c3 --steps 5 --warmup 2" "c4|--config c4 --steps 10 --warmup 3" "s8|--config c3 --shard-of 8 --steps 40 --warmup 5" "c2|--config c2 --steps 40 --warmup 5" "c5|--config c5 --steps 10 --warmup 3"; do
  IFS='|' read -r cn cargs <<< "$cfg"
  bash scripts/r05_ab.sh r6j_$cn "h2||$cargs" "d2||$cargs --handles 4 --streams 2 --depth 2" || exit 1
done
