#!/bin/bash
# Round 6 final build, part D: shard lines + curve (part C), then the c2/c4/c5 profile sets.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash scripts/r06_final_c.sh || exit 1
for c in c2 c4 c5; do
  KRE=scan_kernel timeout -k 10 400 bash scripts/profile.sh r06_$c --config $c --no-ref-model --cpu-budget 8 || exit 1
done
