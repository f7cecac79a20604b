#!/bin/bash
# Round-4 final code: c3 / c2 / c5 profiles and bench lines (CPU oracle over the whole genome).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash scripts/r04_prof.sh r04b c3 600 || exit 1
bash scripts/r04_prof.sh r04b_c2 c2 600 || exit 1
bash scripts/r04_prof.sh r04b_c5 c5 600 || exit 1
