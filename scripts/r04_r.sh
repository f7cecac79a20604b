#!/bin/bash
# The final build's c3 profile and bench line (CPU oracle over the whole genome).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash scripts/r04_prof.sh r04c c3 600 || exit 1
