#!/bin/bash
# Round 6 final build, part A: the GPU suite, smoke, default bench line and two-rank rehearsal
# (scripts/gpu_check.sh), then the c3 rocprofv3 set (trace + PMC passes, scripts/profile.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash scripts/gpu_check.sh r6h3 || exit 1
KRE=scan_kernel bash scripts/profile.sh r06 --steps 20 --warmup 5 || exit 1
