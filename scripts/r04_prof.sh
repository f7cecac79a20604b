#!/bin/bash
# The round's rocprofv3 evidence for one config (trace + PMC passes of the bench command,
# scripts/profile.sh), then its bench line with the full-genome CPU oracle check.
# usage: bash scripts/r04_prof.sh <tag> <config> [cpu-budget] [KRE]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; C=$2; B=${3:-15}
KRE=${4:-scan_kernel} bash scripts/profile.sh $T --config $C --no-ref-model --cpu-budget $B || exit 1
tail -c 600 gpurun_out/prof_$T/trace.log
