#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
T=${1:-r4b}
timeout -k 10 300 python -u scripts/diag_prefix.py c3 40000000 3 > gpurun_out/${T}_diag_prefix.log 2>&1 || { echo "diag rc=$?"; tail -20 gpurun_out/${T}_diag_prefix.log; exit 1; }
grep -v Warn gpurun_out/${T}_diag_prefix.log | cut -c1-300
bash scripts/r04_a.sh $T || exit 1
timeout -k 10 300 python -u scripts/multi_overhead.py 0.125 0,0 > gpurun_out/${T}_multi.log 2>&1 || { echo "multi rc=$?"; tail -20 gpurun_out/${T}_multi.log; exit 1; }
tail -1 gpurun_out/${T}_multi.log
