#!/bin/bash
# Round 6: rocprofv3 --kernel-trace --stats of the bench with one handle (no pipelining), so that
# every scan dispatch runs alone and the summary's average is the isolated duration the bench
# line's roofline uses (its own trace pass is the same shape: --no-pipeline, one handle).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6hh -o run --output-format csv -- \
    python3 $R/bench.py --no-pipeline --no-pmc --no-cpu-baseline --no-e2e --steps 20 --warmup 5 > $R/gpurun_out/r6hh.log 2>&1 \
    || { echo "trace failed rc=$?"; tail -5 $R/gpurun_out/r6hh.log; exit 1; }
f=$(find $R/gpurun_out/r6hh -name '*kernel_stats.csv' | head -1)
cp "$f" $R/gpurun_out/r6hh_kernel_stats.csv
grep '^{' $R/gpurun_out/r6hh.log | cut -c1-200
