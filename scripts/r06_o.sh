#!/bin/bash
# Round 6: kernel timeline of the default pipeline pipelined 1/8 c3 step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r6o_tl -o run --output-format csv -- \
    python3 $R/bench.py --shard-of 8 --steps 40 --warmup 5 --no-cpu-baseline --no-e2e --no-pmc > $R/gpurun_out/r6o_tl.log 2>&1 \
    || { echo "timeline failed rc=$?"; tail -5 $R/gpurun_out/r6o_tl.log; exit 1; }
f=$(find $R/gpurun_out/r6o_tl -name '*kernel_trace.csv' | head -1)
mkdir -p $R/gpurun_out/r6o_tl_flat && cp "$f" $R/gpurun_out/r6o_tl_flat/run_kernel_trace.csv
python3 $R/scripts/timeline_streams.py $R/gpurun_out/r6o_tl_flat 20 4
grep '^{' $R/gpurun_out/r6o_tl.log | cut -c1-300
