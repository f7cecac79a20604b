#!/bin/bash
# Round 6: kernel durations at 1/8 and 1/64 of c3 with no pipelining (one handle, each run alone):
# the post-scan chain's own cost and the gaps between its launches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for k in 8 64; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r6s_sh$k -o run --output-format csv -- \
      python3 $R/bench.py --shard-of $k --no-pipeline --steps 30 --warmup 5 --no-cpu-baseline --no-e2e --no-pmc \
      > $R/gpurun_out/r6s_sh$k.log 2>&1 || { echo "trace sh$k failed rc=$?"; tail -5 $R/gpurun_out/r6s_sh$k.log; exit 1; }
  f=$(find $R/gpurun_out/r6s_sh$k -name '*kernel_trace.csv' | head -1)
  echo "== 1/$k"
  python3 $R/scripts/kernel_medians.py "$f"
done
