#!/bin/bash
# Round 6: pair_kernel's batch claim issued one batch ahead (product) against the ABI-3 build,
# same box; then kernel timelines of pipelined 1/8 c3 and whole c3 steps (product build).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=merpcr_amd/_lib
A="abi3|MERPCR_LIB=$L/ab/libmerpcr_hip_abi3.so"
B="prod|"
for cfg in "c4|--config c4 --steps 10 --warmup 3" "c3|--config c3 --steps 20 --warmup 5" "s8|--config c3 --shard-of 8 --steps 30 --warmup 5"; do
  IFS='|' read -r cn cargs <<< "$cfg"
  bash scripts/r05_ab.sh r6d_$cn "${A}|$cargs" "${B}|$cargs" || exit 1
done
cd /tmp && export TMPDIR=/tmp
for cfg in "s8|--shard-of 8 --steps 30" "c3|--steps 10"; do
  IFS='|' read -r cn cargs <<< "$cfg"
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r6d_tl_$cn -o run --output-format csv -- \
      python3 $R/bench.py $cargs --no-cpu-baseline --no-e2e --no-pmc > $R/gpurun_out/r6d_tl_$cn.log 2>&1 \
      || { echo "timeline $cn failed rc=$?"; tail -5 $R/gpurun_out/r6d_tl_$cn.log; exit 1; }
  f=$(find $R/gpurun_out/r6d_tl_$cn -name '*kernel_trace.csv' | head -1)
  mkdir -p $R/gpurun_out/r6d_tl_${cn}_flat && cp "$f" $R/gpurun_out/r6d_tl_${cn}_flat/run_kernel_trace.csv
  python3 $R/scripts/timeline_streams.py $R/gpurun_out/r6d_tl_${cn}_flat 8 3 | tail -40
done
