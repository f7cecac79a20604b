#!/bin/bash
# Strong-scaling fixed cost of one rank's owned range: per-wave stamps of the scan
# (ablation 40, built on the CPU side beforehand), the shard curve, and the pipelined 1/8 step.
# usage: bash scripts/r05_shard.sh <tag> [extra bench args]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/wave_times.py --shard-of 8 --no-build > gpurun_out/${TAG}_waves8.log 2>&1 \
    || { echo "wave_times failed rc=$?"; tail -5 gpurun_out/${TAG}_waves8.log; exit 1; }
cat gpurun_out/${TAG}_waves8.log | grep -v amdgpu.ids
timeout -k 10 300 python3 -u scripts/shard_curve.py > gpurun_out/${TAG}_curve.log 2>&1 \
    || { echo "shard_curve failed rc=$?"; tail -5 gpurun_out/${TAG}_curve.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_curve.log
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --shard-of 8 --steps 30 --warmup 5 --no-cpu-baseline --no-e2e --no-pmc "$@" \
      > gpurun_out/${TAG}_sh8_$i.log 2>&1 || { echo "bench failed rc=$?"; tail -5 gpurun_out/${TAG}_sh8_$i.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_sh8_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('sh8 step', d['ms_per_step'], 'scan', d['scan_kernel_ms'], 'tail', d['tail_kernel_ms'], 'pair', d['pair_kernel_ms'], 'order', d['order_ms'], 'ok', d['parity_distributed']['ok'])"
done
