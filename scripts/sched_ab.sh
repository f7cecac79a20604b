#!/bin/bash
# Short-scan claim size A/B (MP_SCHUNK_SHORT) on shard-of-8/4 steps, plus one e2e line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for c in 1 2 4; do
  for sh in 8 4; do
    MP_SCHUNK_SHORT=$c timeout -k 10 300 python -u bench.py --shard-of $sh --no-e2e --steps 50 --warmup 5 > gpurun_out/sab_${c}_${sh}.log 2>&1 || { echo "failed $c $sh"; tail -5 gpurun_out/sab_${c}_${sh}.log; exit 1; }
    echo "chunk=$c shard=$sh $(tail -n 1 gpurun_out/sab_${c}_${sh}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['scan_kernel_ms'], (d.get('parity_distributed') or {}).get('ok'))")"
  done
done
timeout -k 10 400 python -u bench.py --steps 10 --cpu-budget 3 --no-ref-model > gpurun_out/sab_e2e.log 2>&1 || { echo e2e failed; tail -5 gpurun_out/sab_e2e.log; exit 1; }
tail -n 1 gpurun_out/sab_e2e.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['scan_kernel_ms'], d['e2e'], d['cpu_baseline']['parity_vs_gpu'])"
