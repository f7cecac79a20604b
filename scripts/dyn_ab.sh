#!/bin/bash
# First-chunk claim A/B (MP_SCHED_DYNFIRST) on shard-of-8 and whole-genome steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for d in 0 1; do
  for args in "--shard-of 8 --steps 50 --warmup 5" "--shard-of 8 --steps 50 --warmup 5 --handles 3" "--steps 20 --warmup 3" "--steps 20 --warmup 3 --handles 3"; do
    MP_SCHED_DYNFIRST=$d timeout -k 10 300 python -u bench.py $args --no-e2e --no-cpu-baseline > gpurun_out/dyn.log 2>&1 || { echo "failed $d $args"; tail -5 gpurun_out/dyn.log; exit 1; }
    echo "dyn=$d $args: $(tail -n 1 gpurun_out/dyn.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['scan_kernel_ms'], (d.get('parity_distributed') or {}).get('ok'))")"
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "c5 or dense or W8 or synthetic or bundled" > gpurun_out/dense_test.log 2>&1 || { echo "dense tests failed"; tail -30 gpurun_out/dense_test.log; exit 1; }
tail -n 1 gpurun_out/dense_test.log
timeout -k 10 400 python -u bench.py --config c5 --no-e2e --cpu-budget 3 --no-ref-model > gpurun_out/c5.log 2>&1 || { echo c5 failed; tail -5 gpurun_out/c5.log; exit 1; }
tail -n 1 gpurun_out/c5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['ms_per_step'], d['scan_kernel_ms'], d['cpu_baseline']['parity_vs_gpu'])"
