#!/bin/bash
# Two-record key-group fields: the -m gpu suite, then c3, c2 and 1/8-shard bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pf_gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -40 gpurun_out/pf_gputest.log; exit 1; }
tail -1 gpurun_out/pf_gputest.log
for b in "c3:--no-e2e --no-ref-model --steps 20" "c2:--config c2 --no-e2e --no-ref-model --steps 20" "sh8:--shard-of 8 --no-e2e --no-ref-model --steps 50 --warmup 5"; do
  name=${b%%:*}; args=${b#*:}
  timeout -k 10 400 python -u bench.py $args > gpurun_out/pf_bench_$name.log 2>&1 || { echo "bench $name failed rc=$?"; tail -3 gpurun_out/pf_bench_$name.log | cut -c1-300; exit 1; }
  grep '^{' gpurun_out/pf_bench_$name.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', {k: d.get(k) for k in ('value','ms_per_step','scan_kernel_ms','tail_kernel_ms','pair_kernel_ms','order_ms','hits')}, d.get('cpu_baseline',{}).get('parity_vs_gpu'), (d.get('parity_distributed') or {}).get('ok'))"
done
