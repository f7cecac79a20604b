#!/bin/bash
# 8-B IUPAC heads round trip: the -m gpu suite, then c4 bench lines with and without them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/h12_gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -40 gpurun_out/h12_gputest.log; exit 1; }
tail -2 gpurun_out/h12_gputest.log
for v in 0 1; do
MP_NO_H12=$v timeout -k 10 400 python -u bench.py --config c4 --no-e2e --no-ref-model --steps 10 --warmup 3 > gpurun_out/h12_c4_$v.log 2>&1 || { echo "bench failed rc=$?"; tail -3 gpurun_out/h12_c4_$v.log | cut -c1-300; exit 1; }
grep '^{' gpurun_out/h12_c4_$v.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('no_h12=$v', {k: d.get(k) for k in ('value','ms_per_step','scan_kernel_ms','tail_kernel_ms','pair_kernel_ms','order_ms','hits','survivors')}, d.get('cpu_baseline',{}).get('parity_vs_gpu'))"
done
