#!/bin/bash
# Split-seed round trip: parity tests (both LDS filter forms), then c5 bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py "tests/test_gpu_fullscale.py::test_full_table_prefix_vs_c_oracle[c5-48000000-2]" -x -v --timeout 120 --timeout-method thread > gpurun_out/split_test.log 2>&1 || { echo "split tests failed rc=$?"; tail -40 gpurun_out/split_test.log; }
tail -3 gpurun_out/split_test.log
MP_LDS_K=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 120 --timeout-method thread > gpurun_out/split_test_k2.log 2>&1 || { echo "split tests (k=2) failed rc=$?"; tail -40 gpurun_out/split_test_k2.log; }
tail -3 gpurun_out/split_test_k2.log
for b in "--scale 0.05" "--scale 0.3"; do
timeout -k 10 400 python -u bench.py --config c5 --no-e2e --no-ref-model --steps 5 --warmup 2 $b > gpurun_out/split_c5.log 2>&1 || { echo "bench failed rc=$?"; tail -3 gpurun_out/split_c5.log | cut -c1-300; }
grep '^{' gpurun_out/split_c5.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','ms_per_step','scan_kernel_ms','tail_kernel_ms','pair_kernel_ms','order_ms','hits')}, d.get('cpu_baseline',{}).get('parity_vs_gpu'), d.get('cpu_baseline',{}).get('hits'))" || true
done
