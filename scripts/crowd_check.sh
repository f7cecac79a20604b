#!/bin/bash
# Hit-order round trip: the order-path GPU tests, then a c4 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py -k "crowded or repeat_order or golden or c4 or dense_tables or order" -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/crowd_test.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/crowd_test.log; exit 1; }
tail -2 gpurun_out/crowd_test.log
timeout -k 10 400 python -u bench.py --config c4 --no-e2e --no-ref-model --steps 10 --warmup 3 > gpurun_out/crowd_c4.log 2>&1 || { echo "bench failed rc=$?"; tail -3 gpurun_out/crowd_c4.log | cut -c1-300; exit 1; }
grep '^{' gpurun_out/crowd_c4.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','ms_per_step','scan_kernel_ms','tail_kernel_ms','pair_kernel_ms','order_ms','hits')}, d.get('cpu_baseline',{}).get('parity_vs_gpu'))"
