#!/bin/bash
# Split-seed / hit-order round trip: parity tests, then c5 and c4 bench lines and a FETCH_SIZE
# pass over c5's scan kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py "tests/test_gpu_fullscale.py::test_full_table_prefix_vs_c_oracle" \
    tests/test_gpu_parity.py -k "split or c5 or c4 or crowded or repeat_order or dense or golden" -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/split_test.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/split_test.log; exit 1; }
tail -2 gpurun_out/split_test.log
for c in c5 c4; do
timeout -k 10 400 python -u bench.py --config $c --no-e2e --no-ref-model --steps 10 --warmup 3 > gpurun_out/split_$c.log 2>&1 || { echo "bench failed rc=$?"; tail -3 gpurun_out/split_$c.log | cut -c1-300; exit 1; }
grep '^{' gpurun_out/split_$c.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','ms_per_step','scan_kernel_ms','tail_kernel_ms','pair_kernel_ms','order_ms','hits')}, d.get('cpu_baseline',{}).get('parity_vs_gpu'))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex scan_kernel -d $R/gpurun_out/split_fetch -o run --output-format csv -- python3 $R/bench.py --config c5 --no-e2e --no-ref-model --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/split_fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
echo fetch ok
