#!/bin/bash
# Wide I = 1 key groups (kgrp4): targeted GPU parity, then c4 A/B against the rank-head path.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
T=${1:-r4g}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "wide_key_groups or iupac_wide or dense_tables or synthetic_vs_oracle" > gpurun_out/${T}_gputest.log 2>&1 \
    || { echo "gpu tests failed rc=$?"; tail -30 gpurun_out/${T}_gputest.log; exit 1; }
tail -1 gpurun_out/${T}_gputest.log
for v in 0 1 0 1; do
  MP_NO_KGRP4=$v timeout -k 10 300 python -u bench.py --config c4 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e \
      > gpurun_out/${T}_c4_no4_$v.log 2>&1 || { echo "bench c4 no4=$v rc=$?"; tail -5 gpurun_out/${T}_c4_no4_$v.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'step', d['ms_per_step'], 'single', d['single_run_ms'], 'scan', d['scan_kernel_ms'], 'tail', d['tail_kernel_ms'], 'pair', d['pair_kernel_ms'], 'order', d['order_ms'], 'hits', d['hits'], d.get('parity_vs_gpu'))" gpurun_out/${T}_c4_no4_$v.log no4=$v
done
timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/${T}_c3.log 2>&1 || { echo "bench c3 rc=$?"; tail -5 gpurun_out/${T}_c3.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c3 step', d['ms_per_step'], 'single', d['single_run_ms'], 'scan', d['scan_kernel_ms'], 'tail', d['tail_kernel_ms'], 'pair', d['pair_kernel_ms'], 'order', d['order_ms'], 'hits', d['hits'])" gpurun_out/${T}_c3.log
