#!/bin/bash
# Full round trip: -m gpu suite, smoke, then one bench line per config (c3 default first).
# usage: bash scripts/r03_all.sh <tag> [configs...]
set -o pipefail
TAG=${1:-r3}; shift
CFGS=${@:-c3 c5 c4 c2}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -40 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -2 gpurun_out/${TAG}_gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
    || { echo "smoke failed rc=$?"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
for c in $CFGS; do
  timeout -k 10 400 python -u bench.py --config $c --no-ref-model > gpurun_out/${TAG}_bench_$c.log 2>&1 \
      || { echo "bench $c failed rc=$?"; tail -3 gpurun_out/${TAG}_bench_$c.log | cut -c1-400; exit 1; }
  grep '^{' gpurun_out/${TAG}_bench_$c.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', {k: d.get(k) for k in ('value','ms_per_step','scan_kernel_ms','tail_kernel_ms','pair_kernel_ms','order_ms','hits')}, d['roofline']['frac'], d.get('cpu_baseline',{}).get('parity_vs_gpu'))"
done
