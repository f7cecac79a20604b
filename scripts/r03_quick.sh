#!/bin/bash
# Quick perf round trip: a few gpu tests (-k), then bench lines.  usage: bash scripts/r03_quick.sh <tag> "<-k expr>" "<args>;<args>"
set -o pipefail
TAG=$1; K=$2; BENCHES=$3
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" \
      > gpurun_out/${TAG}_test.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/${TAG}_test.log; exit 1; }
  tail -2 gpurun_out/${TAG}_test.log
fi
IFS=';' read -ra BS <<< "$BENCHES"
i=0
for b in "${BS[@]}"; do
  [ -z "$b" ] && continue
  timeout -k 10 400 python -u bench.py $b > gpurun_out/${TAG}_bench$i.log 2>&1 \
      || { echo "bench '$b' failed rc=$?"; tail -20 gpurun_out/${TAG}_bench$i.log; exit 1; }
  echo "== $b"; tail -n 1 gpurun_out/${TAG}_bench$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','ms_per_step','scan_kernel_ms','tail_kernel_ms','pair_kernel_ms','order_ms','hits')}, d.get('cpu_baseline',{}).get('parity_vs_gpu'), (d.get('parity_distributed') or {}).get('ok'))"
  i=$((i+1))
done
