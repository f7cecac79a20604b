#!/bin/bash
# Round 6 stage table for the specialised-waves question: level 1 alone
# (1), level 2 on hashed level-1 positives without LDS reads (7), the genome stream with claims
# (5) and without (8), beside the product (0); c3 and c5.  Then the 1/8 c3 step twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for c in c3 c5; do
  timeout -k 10 400 python3 -u scripts/ablate.py --no-build --config $c --steps 5 --variants 0,1,7,5,8,0,1,7,5,8 \
      > gpurun_out/r6l_$c.log 2>&1 || { echo "ablate $c failed rc=$?"; tail -5 gpurun_out/r6l_$c.log; exit 1; }
  grep '^variant' gpurun_out/r6l_$c.log
done
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --shard-of 8 --steps 40 --warmup 5 --no-cpu-baseline --no-e2e --no-pmc \
      > gpurun_out/r6l_sh8_$i.log 2>&1 || { echo "bench sh8 failed rc=$?"; tail -5 gpurun_out/r6l_sh8_$i.log; exit 1; }
  grep '^{' gpurun_out/r6l_sh8_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('sh8 step', d['ms_per_step'], 'scan', d['scan_kernel_ms'], 'tail', d['tail_kernel_ms'], 'pair', d['pair_kernel_ms'], 'order', d['order_ms'], 'ok', d['parity_distributed']['ok'])"
done
