#!/bin/bash
# c4 A/B of the crowded-bucket sort's grid (MP_CROWD_GRID; tuning, not a product switch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for g in 256 64 32 128; do
MP_CROWD_GRID=$g timeout -k 10 400 python -u bench.py --config c4 --no-e2e --no-ref-model --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/cg_$g.log 2>&1 || { echo "bench failed rc=$?"; tail -3 gpurun_out/cg_$g.log | cut -c1-300; exit 1; }
grep '^{' gpurun_out/cg_$g.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('grid $g', {k: d.get(k) for k in ('value','ms_per_step','scan_kernel_ms','pair_kernel_ms','order_ms','hits')})"
done
