#!/bin/bash
# Round 6 final build, part C: the shard lines (1/2, 1/4, 1/8 of c3, pipelined default, each
# with distributed parity) and the shard curve.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for k in 2 4 8; do
  timeout -k 10 300 python3 -u bench.py --shard-of $k --steps 30 --warmup 5 --no-e2e \
      > gpurun_out/r06f_sh$k.log 2>&1 || { echo "bench sh$k failed rc=$?"; tail -5 gpurun_out/r06f_sh$k.log; exit 1; }
  grep '^{' gpurun_out/r06f_sh$k.log | tail -1 > gpurun_out/r06_shard${k}_bench.json
  python3 -c "import json; d=json.load(open('gpurun_out/r06_shard${k}_bench.json')); print('sh$k', d['ms_per_step'], d['scan_kernel_ms'], d['parity_distributed']['ok'])"
done
timeout -k 10 300 python3 -u scripts/shard_curve.py > gpurun_out/r06_curve.log 2>&1 \
    || { echo "shard_curve failed rc=$?"; tail -5 gpurun_out/r06_curve.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_curve.log
