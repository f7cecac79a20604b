#!/bin/bash
# Round 6 final build, part B: 1/8 owned range (shard curve + pipelined 1/8 bench line with
# distributed parity), then the c2/c4/c5 rocprofv3 sets.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/shard_curve.py > gpurun_out/r06_curve.log 2>&1 \
    || { echo "shard_curve failed rc=$?"; tail -5 gpurun_out/r06_curve.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_curve.log
timeout -k 10 300 python3 -u bench.py --shard-of 8 --steps 30 --warmup 5 --no-e2e \
    > gpurun_out/r06_sh8.log 2>&1 || { echo "bench sh8 failed rc=$?"; tail -5 gpurun_out/r06_sh8.log; exit 1; }
grep '^{' gpurun_out/r06_sh8.log > gpurun_out/r06_shard8_bench.json
for c in c2 c4 c5; do
  KRE=scan_kernel timeout -k 10 400 bash scripts/profile.sh r06_$c --config $c --no-ref-model --cpu-budget 8 || exit 1
done
