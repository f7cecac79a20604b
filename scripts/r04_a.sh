#!/bin/bash
# round 4: GPU tests, the 4.5 Gbp diagnostic, then the 1/8 c3 step: product (steal + fused
# tails), no steal, no fused tails
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
T=${1:-r4a}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -40 gpurun_out/${T}_gputest.log; exit 1; }
tail -2 gpurun_out/${T}_gputest.log
bench1() {  # name, lib, extra args
    local v=$1 L=$2; shift 2
    MERPCR_LIB=$L timeout -k 10 300 python -u bench.py --shard-of 8 --steps 30 --warmup 5 --no-cpu-baseline --no-e2e "$@" \
        > gpurun_out/${T}_sh8_${v}.log 2>&1 || { echo "bench $v rc=$?"; tail -5 gpurun_out/${T}_sh8_${v}.log; return 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'step', d['ms_per_step'], 'single', d['single_run_ms'], 'scan', d['scan_kernel_ms'], 'tail', d['tail_kernel_ms'], 'pair', d['pair_kernel_ms'], 'order', d['order_ms'], 'hits', d['hits'], d['parity_distributed']['ok'])" gpurun_out/${T}_sh8_${v}.log $v
}
NS=$PWD/merpcr_amd/_lib/libmerpcr_hip_nosteal.so
for i in 1 2; do
  bench1 prod_$i "" && bench1 nosteal_$i $NS && bench1 nofuse_$i "" --opts fuse_tails=0 || exit 1
done
