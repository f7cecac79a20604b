#!/bin/bash
# Whole GPU suite, then c4 / c3 A/B of tail_kernel's references per thread (MP_TAIL_R).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
T=${1:-r4j}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1 \
    || { echo "gpu tests failed rc=$?"; grep -n "FAILED\|Error" gpurun_out/${T}_gputest.log | head; tail -5 gpurun_out/${T}_gputest.log; exit 1; }
tail -1 gpurun_out/${T}_gputest.log
for cfg in c4 c3; do
  for lib in "" MP_TAIL_R_1 MP_TAIL_R_4_MP_TAIL_BPC_1 ""; do
    L=""; [ -n "$lib" ] && L=$PWD/merpcr_amd/_lib/libmerpcr_hip_ablate$lib.so
    MERPCR_LIB=$L timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-e2e \
        > gpurun_out/${T}_${cfg}_$lib.log 2>&1 || { echo "bench $cfg $lib rc=$?"; tail -5 gpurun_out/${T}_${cfg}_$lib.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'step', d['ms_per_step'], 'single', d['single_run_ms'], 'scan', d['scan_kernel_ms'], 'tail', d['tail_kernel_ms'], 'pair', d['pair_kernel_ms'], 'order', d['order_ms'], 'hits', d['hits'])" gpurun_out/${T}_${cfg}_$lib.log "$cfg ${lib:-prod}"
  done
done
