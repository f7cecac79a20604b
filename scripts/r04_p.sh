#!/bin/bash
# Same-box A/B of the final build against the build before the wide key groups (PRE, 9ee0d2b).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
T=${1:-r4p}
for cfg in c3 c4 c5; do
  for lib in "" PRE "" PRE; do
    L=""; [ -n "$lib" ] && L=$PWD/merpcr_amd/_lib/libmerpcr_hip_ablate$lib.so
    MERPCR_LIB=$L timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-e2e \
        > gpurun_out/${T}_${cfg}_$lib.log 2>&1 || { echo "bench $cfg $lib rc=$?"; tail -5 gpurun_out/${T}_${cfg}_$lib.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'step', d['ms_per_step'], 'single', d['single_run_ms'], 'scan', d['scan_kernel_ms'], 'tail', d['tail_kernel_ms'], 'pair', d['pair_kernel_ms'], 'order', d['order_ms'], 'hits', d['hits'])" gpurun_out/${T}_${cfg}_$lib.log "$cfg ${lib:-prod}"
  done
done
