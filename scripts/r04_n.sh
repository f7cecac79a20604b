#!/bin/bash
# A/B of the wide key groups over 16 keys per word (MP_KGRP4_KEYS=16, a 4 MB table): parity, then c4.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
T=${1:-r4n}
NR=$PWD/merpcr_amd/_lib/libmerpcr_hip_ablateMP_KGRP4_KEYS_16.so
MERPCR_LIB=$NR timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "wide_key_groups or iupac_wide or dense_tables" > gpurun_out/${T}_gputest.log 2>&1 \
    || { echo "gpu tests failed rc=$?"; grep -n "FAILED\|Error" gpurun_out/${T}_gputest.log | head; exit 1; }
tail -1 gpurun_out/${T}_gputest.log
for lib in "" NR "" NR; do
  L=""; [ "$lib" = NR ] && L=$NR
  MERPCR_LIB=$L timeout -k 10 300 python -u bench.py --config c4 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e \
      > gpurun_out/${T}_c4_$lib.log 2>&1 || { echo "bench c4 $lib rc=$?"; tail -5 gpurun_out/${T}_c4_$lib.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'step', d['ms_per_step'], 'single', d['single_run_ms'], 'scan', d['scan_kernel_ms'], 'tail', d['tail_kernel_ms'], 'pair', d['pair_kernel_ms'], 'order', d['order_ms'], 'hits', d['hits'], 'cand', d['candidates'])" gpurun_out/${T}_c4_$lib.log "c4 ${lib:-prod}"
done
