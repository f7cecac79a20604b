#!/bin/bash
# c4 A/B of the wide key groups' reference reservation size (MP_REF_CHUNK 128 / 256 / 512).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
T=${1:-r4s}
for lib in "" MP_REF_CHUNK_512 MP_REF_CHUNK_128 "" MP_REF_CHUNK_512 MP_REF_CHUNK_128; do
  L=""; [ -n "$lib" ] && L=$PWD/merpcr_amd/_lib/libmerpcr_hip_ablate$lib.so
  MERPCR_LIB=$L timeout -k 10 300 python -u bench.py --config c4 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e \
      > gpurun_out/${T}_c4_$lib.log 2>&1 || { echo "bench c4 $lib rc=$?"; tail -5 gpurun_out/${T}_c4_$lib.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'step', d['ms_per_step'], 'single', d['single_run_ms'], 'scan', d['scan_kernel_ms'], 'tail', d['tail_kernel_ms'], 'hits', d['hits'])" gpurun_out/${T}_c4_$lib.log "c4 ${lib:-prod}"
done
