#!/bin/bash
# 1/8 c3 step A/B: variant libraries (scripts/build_ab.py) and search options.
# usage: bash scripts/r04_ab.sh <tag> <name>=<lib-suffix or ''>[:opts] ...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
T=$1; shift
SHARD=${SHARD:-8}; CFG=${CFG:-c3}
for spec in "$@"; do
  name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; opts=""
  [ "$rest" != "$lib" ] && opts=${rest#*:}
  L=""; [ -n "$lib" ] && L=$PWD/merpcr_amd/_lib/libmerpcr_hip_ablate$lib.so
  EXTRA=(); [ -n "$opts" ] && EXTRA=(--opts "$opts")
  MERPCR_LIB=$L timeout -k 10 300 python -u bench.py --config $CFG --shard-of $SHARD --steps 30 --warmup 5 --no-cpu-baseline --no-e2e "${EXTRA[@]}" \
      > gpurun_out/${T}_${name}.log 2>&1 || { echo "bench $name rc=$?"; tail -5 gpurun_out/${T}_${name}.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'step', d['ms_per_step'], 'single', d['single_run_ms'], 'scan', d['scan_kernel_ms'], 'tail', d['tail_kernel_ms'], 'pair', d['pair_kernel_ms'], 'order', d['order_ms'], 'hits', d['hits'], (d.get('parity_distributed') or {}).get('ok'))" gpurun_out/${T}_${name}.log $name
done
