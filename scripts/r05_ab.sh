#!/bin/bash
# Same-box A/B of bench lines: each "name|ENV=VAL ...|bench args" spec runs twice, interleaved.
# usage: bash scripts/r05_ab.sh <tag> <spec> [<spec> ...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for rep in 1 2; do
  for spec in "$@"; do
    IFS='|' read -r name envs bargs <<< "$spec"
    log=gpurun_out/${TAG}_${name}_${rep}.log
    env $envs timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-e2e --no-pmc $bargs > "$log" 2>&1 \
        || { echo "$name failed rc=$?"; tail -5 "$log"; exit 1; }
    grep '^{' "$log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', 'step', d['ms_per_step'], 'scan', d['scan_kernel_ms'], 'tail', d['tail_kernel_ms'], 'pair', d['pair_kernel_ms'], 'order', d['order_ms'], 'hits', d['hits'], 'single', d['single_run_ms'])"
  done
done
