#!/bin/bash
# rocprofv3 evidence for one round: kernel-trace stats of the bench command itself,
# then one PMC pass per counter set (never combined with tracing domains).
# usage: [KRE=dense_kernel] bash scripts/profile.sh <tag> [extra bench args...]
set -o pipefail
TAG=${1:-r01}; shift
KRE=${KRE:-scan_kernel}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # name, bench-args, rocprof args...
  local name=$1; local bargs=$2; shift 2
  timeout -k 10 400 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python3 "$R/bench.py" $bargs \
      > "$OUT/$name.log" 2>&1 || { echo "pass $name failed rc=$?"; tail -5 "$OUT/$name.log"; exit 1; }
  echo "pass $name ok"
}
run trace "--no-pmc $*" --kernel-trace --stats
Q="--no-cpu-baseline --no-pmc --steps 5 --warmup 1 $*"
run fetch "$Q" --pmc FETCH_SIZE --kernel-include-regex $KRE
run write "$Q" --pmc WRITE_SIZE --kernel-include-regex $KRE
run sq "$Q" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-include-regex $KRE
run tcc "$Q" --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex $KRE
run lds "$Q" --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-include-regex $KRE
