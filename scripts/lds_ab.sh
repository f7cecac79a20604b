#!/bin/bash
# Level-1 LDS prefilter A/B: bits per key k = 2 (product) vs 3 (MP_LDS_K=3),
# c3 bench line plus PMC passes of scan_kernel for each.  usage: bash scripts/lds_ab.sh <tag>
set -o pipefail
TAG=${1:-r03_ldsab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="--config c3 --no-e2e --no-cpu-baseline --no-ref-model --one-stream"
for K in 2 3; do
  MP_LDS_K=$K timeout -k 10 300 python3 "$R/bench.py" $B > "$OUT/bench_k$K.log" 2>&1 || { echo "bench k$K failed"; tail -5 "$OUT/bench_k$K.log"; exit 1; }
  tail -n 1 "$OUT/bench_k$K.log" | cut -c1-300
  for P in "lds:SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" "tcc:TCC_HIT_sum TCC_MISS_sum" \
           "sq:SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "fetch:FETCH_SIZE"; do
    name=${P%%:*}; ctrs=${P#*:}
    MP_LDS_K=$K timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-include-regex scan_kernel -d "$OUT/k${K}_$name" -o run --output-format csv \
        -- python3 "$R/bench.py" $B --steps 3 --warmup 1 > "$OUT/k${K}_$name.log" 2>&1 || { echo "pmc $name k$K failed"; tail -5 "$OUT/k${K}_$name.log"; exit 1; }
  done
  echo "k$K pmc ok"
done
