#!/bin/bash
# A/B counters of scan-kernel variants on the same c3 data (scripts/ablate.py variants),
# one rocprofv3 --pmc pass per counter group and variant.
# usage: bash scripts/pmc_ab.sh <tag> <config> <variant> [variant...]
set -o pipefail
TAG=$1; CFG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcab_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
KRE=${KRE:-scan_kernel}
NB=""; [ -n "$NOBUILD" ] && NB="--no-build"   # variant libraries built beforehand (CPU side)
GROUPS_N=${GROUPS_N:-4}                        # the first N counter groups only
for V in "$@"; do
  T=$(echo "$V" | tr -c 'A-Za-z0-9\n' '_')
  timeout -k 10 300 python3 "$R/scripts/ablate.py" --config $CFG --variants "$V" --steps 5 $NB > "$OUT/${T}_time.log" 2>&1 \
      || { echo "time $V failed rc=$?"; tail -5 "$OUT/${T}_time.log"; exit 1; }
  grep "^variant" "$OUT/${T}_time.log"
  i=0
  GL=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
      "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"
      "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum")
  for G in "${GL[@]:0:$GROUPS_N}"; do
    timeout -s KILL 240 rocprofv3 --pmc $G --kernel-include-regex "$KRE" -d "$OUT/${T}_p$i" -o run --output-format csv \
        -- python3 "$R/scripts/ablate.py" --config $CFG --variants "$V" --steps 2 $NB > "$OUT/${T}_p$i.log" 2>&1 \
        || { echo "pass $V $i failed rc=$?"; tail -5 "$OUT/${T}_p$i.log"; exit 1; }
    i=$((i+1))
  done
done
python3 "$R/scripts/pmc_table.py" "$OUT"
