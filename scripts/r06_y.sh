#!/bin/bash
# Round 6: mp_search.hip under alternative AMDGPU machine-scheduler settings (scripts/build_sched_variants.py)
# against the product, c3 / c4 / c5, same box (ablate.py event times; hit counts must match).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
L=merpcr_amd/_lib
V="0,lib:$L/libmerpcr_hip_schedilp.so,lib:$L/libmerpcr_hip_schedmemclause.so,lib:$L/libmerpcr_hip_schedbias0.so"
for c in c3 c4 c5; do
  timeout -k 10 500 python3 -u scripts/ablate.py --no-build --config $c --steps 5 --variants $V,$V \
      > gpurun_out/r6y_$c.log 2>&1 || { echo "ablate $c failed rc=$?"; tail -5 gpurun_out/r6y_$c.log; exit 1; }
  echo "== $c"; grep '^variant' gpurun_out/r6y_$c.log | sed 's/merpcr_amd\/_lib\/libmerpcr_hip_//'
done
