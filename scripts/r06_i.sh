#!/bin/bash
# Round 6: the scan's first chunks claimed per block (a late block takes what is left) against
# the product's static first chunks; both with the default pipeline and with the deeper one
# (4 handles, 2 streams, 2 steps ahead) that had let two scans share the CUs; then the whole
# GPU suite on the new library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=merpcr_amd/_lib
S=MERPCR_LIB=$L/libmerpcr_hip_ablateMP_R6SCHED_1.so
MERPCR_LIB=$L/libmerpcr_hip_ablateMP_R6SCHED_1.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r6i_gputest.log 2>&1 \
    || { echo "gpu tests failed rc=$?"; tail -30 gpurun_out/r6i_gputest.log; exit 1; }
tail -2 gpurun_out/r6i_gputest.log
for cfg in "c3|--config c3 --steps 5 --warmup 2" "c4|--config c4 --steps 10 --warmup 3" "s8|--config c3 --shard-of 8 --steps 40 --warmup 5" "c3l|--config c3 --steps 20 --warmup 5"; do
  IFS='|' read -r cn cargs <<< "$cfg"
  bash scripts/r05_ab.sh r6i_$cn "prod||$cargs" "sched|$S|$cargs" "prodd2||$cargs --handles 4 --streams 2 --depth 2" \
      "schedd2|$S|$cargs --handles 4 --streams 2 --depth 2" || exit 1
done
