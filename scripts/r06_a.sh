#!/bin/bash
# Round 6, first GPU pass: the deferred ambiguity-word join (prefetch no longer waited at issue).
# Stage variants old vs new on c5 and c3, same-box product A/B on c3/c4/c5, then the GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
OLD=merpcr_amd/_lib/ab/libmerpcr_hip_r05
for cfg in c5 c3; do
  timeout -k 10 300 python3 -u scripts/ablate.py --no-build --config $cfg --steps 8 \
      --variants lib:${OLD}_v5.so,5,lib:${OLD}_v1.so,1,lib:${OLD}.so,0 > gpurun_out/r6a_stage_$cfg.log 2>&1 \
      || { echo "stage $cfg failed rc=$?"; tail -5 gpurun_out/r6a_stage_$cfg.log; exit 1; }
  grep '^variant' gpurun_out/r6a_stage_$cfg.log
done
bash scripts/r05_ab.sh r6a "old3|MERPCR_LIB=$OLD.so|--config c3 --steps 20 --warmup 5" "new3||--config c3 --steps 20 --warmup 5" \
    "old5|MERPCR_LIB=$OLD.so|--config c5 --steps 10 --warmup 3" "new5||--config c5 --steps 10 --warmup 3" \
    "old4|MERPCR_LIB=$OLD.so|--config c4 --steps 10 --warmup 3" "new4||--config c4 --steps 10 --warmup 3" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r6a_gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 gpurun_out/r6a_gputest.log; exit 1; }
tail -3 gpurun_out/r6a_gputest.log
