#!/bin/bash
# Round-3 final evidence: -m gpu suite + smoke, the profile set of every config
# (scripts/profile.sh), one-GPU 2/4-rank rehearsals, and the 1/8 and 1/4 shard bench lines.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/fin_gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -40 gpurun_out/fin_gputest.log; exit 1; }
tail -1 gpurun_out/fin_gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 \
    || { echo "smoke failed rc=$?"; tail -20 gpurun_out/fin_smoke.log; exit 1; }
bash scripts/prof_r03.sh || exit 1
for b in "sh8:--shard-of 8 --no-e2e --no-ref-model --steps 50 --warmup 5" "sh4:--shard-of 4 --no-e2e --no-ref-model --steps 30 --warmup 5"; do
  name=${b%%:*}; args=${b#*:}
  timeout -k 10 400 python -u bench.py $args > gpurun_out/fin_bench_$name.log 2>&1 \
      || { echo "bench $name failed rc=$?"; tail -5 gpurun_out/fin_bench_$name.log; exit 1; }
  grep '^{' gpurun_out/fin_bench_$name.log | tail -1 | cut -c1-200
done
