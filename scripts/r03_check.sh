#!/bin/bash
# Round-3 round trip: -m gpu suite, smoke, default bench, shard-of 8/4 bench lines and a
# kernel/copy trace of the shard-of-8 step.  usage: bash scripts/r03_check.sh <tag> [pytest -k]
set -o pipefail
TAG=${1:-r3}; K=${2:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
KARG=()
[ -n "$K" ] && KARG=(-k "$K")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KARG[@]}" \
    > gpurun_out/${TAG}_gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -40 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -3 gpurun_out/${TAG}_gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
    || { echo "smoke failed rc=$?"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
for b in "def:" "sh8:--shard-of 8 --no-e2e --steps 50 --warmup 5" "sh4:--shard-of 4 --no-e2e --steps 30 --warmup 5"; do
  name=${b%%:*}; args=${b#*:}
  timeout -k 10 400 python -u bench.py $args > gpurun_out/${TAG}_bench_$name.log 2>&1 \
      || { echo "bench $name failed rc=$?"; tail -20 gpurun_out/${TAG}_bench_$name.log; exit 1; }
  tail -n 1 gpurun_out/${TAG}_bench_$name.log | cut -c1-400
done
bash scripts/trace_steps.sh ${TAG}_sh8 --shard-of 8 && python scripts/timeline_summary.py gpurun_out/trace_${TAG}_sh8 gpurun_out/${TAG}_sh8_timeline.csv
