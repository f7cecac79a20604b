#!/bin/bash
# GPU round trip: the -m gpu suite, the smoke test and one default bench line.
# usage: bash scripts/gpu_check.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-chk}; K=${2:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
KARG=()
[ -n "$K" ] && KARG=(-k "$K")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KARG[@]}" \
    > gpurun_out/${TAG}_gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -3 gpurun_out/${TAG}_gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
    || { echo "smoke failed rc=$?"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 700 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 \
    || { echo "bench failed rc=$?"; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
# the N-rank path with no outside launcher: bench.py --gpus 2 starts torch.distributed.run itself
timeout -k 10 400 python -u bench.py --gpus 2 --rehearse-one-gpu --steps 5 --warmup 2 \
    > gpurun_out/${TAG}_rehearse2.log 2>&1 \
    || { echo "rehearse2 failed rc=$?"; tail -20 gpurun_out/${TAG}_rehearse2.log; exit 1; }
grep '^{' gpurun_out/${TAG}_rehearse2.log | tail -1
