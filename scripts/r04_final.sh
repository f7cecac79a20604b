#!/bin/bash
# Round-end check of the final build: the whole GPU suite, smoke(), then c3 / c4 / c5 beside the
# build before the wide key groups (PRE, 9ee0d2b) on the same box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
T=${1:-r4final}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1 \
    || { echo "gpu tests failed rc=$?"; grep -n "FAILED\|Error" gpurun_out/${T}_gputest.log | head; tail -5 gpurun_out/${T}_gputest.log; exit 1; }
tail -1 gpurun_out/${T}_gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
bash scripts/r04_p.sh ${T} || exit 1
