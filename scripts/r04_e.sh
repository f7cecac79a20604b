#!/bin/bash
# c4 step A/B (hit decode by bucket sequence ranges) against the r03 build, the CLI end to
# end from a FASTA file (device ingestion), and the multi-device host overhead.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
T=${1:-r4e}
SHARD=1 CFG=c4 bash scripts/r04_ab.sh ${T}_c4 r03=R03 prod= r03b=R03 prod2= || exit 1
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-file > gpurun_out/${T}_c3_e2e.log 2>&1 || { echo "e2e rc=$?"; tail -5 gpurun_out/${T}_c3_e2e.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c3', d['ms_per_step'], d['single_run_ms'], 'e2e', d.get('e2e'), 'e2e_file', d.get('e2e_file'))" gpurun_out/${T}_c3_e2e.log
timeout -k 10 300 python -u scripts/multi_overhead.py 0.125 0,0 > gpurun_out/${T}_multi.log 2>&1 || { echo "multi rc=$?"; tail -20 gpurun_out/${T}_multi.log; exit 1; }
tail -1 gpurun_out/${T}_multi.log
