#!/bin/bash
# Round-3 profile set of the final code: trace + PMC passes per config (scripts/profile.sh),
# then the one-GPU rehearsals of the 2- and 4-rank paths (diagnostic, not the metric).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd)
bash scripts/profile.sh r03 --e2e-file && \
KRE=scan_kernel bash scripts/profile.sh r03_c5 --config c5 --no-ref-model --cpu-budget 8 && \
KRE=scan_kernel bash scripts/profile.sh r03_c4 --config c4 --no-ref-model --cpu-budget 8 && \
KRE=scan_kernel bash scripts/profile.sh r03_c2 --config c2 --no-ref-model --cpu-budget 8 || exit 1
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29400 + n)) bench.py --gpus $n --rehearse-one-gpu --no-ref-model --no-e2e --steps 10 --warmup 3 \
      > gpurun_out/r03_rehearse$n.log 2>&1 || { echo "rehearse $n failed rc=$?"; tail -5 gpurun_out/r03_rehearse$n.log; exit 1; }
  grep '^{' gpurun_out/r03_rehearse$n.log | tail -1 | cut -c1-300
done
