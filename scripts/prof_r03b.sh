set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
KRE=scan_kernel bash scripts/profile.sh r03_c5 --config c5 --no-ref-model --cpu-budget 8 && \
KRE=scan_kernel bash scripts/profile.sh r03_c4 --config c4 --no-ref-model --cpu-budget 8
timeout -k 10 400 python -u scripts/ablate.py --config c4 --variants 0,60 --steps 5 --no-build > gpurun_out/abl_nt_c4.log 2>&1 && tail -4 gpurun_out/abl_nt_c4.log
timeout -k 10 400 python -u scripts/ablate.py --config c3 --variants 0,60 --steps 5 --no-build > gpurun_out/abl_nt_c3.log 2>&1 && tail -4 gpurun_out/abl_nt_c3.log
