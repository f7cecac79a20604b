set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash scripts/profile.sh r02 --e2e-file && \
KRE=scan_kernel bash scripts/profile.sh r02_c4 --config c4 --no-ref-model --cpu-budget 8 && \
KRE=dense_kernel bash scripts/profile.sh r02_c5 --config c5 --no-ref-model --cpu-budget 8 && \
KRE=scan_kernel bash scripts/profile.sh r02_c2 --config c2 --no-ref-model --cpu-budget 8
