set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash scripts/profile.sh r03 --e2e-file && KRE=scan_kernel bash scripts/profile.sh r03_c2 --config c2 --no-ref-model --cpu-budget 8
