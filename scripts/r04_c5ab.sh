#!/bin/bash
# c5 single-pass question: scan time of the product split-seed scans, of level 1
# alone (variant 1) and of the genome stream + validity + scheduler alone (variant 5, the part
# two seed scans could share), and the product with 64 KiB prefilters (MP_LDS_LOG2=19, what
# two filters in one CU's LDS would have); PMC: VALU / LDS / L2 requests per variant.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
NOBUILD=1 GROUPS_N=${GROUPS_N:-3} KRE=scan_kernel bash scripts/pmc_ab.sh ${1:-c5ab} c5 0 1 5 MP_LDS_LOG2=19
