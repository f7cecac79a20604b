#!/bin/bash
# Per-stage instruction and time budget of the c3 scan: the product and the
# timing-only variants 1 (level 1), 2 (+ the positives' list), 3 (+ the level-2 loads,
# consumed), each with the SQ instruction counters and the L2 requests (scripts/pmc_ab.sh).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
NOBUILD=1 GROUPS_N=2 KRE=scan_kernel bash scripts/pmc_ab.sh ${1:-c3stage} c3 0 1 2 3
