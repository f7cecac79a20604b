#!/bin/bash
# c5 round trip: split parity tests (+ the 48 Mbp full-table case), then the c5 profile set.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py "tests/test_gpu_fullscale.py::test_full_table_prefix_vs_c_oracle[c5-48000000-2]" -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/c5f_test.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/c5f_test.log; exit 1; }
tail -1 gpurun_out/c5f_test.log
KRE=scan_kernel bash scripts/profile.sh r03_c5 --config c5 --no-ref-model --cpu-budget 8
