#!/bin/bash
# 8-wave row-linear workgroups (linear_rows_nb 3) against the default 4-wave ones: the row-linear tests
# (every form bitwise), generate with each, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "linear_rows" > gpurun_out/rows8_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/rows8_tests.log; exit 1; }
: > gpurun_out/rows8_ab.txt
for r in 1 2 3; do for nb in 0 3; do timeout -k 10 120 python -u tools/f32_fwd_ab.py gen $nb linear_rows_nb 2>&1 | grep -v amdgpu >> gpurun_out/rows8_ab.txt || exit 1; done; done
echo ok
