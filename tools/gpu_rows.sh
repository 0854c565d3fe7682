#!/bin/bash
# Row-resident fp32 Linears (ln1 + QKV, projection + residual) round trip: their tests, the generate /
# decode / fused-model tests, and generate 256 x 500 with CHARPT_ATTN_ROWS off / on, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "linear_rows or ffn_f32 or gemm_f32" > gpurun_out/rows_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/rows_tests.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -k "generate or decode or fused_ffn" > gpurun_out/rows_gen_tests.log 2>&1 || { echo "gen tests failed"; tail -30 gpurun_out/rows_gen_tests.log; exit 1; }
: > gpurun_out/rows_ab.txt
for r in 1 2; do for nb in 0 1; do timeout -k 10 120 python -u tools/f32_fwd_ab.py gen $nb linear_rows_nb 2>&1 | grep -v amdgpu >> gpurun_out/rows_ab.txt || exit 1; done; done
echo ok
