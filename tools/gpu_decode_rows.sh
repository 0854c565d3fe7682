#!/bin/bash
# generate()'s per-token fp32 products: k_gemm_f32r (clamped loads, look-ahead chain) and the LayerNorm
# inside it (CHARPT_DECODE_ROWS): their tests, generate 256 x 500 with CHARPT_DECODE_ROWS 0 / 1
# interleaved, and a kernel trace of one generate
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -k "linear_rows or small_m or f32 or fp32 or generate or decode or qkv" > gpurun_out/drows_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/drows_tests.log; exit 1; }
: > gpurun_out/drows_ab.txt
for r in 1 2; do for v in 0 1; do
  CHARPT_DECODE_ROWS=$v timeout -k 10 120 python -u tools/f32_fwd_ab.py gen 0 2>&1 | grep -v amdgpu | sed "s/^/decode_rows=$v /" >> gpurun_out/drows_ab.txt || exit 1
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/genprof2 -o gen -- python3 -u tools/f32_fwd_ab.py gen 0 > gpurun_out/genprof2.log 2>&1 || { tail -20 gpurun_out/genprof2.log; exit 1; }
echo ok
