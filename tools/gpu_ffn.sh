#!/bin/bash
# Fused fp32 FFN round trip on the box: its tests, the generate / decode tests, and generate 256 x 500
# with the fused FFN off / on (CHARPT_FFN_FUSED), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "ffn_f32 or gemm_f32" > gpurun_out/ffn_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ffn_tests.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -k "generate or decode" > gpurun_out/ffn_gen_tests.log 2>&1 || { echo "gen tests failed"; tail -30 gpurun_out/ffn_gen_tests.log; exit 1; }
: > gpurun_out/ffn_ab.txt
for f in 0 1 0 1; do CHARPT_FFN_FUSED=$f timeout -k 10 120 python -u tools/f32_fwd_ab.py gen 0 2>&1 | grep -v amdgpu | sed "s/^/fused=$f /" >> gpurun_out/ffn_ab.txt || exit 1; done
echo ok
