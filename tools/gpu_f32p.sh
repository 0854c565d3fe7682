#!/bin/bash
# fp32 persistent GEMM round trip on the box: its tests, the k_gemm_f32 A/B, the what-if table, one
# generate per dispatch, and a kernel-trace profile of generate (csv stats under gpurun_out/genprof).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "gemm_f32" > gpurun_out/f32p_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/f32p_tests.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -k "generate or decode" > gpurun_out/f32p_gen_tests.log 2>&1 || { echo "gen tests failed"; tail -20 gpurun_out/f32p_gen_tests.log; exit 1; }
timeout -k 10 200 python -u tools/f32_fwd_ab.py 3 > gpurun_out/f32p_ab.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/f32p_whatif.py 3 > gpurun_out/f32p_whatif.txt 2>&1 || exit 1
for v in 98 0 98 0; do timeout -k 10 120 python -u tools/f32_fwd_ab.py gen $v >> gpurun_out/f32p_ab.txt 2>&1 || exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/genprof -o run -- python3 $R/tools/f32_fwd_ab.py gen 0 > $R/gpurun_out/genprof.log 2>&1 || exit 1
echo ok
