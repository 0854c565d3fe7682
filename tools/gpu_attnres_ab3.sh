#!/bin/bash
# resident fp32 attention operand-read variants: the fp32 attention / generate tests on the in-tree
# library, then generate 256 x 500 with base / b4 / in-tree libraries, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -k "fp32 or generate or decode" > gpurun_out/ab3_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ab3_tests.log; exit 1; }
: > gpurun_out/ab3.txt
for r in 1 2; do for l in base b4 cur; do
  if [ $l = cur ]; then unset CHARPT_LIB; else export CHARPT_LIB=$PWD/replicatinggpt_amd/libcharpt_hip_$l.so; fi
  timeout -k 10 120 python -u tools/f32_fwd_ab.py gen 0 2>&1 | grep -v amdgpu | sed "s/^/lib=$l /" >> gpurun_out/ab3.txt || exit 1
done; done
echo ok
