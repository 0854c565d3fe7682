#!/bin/bash
# fp32 resident attention forward: its bitwise tests and generate with the previous / current library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -k "fp32 or generate or decode or f32" > gpurun_out/attnres_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/attnres_tests.log; exit 1; }
: > gpurun_out/attnres_ab.txt
for r in 1 2; do for l in prev cur; do
  if [ $l = prev ]; then export CHARPT_LIB=$PWD/replicatinggpt_amd/libcharpt_hip_prev.so; else unset CHARPT_LIB; fi
  timeout -k 10 120 python -u tools/f32_fwd_ab.py gen 0 2>&1 | grep -v amdgpu | sed "s/^/lib=$l /" >> gpurun_out/attnres_ab.txt || exit 1
done; done
echo ok
