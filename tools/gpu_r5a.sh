#!/bin/bash
# round 5: ABI flags / per-stream deferral tests + DP-path timing at W = 1
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_library.py tests/test_gpu_train.py \
  "tests/test_gpu_ops.py::test_gemm_bf16_slabs" "tests/test_gpu_ops.py::test_deferred_partial_reduces_match_immediate" \
  > gpurun_out/r5a_tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/step_ab.py c2 single,seg1,seg2,seg6,red 5 50 > gpurun_out/r5_step_ab.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --overlap 1 --no-census --no-generate --no-cpu-baseline --steps 200 \
  > gpurun_out/r5_bench_overlap.json 2> gpurun_out/r5_bench_overlap.err
