#!/bin/bash
# round 3 session 3: the 128x192 one-block-per-CU tile -- GEMM tests first (stop on any failure), then
# same-box A/B of the C2 step with the automatic pick vs the 128x128 tile forced, and the epilogue costs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "gemm" -m gpu > gpurun_out/r3s3_t192_tests.log 2>&1 || { tail -30 gpurun_out/r3s3_t192_tests.log; exit 5; }
tail -1 gpurun_out/r3s3_t192_tests.log
for r in a b; do
  CHARPT_TUNING=gemm_variant=9 timeout -k 10 200 python bench.py --no-cpu-baseline --no-generate --no-census --steps 60 2>&1 | grep timed | sed "s/^/v9 $r /" || exit 6
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-generate --no-census --steps 60 2>&1 | grep timed | sed "s/^/auto $r /" || exit 7
done
CHARPT_TUNING=gemm_variant=9 timeout -k 10 200 python tools/epi_cost.py > gpurun_out/r3s3_t192_epi_v9.log 2>&1 || exit 8
timeout -k 10 200 python tools/epi_cost.py > gpurun_out/r3s3_t192_epi_auto.log 2>&1 || exit 9
paste gpurun_out/r3s3_t192_epi_v9.log gpurun_out/r3s3_t192_epi_auto.log | grep -v amdgpu
