#!/bin/bash
# round 3 session 3: grouped weight-gradient launch (defer_wgrad) -- tests first (stop on failure), then
# same-box A/B of the C2 step with it off / on
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "grouped or deferred or gemm_splitk or uneven" -m gpu > gpurun_out/r3s3_wg_tests.log 2>&1 || { tail -30 gpurun_out/r3s3_wg_tests.log; exit 5; }
tail -1 gpurun_out/r3s3_wg_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_dp.py tests/test_gpu_model.py -m gpu > gpurun_out/r3s3_wg_tests2.log 2>&1 || { tail -30 gpurun_out/r3s3_wg_tests2.log; exit 6; }
tail -1 gpurun_out/r3s3_wg_tests2.log
for r in a b; do
  CHARPT_DEFER_WGRAD=0 timeout -k 10 200 python bench.py --no-cpu-baseline --no-generate --no-census --steps 60 2>&1 | grep timed | sed "s/^/wg0 $r /" || exit 7
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-generate --no-census --steps 60 2>&1 | grep timed | sed "s/^/wg1 $r /" || exit 8
done
CHARPT_DEFER_WGRAD=0 timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --no-generate --no-census --steps 8 --warmup 3 2>&1 | grep timed | sed "s/^/c4 wg0 /" || exit 9
timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --no-generate --no-census --steps 8 --warmup 3 2>&1 | grep timed | sed "s/^/c4 wg1 /" || exit 10
