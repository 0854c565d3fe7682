#!/bin/bash
# embedding forward rows kernel + head logits staged through LDS: tests (stop on failure), then the C2 step
# against the previous commit's library (libcharpt_hip_prev.so), same box, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_train.py -m gpu > gpurun_out/r3s3_small_tests2.log 2>&1 || { tail -30 gpurun_out/r3s3_small_tests2.log; exit 4; }
tail -1 gpurun_out/r3s3_small_tests2.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "embedding or head or cross" -m gpu > gpurun_out/r3s3_small_tests.log 2>&1 || { tail -30 gpurun_out/r3s3_small_tests.log; exit 5; }
tail -1 gpurun_out/r3s3_small_tests.log
for r in a b c; do
  CHARPT_LIB=replicatinggpt_amd/libcharpt_hip_prev.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-generate --no-census --steps 60 2>&1 | grep timed | sed "s/^/prev $r /" || exit 7
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-generate --no-census --steps 60 2>&1 | grep timed | sed "s/^/new $r /" || exit 8
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3s3_prof_small -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-generate --no-census > $GRAFT_REPO_ROOT/gpurun_out/r3s3_prof_small.log 2>&1 || exit 9
