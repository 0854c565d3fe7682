#!/bin/bash
# get_batch offsets in the gather launch's kernel arguments (CHARPT_GATHER_ARGS): the gather / train /
# DP tests, then the C2 bench with it off / on, interleaved (bench lines to gpurun_out/gather_ab.txt)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_train.py -x -q --timeout 250 --timeout-method thread -k "gather or train_steps or segmented or get_batch" > gpurun_out/gather_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gather_tests.log; exit 1; }
: > gpurun_out/gather_ab.txt
for r in 1 2 3; do for v in 0 1; do
  CHARPT_GATHER_ARGS=$v timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-generate 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gather_args=$v', d['ms_per_step'], 'ms/step')" >> gpurun_out/gather_ab.txt || exit 1
done; done
echo ok
