#!/bin/bash
# window step's last-block K / V written head-major (CHARPT_LAST_KV_HEADS): its tests, the generate /
# decode / linear-rows tests, generate with it off / on interleaved, and a kernel trace of one generate
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "generate or decode or linear_rows or head_major" > gpurun_out/lheads_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/lheads_tests.log; exit 1; }
: > gpurun_out/lheads_ab.txt
for r in 1 2 3; do for v in 0 1; do
  CHARPT_LAST_KV_HEADS=$v timeout -k 10 120 python -u tools/f32_fwd_ab.py gen 0 2>&1 | grep -v amdgpu | sed "s/^/last_kv_heads=$v /" >> gpurun_out/lheads_ab.txt || exit 1
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/genprof3 -o gen -- python3 -u tools/f32_fwd_ab.py gen 0 > gpurun_out/genprof3.log 2>&1 || { tail -20 gpurun_out/genprof3.log; exit 1; }
echo ok
