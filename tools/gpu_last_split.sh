#!/bin/bash
# window step's last block: K/V for every row + Q for the final rows (CHARPT_LAST_KV_SPLIT) -- the
# generate / decode tests, then generate 256 x 500 with the split off / on, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "generate or decode" > gpurun_out/lsplit_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/lsplit_tests.log; exit 1; }
: > gpurun_out/lsplit_ab.txt
for r in 1 2 3; do for v in 0 1; do
  CHARPT_LAST_KV_SPLIT=$v timeout -k 10 120 python -u tools/f32_fwd_ab.py gen 0 2>&1 | grep -v amdgpu | sed "s/^/last_kv_split=$v /" >> gpurun_out/lsplit_ab.txt || exit 1
done; done
echo ok
