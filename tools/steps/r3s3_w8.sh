#!/bin/bash
# resident attention forward with 8 one-group waves (attn_w8=1, default here) vs 4 two-group waves:
# attention tests (stop on failure), kernel A/B in one process, then the C2 step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "attention or attn" -m gpu > gpurun_out/r3s3_w8_tests.log 2>&1 || { tail -30 gpurun_out/r3s3_w8_tests.log; exit 5; }
tail -1 gpurun_out/r3s3_w8_tests.log
timeout -k 10 200 python tools/ab_interleave.py attn_fwd attn_w8 0,1 7 c2 2>&1 | grep -v amdgpu || exit 6
for r in a b; do
  CHARPT_TUNING=attn_w8=0 timeout -k 10 200 python bench.py --no-cpu-baseline --no-generate --no-census --steps 60 2>&1 | grep timed | sed "s/^/w4 $r /" || exit 7
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-generate --no-census --steps 60 2>&1 | grep timed | sed "s/^/w8 $r /" || exit 8
done
