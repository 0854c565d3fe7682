#!/bin/bash
# resident fp32 attention with XCD-contiguous (b, h): fp32 attention / generate tests, generate with the
# base / in-tree library interleaved, the window launches' times, and one FETCH_SIZE / WRITE_SIZE pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/pmcx
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -k "fp32 or generate or decode or decode_attn" > gpurun_out/xcd_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/xcd_tests.log; exit 1; }
: > gpurun_out/xcd_ab.txt
for r in 1 2 3; do for l in base cur; do
  if [ $l = cur ]; then unset CHARPT_LIB; else export CHARPT_LIB=$R/replicatinggpt_amd/libcharpt_hip_$l.so; fi
  timeout -k 10 120 python -u tools/f32_fwd_ab.py gen 0 2>&1 | grep -v amdgpu | sed "s/^/lib=$l /" >> gpurun_out/xcd_ab.txt || exit 1
done; done
unset CHARPT_LIB
timeout -k 10 120 python -u tools/f32_window_ops.py > gpurun_out/xcd_times.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcx/f -o run -- python3 $R/tools/f32_window_ops.py > $R/gpurun_out/pmcx/f.log 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcx/w -o run -- python3 $R/tools/f32_window_ops.py > $R/gpurun_out/pmcx/w.log 2>&1 || exit 3
echo ok
