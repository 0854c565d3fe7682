#!/bin/bash
# Kernel trace of one C5 generate (256 x 500, greedy, fp32) for the per-kernel breakdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/genprof -o gen -- python3 -u tools/f32_fwd_ab.py gen 0 > gpurun_out/genprof.log 2>&1 || { tail -20 gpurun_out/genprof.log; exit 1; }
find gpurun_out/genprof -name "*.csv" | head
echo ok
