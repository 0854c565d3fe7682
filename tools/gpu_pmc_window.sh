#!/bin/bash
# C5 window launches: per-launch times, then the PMC passes (tools/pmc_run.sh) over them
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/f32_window_ops.py > gpurun_out/f32win_times.txt 2>&1 || { cat gpurun_out/f32win_times.txt; exit 1; }
timeout -k 10 900 bash tools/pmc_run.sh f32win6 tools/f32_window_ops.py || exit 1
echo ok
