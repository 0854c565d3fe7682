#!/bin/bash
# rocprofv3 kernel trace + stats of the default C2 bench (the round's profile evidence), then the
# in-step census table (tools/step_kernels.py).  usage: tools/gpu_prof_bench.sh <tag> [config]
set -o pipefail
tag=${1:-r5}; cfg=${2:-c2}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out/prof_$tag
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$tag -o run -- \
  python3 $R/bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-generate \
  > $R/gpurun_out/prof_$tag/bench.json 2> $R/gpurun_out/prof_$tag/bench.err || exit $?
trace=$(find $R/gpurun_out/prof_$tag -name 'run_kernel_trace.csv' | head -1)
stats=$(find $R/gpurun_out/prof_$tag -name 'run_kernel_stats.csv' | head -1)
cp "$stats" $R/gpurun_out/prof_$tag/kernel_stats.csv
cd $R && python3 tools/step_kernels.py "$trace" $cfg gpurun_out/prof_$tag/step_kernels_$cfg.json 10 8 \
  > gpurun_out/prof_$tag/step_kernels.txt 2>&1
python3 tools/trace_timeline.py "$trace" k_embed_fwd 10 8 > gpurun_out/prof_$tag/timeline.txt 2>&1
rm -f "$trace"
echo done
