#!/bin/bash
# C4 bench with the library of commit ad1f3f9 (the round's first C4 line) and the current one, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/c4_ab.txt
for r in 1 2; do for l in c4old cur; do
  if [ $l = cur ]; then unset CHARPT_LIB; else export CHARPT_LIB=$PWD/replicatinggpt_amd/libcharpt_hip_$l.so; fi
  timeout -k 10 300 python bench.py --config c4 --steps 50 --warmup 10 --no-cpu-baseline --no-generate 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lib=$l', d['ms_per_step'], 'ms/step')" >> gpurun_out/c4_ab.txt || exit 1
done; done
echo ok
