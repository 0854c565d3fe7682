#!/bin/bash
# generate 256 x 500 with the fused FFN's LayerNorm in its launch / in its own launch / FFN unfused, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ffn_ln_ab.txt
for r in 1 2 3; do
  for cfg in "1 1" "1 0" "0 1"; do
    set -- $cfg
    CHARPT_FFN_FUSED=$1 CHARPT_FFN_LN=$2 timeout -k 10 120 python -u tools/f32_fwd_ab.py gen 0 2>&1 | grep -v amdgpu | sed "s/^/fused=$1 ln=$2 /" >> gpurun_out/ffn_ln_ab.txt || exit 1
  done
done
echo ok
