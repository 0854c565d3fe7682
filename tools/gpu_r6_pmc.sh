#!/bin/bash
# Round 6 counter evidence: GEMM HBM traffic (C2, C4 census ops with the step's epilogues) and the
# attention kernels' PMC passes (C2, C4; p = 0.2).  Every rocprofv3 pass is its own run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
bash $R/tools/pmc_gemm_traffic.sh || exit $?
ATTN_CFG=c2 ATTN_P=0.2 bash $R/tools/pmc_attn.sh r6c2 || exit $?
ATTN_CFG=c4 ATTN_P=0.2 bash $R/tools/pmc_attn.sh r6c4 || exit $?
echo all-done
