#!/bin/bash
# PMC passes over the attention kernels alone (tools/attn_bench.py): one counter set per rocprofv3 run.
# usage: tools/pmc_attn.sh <tag> [attn_bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; tag=$1; shift
mkdir -p gpurun_out/pmca_$tag
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
            "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $R/gpurun_out/pmca_$tag/p$i -o run -- python3 $R/tools/attn_bench.py "$@" > $R/gpurun_out/pmca_$tag/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmca_$tag/p$i.log; exit 3; }
done
echo ok
