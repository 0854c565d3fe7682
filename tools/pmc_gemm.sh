#!/bin/bash
# PMC passes over one GEMM shape/variant: tools/pmc_gemm.sh <tag> M N K at bt variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; tag=$1; shift
mkdir -p gpurun_out/pmc_$tag
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_LDS" \
            "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $ctrs --output-format csv -d $R/gpurun_out/pmc_$tag/p$i -o run -- python3 $R/tools/gemm_one.py "$@" > $R/gpurun_out/pmc_$tag/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $R/gpurun_out/pmc_$tag/p$i.log; exit 3; }
done
echo ok
