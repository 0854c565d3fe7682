#!/bin/bash
# Issue / memory-pipe PMC passes over one GEMM shape/variant (tools/gemm_one.py): where the 128x128
# persistent kernel's non-MFMA cycles go.  usage: tools/pmc_gemm2.sh <tag> M N K at bt variant [reps] [split]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; tag=$1; shift
mkdir -p gpurun_out/pmc2_$tag
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VALU_MFMA_COEXEC_CYCLES TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
            "SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $ctrs --output-format csv -d $R/gpurun_out/pmc2_$tag/p$i -o run -- python3 $R/tools/gemm_one.py "$@" > $R/gpurun_out/pmc2_$tag/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $R/gpurun_out/pmc2_$tag/p$i.log; exit 3; }
done
echo ok
