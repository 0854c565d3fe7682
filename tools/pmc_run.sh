#!/bin/bash
# PMC passes (the pmc_gemm.sh + pmc_gemm2.sh counter sets, one rocprofv3 run each) over any python
# workload: tools/pmc_run.sh <tag> <script.py> [args...]; results in gpurun_out/pmc_<tag>, pmc2_<tag>
# (tools/pmc_gemm_table.py reads them).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; tag=$1; shift
mkdir -p gpurun_out/pmc_$tag gpurun_out/pmc2_$tag
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_LDS" \
            "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d $R/gpurun_out/pmc_$tag/p$i -o run -- python3 "$R/$@" > $R/gpurun_out/pmc_$tag/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc_$tag/p$i.log; exit 3; }
done
i=0
for ctrs in "SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VALU_MFMA_COEXEC_CYCLES TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
            "SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d $R/gpurun_out/pmc2_$tag/p$i -o run -- python3 "$R/$@" > $R/gpurun_out/pmc2_$tag/p$i.log 2>&1 || { echo "pass2 $i failed"; tail -5 $R/gpurun_out/pmc2_$tag/p$i.log; exit 3; }
done
echo ok
