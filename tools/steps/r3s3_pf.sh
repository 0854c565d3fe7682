#!/bin/bash
# round 3 session 3: L2-prefetch A/B (make pf PF=1,2,3): GEMM tests on the product and pf2 builds, then
# the C2 GEMM scan per build (same box, separate processes, base first and last)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
rm -f gpurun_out/r3s3_scan_all.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "gemm" -m gpu > gpurun_out/r3s3_base_tests.log 2>&1 || { tail -5 gpurun_out/r3s3_base_tests.log; exit 5; }
tail -1 gpurun_out/r3s3_base_tests.log
CHARPT_LIB=replicatinggpt_amd/libcharpt_hip_pf2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "gemm" -m gpu > gpurun_out/r3s3_pf2_tests.log 2>&1 || { tail -5 gpurun_out/r3s3_pf2_tests.log; exit 6; }
tail -1 gpurun_out/r3s3_pf2_tests.log
for v in ${PF_VARIANTS:-base pf1 pf2 pf3 base}; do
  if [ $v = base ]; then L=replicatinggpt_amd/libcharpt_hip.so; else L=replicatinggpt_amd/libcharpt_hip_$v.so; fi
  echo "== $v" >> gpurun_out/r3s3_scan_all.log
  CHARPT_LIB=$L timeout -k 10 200 python tools/gemm_scan2.py ${PF_CFG:-c2} 9 9 ${PF_SPLITS:-14,32} >> gpurun_out/r3s3_scan_all.log 2>&1 || exit 7
done
cat gpurun_out/r3s3_scan_all.log
