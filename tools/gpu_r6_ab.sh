set -o pipefail
timeout -k 10 200 python -u tools/pair_overlap_probe.py > gpurun_out/pair_probe.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/adamw_blk_ab.py c4 > gpurun_out/adamw_blk_c4.txt 2>&1 || exit $?
CHARPT_LIB=$PWD/replicatinggpt_amd/libcharpt_hip_ab.so timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -k "variants or ring or resident or 256" > gpurun_out/r6_ab_variant_tests.log 2>&1
