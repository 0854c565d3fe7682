set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pair_train_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/step_ab.py c2 single,single:Fn.PAIR=0 5 50 > gpurun_out/pair_step_ab.txt 2>&1 || exit $?
bash tools/lib_ab.sh pairlib libcharpt_hip_base.so 3 > gpurun_out/pairlib_ab.txt 2>&1
