set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_epilogue.py tests/test_gpu_layers.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_k.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_k.log; [ $rc -eq 0 ] || exit $rc
MS=1,8,16 SHAPES=4096x4096,14336x4096 timeout -k 10 300 python -u tools/dev/gemv_quick.py > gpurun_out/gq8.txt 2>&1 || exit $?
cat gpurun_out/gq8.txt
