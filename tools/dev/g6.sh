set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_attn.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_attn.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dev/attn_prefill_bench.py > gpurun_out/apb.txt 2>&1 || exit $?
S=512 timeout -k 10 300 python -u tools/dev/attn_prefill_bench.py >> gpurun_out/apb.txt 2>&1 || exit $?
cat gpurun_out/apb.txt
