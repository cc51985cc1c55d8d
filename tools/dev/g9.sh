set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_layers.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_m.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_m.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/ppl_llama3_8b.py > gpurun_out/ppl9.json 2> gpurun_out/ppl9.err || exit $?
cat gpurun_out/ppl9.json
