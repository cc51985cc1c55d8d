set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider ${PYT:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -25 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
for c in ${EXTRA:-"python tools/bench_decode.py"}; do :; done
timeout -k 10 400 ${EXTRA:-python tools/bench_decode.py} > gpurun_out/extra.json 2>gpurun_out/extra.err || exit 3
cat gpurun_out/extra.json
