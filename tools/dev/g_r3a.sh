set -u -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/dev/m1_order.py > gpurun_out/m1_order.log 2>&1 || { echo m1 failed $?; exit 1; }
cat gpurun_out/m1_order.log | grep -v amdgpu.ids
export TMPDIR=/tmp
R=$(pwd)
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pd -o run -- python $R/tools/bench_decode.py > $R/gpurun_out/pd.log 2>&1) || { echo prof failed; exit 1; }
find gpurun_out/pd -name "*kernel_stats.csv" -exec cut -c1-200 {} \; | head -30
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; echo pytest rc=$?; tail -8 gpurun_out/pytest_gpu.log
