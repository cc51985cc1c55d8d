set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for w in ${WL:-gemm_int4_g128_m2048 gemm_int4_g64_hqq_m2048 gemm_int4_g128_m65536}; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_$w.json 2>gpurun_out/bench_$w.err || exit 3
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_$w.json')); print('$w', d['value'], d['roofline']['us_per_launch'], d['roofline']['frac'])"
done
