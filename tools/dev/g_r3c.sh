set -u -o pipefail
mkdir -p gpurun_out
for v in pf8 pf4; do
  QLIN_LIBRARY=llama3-quantization_amd/csrc/libqlin_gfx950_$v.so timeout -k 10 300 python tools/bench_decode.py --reps 10 > gpurun_out/bd_$v.log 2>&1 || { echo bd $v failed $?; exit 1; }
  echo $v; grep -o '"engine_us[^,]*' gpurun_out/bd_$v.log; grep -o '"packed_fused_kv_cache_us[^,]*' gpurun_out/bd_$v.log
done
QLIN_PARITY_OUT=gpurun_out/r3_decode_parity.json timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decode.py -p no:cacheprovider -k decode > gpurun_out/t_dec.log 2>&1; echo rc=$?; tail -3 gpurun_out/t_dec.log
QLIN_PARITY_OUT=gpurun_out/r3_prefill_parity.json timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decode.py -p no:cacheprovider -k prefill > gpurun_out/t_pre.log 2>&1; echo rc=$?; tail -3 gpurun_out/t_pre.log
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed $?; tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
