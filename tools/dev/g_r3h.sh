set -u -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_epilogue.py tests/test_gpu_attn.py tests/test_gpu_decode_engine.py tests/test_gpu_model.py tests/test_host.py -p no:cacheprovider > $O/t_h.log 2>&1; rc=$?; echo rc=$rc; tail -5 $O/t_h.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-other-mode > $O/bh.log 2>&1 || { echo bench failed; tail -3 $O/bh.log; exit 1; }; grep -o '"us_per_layer": [0-9.]*' $O/bh.log; done
QLIN_PARITY_OUT=$O/r3_decode_parity_h.json timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decode.py -p no:cacheprovider -k decode_three_way > $O/t_dh.log 2>&1; echo rc=$?; tail -2 $O/t_dh.log
