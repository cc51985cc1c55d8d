set -u -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
run() { timeout -k 10 200 env "$@" python bench.py --steps 20 --no-cpu-baseline --no-other-mode > $O/bi.log 2>&1 || { echo bench failed; tail -3 $O/bi.log; exit 1; }; echo "$@" $(grep -o '"us_per_layer": [0-9.]*' $O/bi.log); }
for r in 1 2; do
  run QLIN_X=0
  run QLIN_DEV_NO_SUMSQ=1
  run QLIN_DEV_NO_ROPE_GATHER=1
  run QLIN_DEV_NO_SUMSQ=1 QLIN_DEV_NO_ROPE_GATHER=1
done
for r in 1 2; do
  run QLIN_LIBRARY=tools/dev/libnrm_late.so
  run QLIN_LIBRARY=tools/dev/libnrm_late.so QLIN_DEV_NO_SUMSQ=1
done
QLIN_LIBRARY=tools/dev/libnrm_late.so timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_epilogue.py -p no:cacheprovider -k rmsnorm > $O/t_late.log 2>&1; echo late-tests rc=$?; tail -3 $O/t_late.log
QLIN_LIBRARY=tools/dev/libnrm_late.so QLIN_PARITY_OUT=$O/r3_decode_parity_late.json timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decode.py -p no:cacheprovider -k decode_three_way > $O/t_dl.log 2>&1; echo rc=$?; tail -2 $O/t_dl.log
