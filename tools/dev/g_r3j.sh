set -u -o pipefail
mkdir -p gpurun_out/r3j
R=$(pwd); O=$R/gpurun_out/r3j
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
QLIN_PARITY_OUT=$O/r3_decode_parity.json timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decode.py -p no:cacheprovider -k decode_three_way > $O/t_dec.log 2>&1 || { echo parity failed; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -3 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-600
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/kt.log 2>&1) || { echo kt failed; exit 1; }
(cd /tmp && timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcd -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-other-mode --ramp-s 0 > $O/pmcd.log 2>&1) || { echo pmcd failed; exit 1; }
python tools/decode_traffic.py $O/pmcd $O/r3_decode_layer_int4_g128_pmc.json | cut -c1-200
timeout -k 10 300 python tools/bench_decode.py > $O/bd.log 2>&1 || { echo bd failed; exit 1; }
tail -1 $O/bd.log
