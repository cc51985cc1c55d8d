set -u -o pipefail
mkdir -p gpurun_out/r3
R=$(pwd); O=$R/gpurun_out/r3
export TMPDIR=/tmp
QLIN_PARITY_OUT=$O/r3_decode_parity.json timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decode.py -p no:cacheprovider -k decode_three_way > $O/t_dec.log 2>&1 || { echo dec parity failed; tail -5 $O/t_dec.log; exit 1; }
tail -1 $O/t_dec.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/kt.log 2>&1) || { echo kt failed; exit 1; }
tail -1 $O/kt.log | cut -c1-300
(cd /tmp && timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcd -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-other-mode --ramp-s 0 > $O/pmcd.log 2>&1) || { echo pmcd failed; exit 1; }
python tools/decode_traffic.py $O/pmcd $O/r3_decode_layer_int4_g128_pmc.json | cut -c1-300
(cd /tmp && timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcg -o run -- python $R/bench.py --workload gemm_int4_g128_m65536 --steps 2 --warmup 1 --no-cpu-baseline --ramp-s 0 > $O/pmcg.log 2>&1) || { echo pmcg failed; exit 1; }
python tools/pmc_traffic.py $O/pmcg gemm_kernel gemm_int4_g128_m65536 $O/r3_gemm_int4_g128_m65536_pmc.json | cut -c1-300
bash tools/dev/pmc_any.sh gemm65536 gemm_kernel bench.py --workload gemm_int4_g128_m65536 --steps 2 --warmup 1 --no-cpu-baseline --ramp-s 0 > $O/r3_gemm_m65536_sq_counters.txt 2>&1 || { echo sq failed; exit 1; }
cat $O/r3_gemm_m65536_sq_counters.txt
