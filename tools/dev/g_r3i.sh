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
