set -u -o pipefail
for rep in 1 2; do
 for lib in head new; do
  for w in ${AB_WORKLOADS:-gemm_int4_g128_m65536 gemm_int4_g128_m2048}; do
   if [ $lib = head ]; then export QLIN_LIBRARY=$PWD/tools/dev/libqlin_head.so; else unset QLIN_LIBRARY; fi
   timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > gpurun_out/ab_$lib.$w.$rep.json 2>/dev/null || exit $?
   python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],sys.argv[3],sys.argv[4],d['value'])" gpurun_out/ab_$lib.$w.$rep.json $lib $w $rep
  done
 done
done
