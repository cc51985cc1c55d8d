set -u -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
NCFG=3 timeout -k 10 300 python tools/dev/attn_ab.py libattn_old.so libattn_v3.so libattn_v3t512.so libattn_v3t256.so > $O/attn_ab2.log 2>&1 || { echo attn failed; tail -3 $O/attn_ab2.log; exit 1; }
grep -v amdgpu $O/attn_ab2.log
for lib in llama3-quantization_amd/csrc/libqlin_gfx950.so tools/dev/libnrm_ab.so llama3-quantization_amd/csrc/libqlin_gfx950.so tools/dev/libnrm_ab.so; do
  QLIN_LIBRARY=$lib timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-other-mode > $O/bnrm.log 2>&1 || { echo bench failed; tail -3 $O/bnrm.log; exit 1; }
  echo $lib $(grep -o '"us_per_layer": [0-9.]*' $O/bnrm.log)
done
bash tools/dev/pmc_any.sh ap attn_prefill tools/dev/attn_prefill_bench.py > $O/r3_attn_prefill_sq.txt 2>&1 || { echo pmc failed; exit 1; }
cat $O/r3_attn_prefill_sq.txt
