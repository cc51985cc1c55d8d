set -u -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
QLIN_LIBRARY=llama3-quantization_amd/csrc/libqlin_gfx950_trace.so timeout -k 10 200 python tools/dev/decode_trace.py > $O/trace.json 2>$O/trace.err || { echo trace failed; tail -5 $O/trace.err; exit 1; }
cat $O/trace.json
for cfg in "96 4096 4096 2 64" "64 4096 4096 3 64" "64 4096 4096 4 128"; do
  timeout -k 10 200 python tools/dev/batch_geo.py $cfg > $O/bgeo.log 2>&1 || { echo bgeo failed; tail -5 $O/bgeo.log; exit 1; }
  echo "== $cfg"; grep -v amdgpu $O/bgeo.log | tail -6
done
