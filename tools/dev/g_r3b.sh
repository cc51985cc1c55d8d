set -u -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/dev/flinear_order.py > gpurun_out/forder.log 2>&1 || { echo forder failed $?; exit 1; }
grep -v amdgpu.ids gpurun_out/forder.log
QLIN_LIBRARY=llama3-quantization_amd/csrc/libqlin_gfx950_so.so timeout -k 10 300 python tools/bench_decode.py > gpurun_out/bd_so.log 2>&1 || { echo bd_so failed $?; exit 1; }
grep -v amdgpu.ids gpurun_out/bd_so.log
