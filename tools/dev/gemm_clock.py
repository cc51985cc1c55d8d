"""Dev (round 6): the configs[2] GEMM (M = 65,536, N = K = 4096, int4 g128)
for an effective-clock pass (tools/dev/pmc_any.sh: GRBM_GUI_ACTIVE / 8 / duration per dispatch):
  python tools/dev/gemm_clock.py product   the product kernel (qlin_gemm_f16, 128 x 512 block)
  python tools/dev/gemm_clock.py nodq      the same block with its dequant VALU skipped (B = raw
                                           packed words: wrong values, the issue-only ceiling)
Runs >= 2 s of back-to-back launches first (clock settled), then 10 timed launches."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch  # noqa: E402

from quant import qlin  # noqa: E402

mode = sys.argv[1]
dev = torch.device("cuda:0")
M, N, K = 65536, 4096, 4096
w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
x = torch.randn(M, K, device=dev, dtype=torch.float16)
y = torch.empty(M, N, device=dev, dtype=torch.float16)
if mode == "product":
    run = lambda: qlin.gemm(x, o["qweight"], o["qsz"], None, N, K, 4, 128, o["flags"])  # noqa: E731
else:
    lab = ctypes.CDLL(os.path.join(ROOT, "tools/dev/libgemmlab.so"))
    P = ctypes.c_void_p

    def run():
        lab.lab_gemm_nodq(P(o["qweight"].data_ptr()), P(o["qsz"].data_ptr()), P(x.data_ptr()),
                          P(y.data_ptr()), ctypes.c_int64(M), N, K, 512, 1,
                          P(torch.cuda.current_stream().cuda_stream))
t0 = time.perf_counter()
while time.perf_counter() - t0 < 2.0:
    run()
    torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
e0.record()
for _ in range(10):
    run()
e1.record()
torch.cuda.synchronize()
t = e0.elapsed_time(e1) / 10 * 1e-3
print(f"{mode}: {t * 1e6:.1f} us per launch, {2 * M * N * K / t / 1e12:.0f} TFLOP/s", flush=True)
