"""Dev: split-K (small grids) vs unsplit GEMM timings at prefill-sized M."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin
dev = torch.device("cuda:0")


def timeit(fn, reps=50):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


lib = qlin.load_library()
for (N, K) in [(4096, 4096), (6144, 4096), (4096, 14336), (1024, 4096), (28672, 4096)]:
    w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
    o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
    del w
    for M in (65, 128, 192, 256, 384, 512):
        x = torch.randn(M, K, device=dev, dtype=torch.float16)
        ws = lib.qlin_linear_workspace_bytes(M, N, K, 4, 128, 0)
        t0 = min(timeit(lambda: qlin.gemm(x, o["qweight"], o["qsz"], None, N, K, 4, 128, o["flags"], split=False)) for _ in range(3))
        t1 = min(timeit(lambda: qlin.gemm(x, o["qweight"], o["qsz"], None, N, K, 4, 128, o["flags"])) for _ in range(3))
        print(f"N={N} K={K} M={M}: unsplit {t0*1e6:6.1f} us | split (ws {ws >> 10} KB) {t1*1e6:6.1f} us  x{t0/t1:.2f}", flush=True)
