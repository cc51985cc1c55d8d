"""GEMM ablation timings: full / no compute / no DMA / neither (int4 g128, N = K = 4096)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin
dev = torch.device("cuda:0")
lab = ctypes.CDLL(os.path.join(ROOT, "tools/dev/libgemmlab.so"))
P = ctypes.c_void_p
N = K = 4096
w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)


def timeit(fn, reps):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


for M, wide in ((2048, 0), (2048, 4), (16384, 0), (16384, 4)):
    x = torch.randn(M, K, device=dev, dtype=torch.float16)
    y = torch.empty(M, N, device=dev, dtype=torch.float16)
    st = P(torch.cuda.current_stream().cuda_stream)
    res = []
    for abl in (0 | wide, 1 | wide, 2 | wide, 3 | wide):
        t = timeit(lambda: lab.lab_gemm(P(o["qweight"].data_ptr()), P(o["qsz"].data_ptr()),
                                        P(x.data_ptr()), P(y.data_ptr()), ctypes.c_int64(M), N, K,
                                        abl, st), 10)
        res.append(t)
    f = 2 * M * N * K
    print(f"M={M} {'wide' if wide else 'narrow'}: full {res[0]*1e6:.1f} us ({f/res[0]/1e12:.0f} TF/s) | no-compute {res[1]*1e6:.1f} | "
          f"no-DMA {res[2]*1e6:.1f} ({f/res[2]/1e12:.0f} TF/s) | neither {res[3]*1e6:.1f}", flush=True)
