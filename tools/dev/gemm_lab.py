"""GEMM ablation timings: full / no compute / no DMA / neither (int4 g128, N = K = 4096), for the
4- and 8-wave blocks, plus a correctness check of every variant against the product GEMM."""
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


def run(abl, M, x, y):
    st = P(torch.cuda.current_stream().cuda_stream)
    return lab.lab_gemm(P(o["qweight"].data_ptr()), P(o["qsz"].data_ptr()), P(x.data_ptr()),
                        P(y.data_ptr()), ctypes.c_int64(M), N, K, abl, st)


x = torch.randn(512, K, device=dev, dtype=torch.float16)
ref = qlin.gemm(x, o["qweight"], o["qsz"], None, N, K, 4, 128)
for v in (0, 4, 8, 12):
    y = torch.zeros_like(ref)
    assert run(v, 512, x, y) == 0
    torch.cuda.synchronize()
    print(f"variant {v}: max |y - product| = {(y.float() - ref.float()).abs().max().item():.3g}", flush=True)

for M in (2048, 16384, 65536):
    x = torch.randn(M, K, device=dev, dtype=torch.float16)
    y = torch.empty(M, N, device=dev, dtype=torch.float16)
    f = 2 * M * N * K
    for var in (4, 12, 0, 8):
        res = [timeit(lambda: run(a | var, M, x, y), 10) for a in (0, 1, 2, 3)]
        name = f"{'wide' if var & 4 else 'narrow'} {8 if var & 8 else 4}w"
        print(f"M={M} {name}: full {res[0]*1e6:.1f} us ({f/res[0]/1e12:.0f} TF/s) | no-compute {res[1]*1e6:.1f} | "
              f"no-DMA {res[2]*1e6:.1f} ({f/res[2]/1e12:.0f} TF/s) | neither {res[3]*1e6:.1f}", flush=True)
