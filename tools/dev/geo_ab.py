"""Dev: same-box A/B of two builds of gemv_kernel (libgeo.so vs libgeo_old.so), product geometry."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin
dev = torch.device("cuda:0")
libs = {n: ctypes.CDLL(os.path.join(ROOT, f"tools/dev/{n}.so")) for n in ("libgeoprev", "libgeo")}
P = ctypes.c_void_p


def timed(fn, n, reps=10):
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps / n


st = lambda: P(torch.cuda.current_stream().cuda_stream)
for (N, K, M, W, PF, NTB) in ((4096, 4096, 8, 16, 2, 1), (4096, 4096, 16, 16, 2, 1),
                              (14336, 4096, 8, 8, 2, 2), (14336, 4096, 16, 8, 2, 2),
                              (4096, 14336, 1, 16, 2, 1)):
    R = max(4, int(600e6 // (N * K // 2)) + 1)
    mats = []
    for i in range(R):
        w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
        o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
        mats.append((o["qweight"], o["qsz"]))
        del w
    x = torch.randn(M, K, device=dev, dtype=torch.float16)
    y = torch.empty(M, N, device=dev, dtype=torch.float16)
    line = f"{N}x{K} M={M} W={W} PF={PF} NTB={NTB}:"
    for rep in range(2):
        for name, lib in libs.items():
            us = timed(lambda: [lib.geo_gemv(P(m[0].data_ptr()), P(m[1].data_ptr()), P(x.data_ptr()),
                                             P(y.data_ptr()), M, N, K, W, PF, NTB, st()) for m in mats], R)
            line += f" {'old' if name == 'libgeoprev' else 'new'} {us:.2f}"
    print(line, flush=True)
    del mats
    torch.cuda.empty_cache()
