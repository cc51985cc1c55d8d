"""Dev sweep: qlin_gemv_batched_f16 geometry (waves per block) on the bench's ring.

Loads the product library (ring setup, reference output) and each tools/dev/libgs<P>_<PF>.so variant
(GEMV_STREAM_PERSIST / GEMV_STREAM_PF) through ctypes, times one strided-batch launch over a ring of R 4096^2 int4
g128 matrices (graph-replayed, HIP events), checks every variant bit-identical to the product.
Usage: python tools/dev/batch_geo.py [R] [N] [K] [bits] [group]
"""
import ctypes
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llama3-quantization_amd")]
import torch  # noqa: E402
from quant import qlin  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 64
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
K = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
bits = int(sys.argv[4]) if len(sys.argv) > 4 else 4
group = int(sys.argv[5]) if len(sys.argv) > 5 else 128
M = 1
dev = torch.device("cuda", 0)
lib = qlin.load_library()
qw = torch.zeros((R, *qlin.packed_shape(N, K, bits)), dtype=torch.int32, device=dev)
sz = torch.zeros((R, *qlin.sz_shape(N, K, group)), dtype=torch.int32, device=dev)
g = torch.Generator(device=dev)
for i in range(R):
    g.manual_seed(i)
    w = torch.empty(N, K, device=dev, dtype=torch.float16).normal_(0, 0.02, generator=g)
    o = qlin.quantize(w, bits, group, 0, want_xdq=False, want_params=False, pack=True)
    qw[i].copy_(o["qweight"])
    sz[i].copy_(o["qsz"])
xs = torch.randn(R, M, K, device=dev, dtype=torch.float16, generator=g)
ref = torch.empty(R, M, N, device=dev, dtype=torch.float16)
nbytes = R * (N * K * bits // 8 + N * (K // group) * 3 + 2 * M * K + 2 * M * N)

libs = [("product", lib)]
for p in sorted(glob.glob(os.path.join(ROOT, "tools", "dev", "libgs*.so"))):
    L = ctypes.CDLL(p)
    L.qlin_gemv_batched_f16.argtypes = qlin.SIGNATURES["qlin_gemv_batched_f16"][0]
    L.qlin_gemv_batched_f16.restype = ctypes.c_int
    libs.append((os.path.basename(p), L))


def call(L, y, st):
    return L.qlin_gemv_batched_f16(qw.data_ptr(), qw[0].numel(), sz.data_ptr(), sz[0].numel(), 0,
                                   xs.data_ptr(), M * K, None, 0, y.data_ptr(), M * N, R, M, N,
                                   K, bits, group, st)


assert call(lib, ref, torch.cuda.current_stream().cuda_stream) == 0
torch.cuda.synchronize()
for rep in range(3):
    for name, L in libs:
        y = torch.zeros_like(ref)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            assert call(L, y, s.cuda_stream) == 0
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        same = torch.equal(y.view(torch.int16), ref.view(torch.int16))
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            call(L, y, torch.cuda.current_stream().cuda_stream)
        for _ in range(5):
            gr.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        steps = 50
        torch.cuda.synchronize()
        e0.record()
        for _ in range(steps):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / steps
        print(f"{name:14s} R={R} {N}x{K} b{bits} g{group}: {us:8.2f} us/launch  {us / R:6.3f} us/matrix  "
              f"{nbytes / us / 1e3:7.1f} GB/s  {nbytes / us / 1e3 / 8000:.3f}  bit-identical={same}",
              flush=True)
