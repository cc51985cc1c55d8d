"""Dev: ablations of the batched streaming GEMV (tools/dev/stream_lab.hip -> libslab.so) on the
bench's ring (graph-replayed, HIP events, best of 3 reps), against the product launch.
Usage: python tools/dev/stream_lab.py R bits group [abl:wpe ...]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llama3-quantization_amd")]
import torch  # noqa: E402
from quant import qlin  # noqa: E402

R, bits, group = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
variants = [tuple(int(t) for t in v.split(":")) for v in sys.argv[4:]] or [(0, 0)]
N = K = 4096
dev = torch.device("cuda", 0)
lib = qlin.load_library()
lab = ctypes.CDLL(os.path.join(ROOT, "tools/dev/libslab.so"))
P = ctypes.c_void_p
lab.lab_stream.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, P, ctypes.c_int64, ctypes.c_int64,
                           ctypes.c_int64, ctypes.c_int, ctypes.c_int, P]
qw = torch.zeros((R, *qlin.packed_shape(N, K, bits)), dtype=torch.int32, device=dev)
sz = torch.zeros((R, *qlin.sz_shape(N, K, group)), dtype=torch.int32, device=dev)
g = torch.Generator(device=dev)
for i in range(R):
    g.manual_seed(i)
    w = torch.empty(N, K, device=dev, dtype=torch.float16).normal_(0, 0.02, generator=g)
    o = qlin.quantize(w, bits, group, 0, want_xdq=False, want_params=False, pack=True)
    qw[i].copy_(o["qweight"])
    sz[i].copy_(o["qsz"])
xs = torch.randn(R, 1, K, device=dev, dtype=torch.float16, generator=g)
ref = torch.empty(R, 1, N, device=dev, dtype=torch.float16)
nbytes = R * (N * K * bits // 8 + N * (K // group) * 3 + 2 * K + 2 * N)


def prod(y, st):
    return lib.qlin_gemv_batched_f16(qw.data_ptr(), qw[0].numel(), sz.data_ptr(), sz[0].numel(), 0,
                                     xs.data_ptr(), K, None, 0, y.data_ptr(), N, R, 1, N, K, bits,
                                     group, st)


def labv(abl, wpe):
    def f(y, st):
        rc = lab.lab_stream(abl, wpe, P(qw.data_ptr()), P(sz.data_ptr()), P(xs.data_ptr()),
                            P(y.data_ptr()), R, N, K, bits, group, P(st))
        return 0 if rc > 0 else rc
    return f


assert prod(ref, torch.cuda.current_stream().cuda_stream) == 0
torch.cuda.synchronize()
runs = [("product", prod)] + [(f"abl{a}:wpe{w}", labv(a, w)) for a, w in variants]
best = {}
for rep in range(3):
    for name, fn in runs:
        y = torch.zeros_like(ref)
        assert fn(y, torch.cuda.current_stream().cuda_stream) == 0, name
        torch.cuda.synchronize()
        same = torch.equal(y.view(torch.int16), ref.view(torch.int16))
        gr = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.graph(gr, stream=s):
            fn(y, s.cuda_stream)
        torch.cuda.current_stream().wait_stream(s)
        for _ in range(5):
            gr.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(50):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 50
        best[name] = min(best.get(name, (1e9,))[0], us), same
for name, _ in runs:
    us, same = best[name]
    print(f"{name:14s} R={R} b{bits} g{group}: {us:8.2f} us  {nbytes / us / 1e3:7.1f} GB/s "
          f"{nbytes / us / 1e3 / 8000:.3f}  bit-identical={same}", flush=True)
