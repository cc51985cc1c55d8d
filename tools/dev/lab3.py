"""Dev: GEMV compute vs weight stream variants (tools/dev/gemv_lab3.hip), int4 g128 4096^2, M = 1,
ring of 64 matrices, HIP events over graph replays; stamp timelines of selected variants."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin

dev = torch.device("cuda:0")
lab = ctypes.CDLL(os.path.join(ROOT, "tools/dev/liblab3.so"))
R, N, K = 64, 4096, 4096
mats = []
for i in range(R):
    w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
    o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
    mats.append((o["qweight"], o["qsz"]))
x = torch.randn(1, K, device=dev, dtype=torch.float16)
ys = [torch.empty(1, N, device=dev, dtype=torch.float16) for _ in range(8)]
P = ctypes.c_void_p
st = lambda: P(torch.cuda.current_stream().cuda_stream)


def launch(m, y, V):
    rc = lab.lab3_launch(P(m[0].data_ptr()), P(m[1].data_ptr()), P(x.data_ptr()), P(y.data_ptr()),
                         N, K, V, st())
    assert rc == 0


def timed(fn, reps=20):
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps / R


ref = qlin.gemv(x, mats[0][0], mats[0][1], None, N, K, 4, 128)
for V in (0, 13):
    y = torch.empty(1, N, device=dev, dtype=torch.float16)
    launch(mats[0], y, V)
    torch.cuda.synchronize()
    d = (y.float() - ref.float()).abs().max().item() / ref.float().abs().max().item()
    print(f"check V={V}: max |lab - product| / max|y| = {d:.3g}", flush=True)
for rep in range(2):
    prod = timed(lambda: [qlin.gemv(x, m[0], m[1], None, N, K, 4, 128) for m in mats])
    print(f"product: {prod:.3f} us", flush=True)
    for V in (0, 13):
        us = timed(lambda: [launch(m, ys[j % 8], V) for j, m in enumerate(mats)])
        print(f"V={V}: {us:.3f} us", flush=True)
