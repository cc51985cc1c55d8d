"""A/B: per-token activation fake-quant fused into the GEMV vs the quantizer kernel + GEMV (dev)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "../../llama3-quantization_amd"))
import torch
from quant import qlin
dev = torch.device("cuda:0")


def timed(fn, n, reps=20):
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
    return e0.elapsed_time(e1) * 1e3 / reps / n


for N, K in ((4096, 4096), (6144, 4096), (28672, 4096), (4096, 14336)):
    R = max(4, int(600e6 // (N * K // 2)) + 1)
    mats = []
    for i in range(R):
        o = qlin.quantize(torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02, 4, 128, 0,
                          want_xdq=False, want_params=False, pack=True)
        mats.append((o["qweight"], o["qsz"]))
    x = torch.randn(1, K, device=dev, dtype=torch.float16)
    plain = timed(lambda: [qlin.linear(x, m[0], m[1], None, N, K, 4, 128) for m in mats], R)
    fused = timed(lambda: [qlin.linear_ep(x, m[0], m[1], None, N, K, 4, 128, act_bits=8) for m in mats], R)
    two = timed(lambda: [qlin.linear(qlin.quantize(x, 8, K, 0, want_params=False)["x_dq"], m[0], m[1],
                                     None, N, K, 4, 128) for m in mats], R)
    print(f"N={N} K={K}: GEMV {plain:.2f} us | act-quant fused {fused:.2f} us | quantizer + GEMV {two:.2f} us", flush=True)
    del mats
    torch.cuda.empty_cache()
