"""Dev: one decode GEMV launch (M = 1, int4 g128, no epilogue) on the decode layer's shapes, the
product route (qlin_linear_ep_f16) against the batched streaming kernel with one problem
(qlin_gemv_batched_f16, B = 1), each as a HIP graph of dependent launches over a ring of distinct
matrices (> 700 MB per shape, beyond the MALL).  Prints us per launch and GB/s."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch  # noqa: E402
from quant import qlin  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = [("gateup", 28672, 4096), ("down", 4096, 14336), ("qkv", 6144, 4096), ("o", 4096, 4096)]
for name, N, K in SHAPES:
    ring = max(8, -(-700_000_000 // (N * K // 2)))
    mats = []
    for i in range(ring):
        w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
        o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
        mats.append((o["qweight"], o["qsz"]))
        del w
    x = torch.randn(1, K, device=dev, dtype=torch.float16)
    y = torch.empty(1, N, device=dev, dtype=torch.float16)
    yb = torch.empty(1, 1, N, device=dev, dtype=torch.float16)

    def prod():
        for qw, qsz in mats:
            qlin.linear_ep(x, qw, qsz, None, N, K, 4, 128)

    def batched():
        for qw, qsz in mats:
            qlin.gemv_batched(x, qw[None], qsz[None], None, N, K, 4, 128, out=yb)

    res = {}
    for nm, fn in (("product", prod), ("batched1", batched)):
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        for _ in range(10):
            g.replay()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(5):
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            for _ in range(5):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e3 / (5 * ring))
        res[nm] = round(best, 2)
        del g
    gb = N * K / 2 * (1 + 3 / 64) / 1e3
    print(f"{name} N={N} K={K}: us/launch {res}  GB/s { {k: round(gb / v) for k, v in res.items()} }",
          flush=True)
    del mats
    torch.cuda.empty_cache()
