"""GEMM block-width sweep (dev): 128 x 256 / 384 / 512 tiles (8 waves, int4 g128) on the LLaMA
projection shapes, against the product's own choice (pick_bn), plus an exactness check of the
384 tile against the product GEMM."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin
dev = torch.device("cuda:0")
lab = ctypes.CDLL(os.path.join(ROOT, "tools/dev/libgemmlab.so"))
P = ctypes.c_void_p
SHAPES = [tuple(map(int, t.split("x"))) for t in os.environ.get(
    "SHAPES", "4096x4096,6144x4096,14336x4096,28672x4096,4096x14336").split(",")]
MS = [int(m) for m in os.environ.get("MS", "2048,8192,65536").split(",")]


def timeit(fn, reps):
    fn(); torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    g.replay()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


for (N, K) in SHAPES:
    w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
    o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
    del w

    def run(abl, M, x, y):
        st = P(torch.cuda.current_stream().cuda_stream)
        return lab.lab_gemm(P(o["qweight"].data_ptr()), P(o["qsz"].data_ptr()), P(x.data_ptr()),
                            P(y.data_ptr()), ctypes.c_int64(M), N, K, abl, st)

    x = torch.randn(333, K, device=dev, dtype=torch.float16)
    ref = qlin.gemm(x, o["qweight"], o["qsz"], None, N, K, 4, 128)
    for v in (8, 12, 16, 32):
        y = torch.zeros_like(ref)
        assert run(v, 333, x, y) == 0
        torch.cuda.synchronize()
        d = (y.float() - ref.float()).abs().max().item()
        assert d == 0.0, (N, K, v, d)
    for M in MS:
        x = torch.randn(M, K, device=dev, dtype=torch.float16)
        y = torch.empty(M, N, device=dev, dtype=torch.float16)
        f = 2 * M * N * K
        reps = max(3, min(50, int(4e12 / f)))
        t = {name: timeit(lambda: run(v, M, x, y), reps) for name, v in
             (("64x128", 32), ("256", 8), ("384", 16), ("512", 12))}
        t["product"] = timeit(lambda: qlin.gemm(x, o["qweight"], o["qsz"], None, N, K, 4, 128), reps)
        print(f"N={N} K={K} M={M}: " + "  ".join(f"{k} {v*1e6:.1f} us ({f/v/1e12:.0f})" for k, v in t.items()),
              flush=True)
        del x, y
