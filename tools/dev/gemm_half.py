"""Dev: 64-row GEMM blocks (two per CU at width 256) vs the product's choice at M = 2048 shapes."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin
dev = torch.device("cuda:0")
lab = ctypes.CDLL(os.path.join(ROOT, "tools/dev/libgemmlab.so"))
P = ctypes.c_void_p
SHAPES = [tuple(map(int, t.split("x"))) for t in os.environ.get(
    "SHAPES", "4096x4096,4096x14336,6144x4096,28672x4096").split(",")]
MS = [int(m) for m in os.environ.get("MS", "1024,2048,4096").split(",")]


def timeit(fn, reps):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


for (N, K) in SHAPES:
    w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
    o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
    del w
    for M in MS:
        x = torch.randn(M, K, device=dev, dtype=torch.float16)
        y = torch.empty(M, N, device=dev, dtype=torch.float16)
        prod = lambda: qlin.gemm(x, o["qweight"], o["qsz"], None, N, K, 4, 128, o["flags"])
        def half(bn):
            st = P(torch.cuda.current_stream().cuda_stream)
            assert lab.lab_gemm_half(P(o["qweight"].data_ptr()), P(o["qsz"].data_ptr()),
                                     P(x.data_ptr()), P(y.data_ptr()), ctypes.c_int64(M), N, K,
                                     bn, st) == 0
        ref = prod()
        half(256); torch.cuda.synchronize()
        same = bool(torch.equal(y, ref))
        f = 2 * M * N * K
        reps = max(3, int(2e9 / f * 20))
        best = [1e9, 1e9]
        for _ in range(3):
            best[0] = min(best[0], timeit(prod, reps))
            best[1] = min(best[1], timeit(lambda: half(256), reps))
        bn = qlin.load_library().qlin_gemm_block_cols(M, N, 4)
        print(f"N={N} K={K} M={M}: product (bn {bn}) {f/best[0]/1e12:6.0f} TF/s ({best[0]*1e6:7.1f} us) | "
              f"64x256 {f/best[1]/1e12:6.0f} ({best[1]*1e6:7.1f} us) bit-identical {same}", flush=True)
