"""GEMV geometry sweep (waves per block x prefetch depth x row tiles per block) per M on the
decode shapes, ring of distinct matrices beyond the MALL, HIP events over graph replays (dev)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin
dev = torch.device("cuda:0")
lib = ctypes.CDLL(os.path.join(ROOT, "tools/dev/libgeo.so"))
P = ctypes.c_void_p
SHAPES = [tuple(map(int, s.split("x"))) for s in os.environ.get("SHAPES", "4096x4096").split(",")]
MS = [int(m) for m in os.environ.get("MS", "1,8,16").split(",")]


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


for (N, K) in SHAPES:
    R = max(4, int(600e6 // (N * K // 2)) + 1)
    mats = []
    for i in range(R):
        w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
        o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
        mats.append((o["qweight"], o["qsz"]))
        del w
    nbytes = N * K // 2 + N * K // 128 * 4
    st = lambda: P(torch.cuda.current_stream().cuda_stream)
    for M in MS:
        x = torch.randn(M, K, device=dev, dtype=torch.float16)
        y = torch.empty(M, N, device=dev, dtype=torch.float16)
        ref = qlin.gemv(x, mats[0][0], mats[0][1], None, N, K, 4, 128)
        prod = timed(lambda: [qlin.gemv(x, m[0], m[1], None, N, K, 4, 128) for m in mats], R)
        print(f"N={N} K={K} M={M} ring={R}: product {prod:.2f} us ({nbytes / prod / 1e3:.0f} GB/s)", flush=True)
        for NTB in (1, 2):
            for W in (4, 8, 16):
                for PF in (2, 4):
                    if M > 1 and PF == 4 and M > 8:
                        continue
                    if -(-(K // 128) // W) < PF // 2:
                        continue
                    rc = lib.geo_gemv(P(mats[0][0].data_ptr()), P(mats[0][1].data_ptr()),
                                      P(x.data_ptr()), P(y.data_ptr()), M, N, K, W, PF, NTB, st())
                    assert rc == 0
                    torch.cuda.synchronize()
                    err = ((y.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
                    assert err < 2e-3, (M, NTB, W, PF, err)  # other split-K order than the product's
                    us = timed(lambda: [lib.geo_gemv(P(m[0].data_ptr()), P(m[1].data_ptr()), P(x.data_ptr()),
                                                     P(y.data_ptr()), M, N, K, W, PF, NTB, st()) for m in mats], R)
                    print(f"   NTB={NTB} W={W:2d} PF={PF}: {us:.2f} us ({nbytes / us / 1e3:.0f} GB/s)", flush=True)
        prod = timed(lambda: [qlin.gemv(x, m[0], m[1], None, N, K, 4, 128) for m in mats], R)
        print(f"   product again: {prod:.2f} us ({nbytes / prod / 1e3:.0f} GB/s)", flush=True)
    del mats
    torch.cuda.empty_cache()
