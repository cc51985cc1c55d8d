"""Dev: old (gemv_kernel, contiguous tiles per wave) vs decode fast path (gemv_fast_kernel,
strided tiles) per geometry on the decode shapes, M = 1, ring beyond the MALL, same box."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin
dev = torch.device("cuda:0")
lib = ctypes.CDLL(os.path.join(ROOT, "tools/dev/libgeo.so"))
P = ctypes.c_void_p
SHAPES = [tuple(map(int, s.split("x"))) for s in
          os.environ.get("SHAPES", "4096x4096,6144x4096,28672x4096,4096x14336").split(",")]


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
for (N, K) in SHAPES:
    R = max(4, int(600e6 // (N * K // 2)) + 1)
    mats = []
    for i in range(R):
        w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
        o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
        mats.append((o["qweight"], o["qsz"]))
        del w
    x = torch.randn(1, K, device=dev, dtype=torch.float16)
    y = torch.empty(1, N, device=dev, dtype=torch.float16)
    ref = qlin.gemv(x, mats[0][0], mats[0][1], None, N, K, 4, 128).float()
    Kt = K // 128
    prod = timed(lambda: [qlin.gemv(x, m[0], m[1], None, N, K, 4, 128) for m in mats], R)
    print(f"{N}x{K} ring={R}: product {prod:.2f} us", flush=True)
    res = []
    for W in (4, 8, 16):
        for PF in (2, 4, 8):
            if -(-Kt // W) < PF // 2:
                continue
            if PF == 8:
                if -(-Kt // W) > 8:
                    continue
                rc = lib.geo_fast(P(mats[0][0].data_ptr()), P(mats[0][1].data_ptr()), P(x.data_ptr()),
                                  P(y.data_ptr()), N, K, W, 8, 0, st())
                assert rc == 0
                torch.cuda.synchronize()
                assert ((y.float() - ref).abs().max() / ref.abs().max()).item() < 2e-3
                us = timed(lambda: [lib.geo_fast(P(m[0].data_ptr()), P(m[1].data_ptr()), P(x.data_ptr()),
                                                 P(y.data_ptr()), N, K, W, 8, 0, st()) for m in mats], R)
                res.append((us, f"fast W={W:2d} PF=8 LOOP=0"))
                continue
            lib.geo_gemv(P(mats[0][0].data_ptr()), P(mats[0][1].data_ptr()), P(x.data_ptr()),
                         P(y.data_ptr()), 1, N, K, W, PF, 1, st())
            torch.cuda.synchronize()
            assert ((y.float() - ref).abs().max() / ref.abs().max()).item() < 2e-3
            us = timed(lambda: [lib.geo_gemv(P(m[0].data_ptr()), P(m[1].data_ptr()), P(x.data_ptr()),
                                             P(y.data_ptr()), 1, N, K, W, PF, 1, st()) for m in mats], R)
            res.append((us, f"old  W={W:2d} PF={PF}"))
            for LOOP in (0, 1):
                if -(-Kt // W) > PF and not LOOP:
                    continue
                rc = lib.geo_fast(P(mats[0][0].data_ptr()), P(mats[0][1].data_ptr()), P(x.data_ptr()),
                                  P(y.data_ptr()), N, K, W, PF, LOOP, st())
                assert rc == 0
                torch.cuda.synchronize()
                assert ((y.float() - ref).abs().max() / ref.abs().max()).item() < 2e-3
                us = timed(lambda: [lib.geo_fast(P(m[0].data_ptr()), P(m[1].data_ptr()), P(x.data_ptr()),
                                                 P(y.data_ptr()), N, K, W, PF, LOOP, st()) for m in mats], R)
                res.append((us, f"fast W={W:2d} PF={PF} LOOP={LOOP}"))
    for us, nm in sorted(res):
        print(f"   {nm}: {us:.2f} us", flush=True)
    del mats
    torch.cuda.empty_cache()
