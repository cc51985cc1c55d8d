"""Dev: product GEMV per-launch time over a ring of distinct matrices (HIP events over graph
replays) for the decode shapes, with an accuracy check against dequant + F.linear; optional
lab3 V0 reference kernel (LAB3=1)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin

dev = torch.device("cuda:0")
SHAPES = [tuple(map(int, s.split("x"))) for s in
          os.environ.get("SHAPES", "4096x4096,6144x4096,28672x4096,4096x14336").split(",")]
MS = [int(m) for m in os.environ.get("MS", "1").split(",")]
P = ctypes.c_void_p


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


lab = ctypes.CDLL(os.path.join(ROOT, "tools/dev/liblab3.so")) if os.environ.get("LAB3") else None
for (N, K) in SHAPES:
    R = max(4, int(600e6 // (N * K // 2)) + 1)
    mats = []
    for i in range(R):
        w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
        o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
        mats.append((o["qweight"], o["qsz"]))
        del w
    nbytes = N * K // 2 + N * K // 128 * 3 + 2 * K + 2 * N
    for M in MS:
        x = torch.randn(M, K, device=dev, dtype=torch.float16)
        wdq = qlin.dequant(mats[0][0], mats[0][1], N, K, 4, 128)
        ref = torch.nn.functional.linear(x.float(), wdq.float())
        y = qlin.gemv(x, mats[0][0], mats[0][1], None, N, K, 4, 128)
        err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
        us = timed(lambda: [qlin.gemv(x, m[0], m[1], None, N, K, 4, 128) for m in mats], R)
        line = f"{N}x{K} M={M} ring={R}: product {us:.3f} us ({nbytes / us / 1e3:.0f} GB/s, err {err:.2e})"
        if lab is not None and (N, K, M) == (4096, 4096, 1):
            ys = torch.empty(1, N, device=dev, dtype=torch.float16)
            st = lambda: P(torch.cuda.current_stream().cuda_stream)
            lu = timed(lambda: [lab.lab3_launch(P(m[0].data_ptr()), P(m[1].data_ptr()), P(x.data_ptr()),
                                                P(ys.data_ptr()), N, K, 0, st()) for m in mats], R)
            line += f"; lab3 V0 {lu:.3f} us"
        print(line, flush=True)
    del mats
    torch.cuda.empty_cache()
