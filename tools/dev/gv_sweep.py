"""Dev: decode GEMV shapes (M = 1) under GEMV geometry variants (libgv<maxtpw>_<target>.so), HIP
graph over a ring of distinct matrices (> 600 MB per shape, beyond the MALL)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin
dev = torch.device("cuda:0")
P, L64, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
libs = [(nm, ctypes.CDLL(os.path.join(ROOT, "tools/dev", nm))) for nm in sys.argv[1:]]
SHAPES = [(4096, 4096, qlin.EP_NONE), (6144, 4096, qlin.EP_NONE), (28672, 4096, qlin.EP_SILU_MUL),
          (4096, 14336, qlin.EP_RESIDUAL)]
for (N, K, ep) in SHAPES:
    ring = max(8, -(-600_000_000 // (N * K // 2)))
    mats = []
    for i in range(ring):
        w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
        o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
        mats.append((o["qweight"], o["qsz"]))
        del w
    x = torch.randn(1, K, device=dev, dtype=torch.float16)
    ny = N // 2 if ep == qlin.EP_SILU_MUL else N
    y = torch.empty(1, ny, device=dev, dtype=torch.float16)
    r = torch.randn(1, ny, device=dev, dtype=torch.float16)
    res = {}
    outs = {}
    for nm, lib in libs:
        def step():
            st = P(torch.cuda.current_stream().cuda_stream)
            for qw, qsz in mats:
                rc = lib.qlin_linear_ep_f16(P(qw.data_ptr()), P(qsz.data_ptr()), 0, P(x.data_ptr()), None,
                                            P(r.data_ptr()) if ep == qlin.EP_RESIDUAL else None,
                                            P(y.data_ptr()), L64(1), L64(N), L64(K), 4, 128, ep, 0, 0,
                                            None, st)
                assert rc == 0, rc
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        g.replay(); torch.cuda.synchronize()
        best = 1e9
        for _ in range(5):
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            for _ in range(5):
                g.replay()
            e1.record(); torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e3 / (5 * ring))
        res[nm] = round(best, 2)
        outs[nm] = y.clone()
    base = next(iter(outs.values()))
    same = {nm: bool(torch.equal(o, base)) for nm, o in outs.items()}
    print(f"N={N} K={K} ep={ep} ring={ring}: us/launch {res}  same-as-first {same}", flush=True)
