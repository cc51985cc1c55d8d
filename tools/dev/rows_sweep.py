"""Dev: the decode layer's four linear launches (M = 1, int4 g128) under library variants, each a HIP
graph of dependent launches over a ring of distinct matrices (> 600 MB per shape, beyond the
MALL).  Usage: rows_sweep.py lib1.so [lib2.so ...]; a library named libr3*.so is called with the
round-3 (ABI 9) signature of qlin_rmsnorm_linear_ep_f16; lib.so@w16 is lib.so with the norm weight
in fp16 (QLIN_NORM_W16)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch  # noqa: E402
from quant import qlin  # noqa: E402

dev = torch.device("cuda:0")
P, L64, F = ctypes.c_void_p, ctypes.c_int64, ctypes.c_float

def _open(nm):
    f = nm.split("@")[0]
    if f == "libqlin_gfx950.so" and "/" not in f:
        f = os.path.join(ROOT, "llama3-quantization_amd/csrc", f)
    return ctypes.CDLL(f if "/" in f else os.path.join(ROOT, "tools/dev", f))


libs = [(os.path.basename(nm), _open(nm)) for nm in sys.argv[1:]]
# (name, N, K, epilogue, fused RMSNorm)
SHAPES = [("qkv+norm", 6144, 4096, qlin.EP_NONE, True), ("o+res", 4096, 4096, qlin.EP_RESIDUAL, False),
          ("gateup+norm+silu", 28672, 4096, qlin.EP_SILU_MUL, True),
          ("down+res", 4096, 14336, qlin.EP_RESIDUAL, False), ("plain4096", 4096, 4096, qlin.EP_NONE, False)]
only = os.environ.get("ROWS_ONLY")
for (name, N, K, ep, nrm) in SHAPES:
    if only and name not in only.split(","):
        continue
    ring = max(8, -(-700_000_000 // (N * K // 2)))
    mats = []
    for i in range(ring):
        w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
        o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
        mats.append((o["qweight"], o["qsz"]))
        del w
    x = torch.randn(1, K, device=dev, dtype=torch.float16)
    nw16 = (1 + 0.1 * torch.randn(K, device=dev)).half()
    nw = nw16.float()
    ny = N // 2 if ep == qlin.EP_SILU_MUL else N
    y = torch.empty(1, ny, device=dev, dtype=torch.float16)
    r = torch.randn(1, ny, device=dev, dtype=torch.float16)
    res, outs = {}, {}
    for nm, lib in libs:
        r3 = nm.startswith("libr3")
        w16 = nm.endswith("@w16")

        def step():
            st = P(torch.cuda.current_stream().cuda_stream)
            for qw, qsz in mats:
                if nrm:
                    extra = (None, L64(0), None, None, None, L64(0), None) if r3 else ()
                    rc = lib.qlin_rmsnorm_linear_ep_f16(
                        P(qw.data_ptr()), P(qsz.data_ptr()), qlin.NORM_W16 if w16 else 0,
                        P(x.data_ptr()), P((nw16 if w16 else nw).data_ptr()),
                        F(1e-5), None, None, P(y.data_ptr()), L64(1), L64(N), L64(K), 4, 128, ep,
                        *extra, st)
                else:
                    rc = lib.qlin_linear_ep_f16(
                        P(qw.data_ptr()), P(qsz.data_ptr()), 0, P(x.data_ptr()), None,
                        P(r.data_ptr()) if ep == qlin.EP_RESIDUAL else None, P(y.data_ptr()),
                        L64(1), L64(N), L64(K), 4, 128, ep, 0, 0, None, L64(0), st)
                assert rc == 0, (nm, rc)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        for _ in range(20):
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
        outs[nm] = y.clone()
        del g
    base = next(iter(outs.values()))
    diff = {nm: round(((o.float() - base.float()).abs().max() / base.float().abs().max()).item(), 5)
            for nm, o in outs.items()}
    gb = N * K / 2 * (1 + 3 / 64) / 1e3
    print(f"{name} N={N} K={K} ring={ring}: us/launch {res}  GB/s "
          f"{ {k: round(gb / v) for k, v in res.items()} }  rel-diff-vs-first {diff}", flush=True)
    del mats
    torch.cuda.empty_cache()
