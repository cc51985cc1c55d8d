"""Dev: per-wave timelines of the rows / whole-row GEMV kernels (stamped build, GEMV_ROWS_STAMP): for each decode
shape, a graph of dependent launches over a ring of distinct matrices; every launch records per
wave s_memrealtime (100 MHz) at entry (0), prologue loads issued (1), x parked (2), first tile
computed (3), last tile computed (4), exit (5).  Prints percentiles over waves, in us from the
launch's first wave entry, and the gap from the previous launch's last exit."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch  # noqa: E402
from quant import qlin  # noqa: E402

dev = torch.device("cuda:0")
P, L64, F = ctypes.c_void_p, ctypes.c_int64, ctypes.c_float
lib = ctypes.CDLL(os.path.join(ROOT, "tools/dev", sys.argv[1]))
SHAPES = [("qkv+norm", 6144, 4096, qlin.EP_NONE, True), ("o+res", 4096, 4096, qlin.EP_RESIDUAL, False),
          ("gateup+norm+silu", 28672, 4096, qlin.EP_SILU_MUL, True),
          ("down+res", 4096, 14336, qlin.EP_RESIDUAL, False)]
for (name, N, K, ep, nrm) in SHAPES:
    ring = 8
    mats = []
    for i in range(ring):
        w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
        o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
        mats.append((o["qweight"], o["qsz"]))
    x = torch.randn(1, K, device=dev, dtype=torch.float16)
    nw = (1 + 0.1 * torch.randn(K, device=dev)).float()
    ny = N // 2 if ep == qlin.EP_SILU_MUL else N
    y = torch.empty(1, ny, device=dev, dtype=torch.float16)
    r = torch.randn(1, ny, device=dev, dtype=torch.float16)
    nbmax = 4096
    st = torch.zeros(ring, nbmax * 16 * 8, dtype=torch.int64, device=dev)

    def step():
        s_ = P(torch.cuda.current_stream().cuda_stream)
        for i, (qw, qsz) in enumerate(mats):
            lib.qlin_dev_rows_stamps(P(st[i].data_ptr()))
            if nrm:
                rc = lib.qlin_rmsnorm_linear_ep_f16(
                    P(qw.data_ptr()), P(qsz.data_ptr()), 0, P(x.data_ptr()), P(nw.data_ptr()),
                    F(1e-5), None, None, P(y.data_ptr()), L64(1), L64(N), L64(K), 4, 128, ep, s_)
            else:
                rc = lib.qlin_linear_ep_f16(
                    P(qw.data_ptr()), P(qsz.data_ptr()), 0, P(x.data_ptr()), None,
                    P(r.data_ptr()) if ep == qlin.EP_RESIDUAL else None, P(y.data_ptr()),
                    L64(1), L64(N), L64(K), 4, 128, ep, 0, 0, None, L64(0), s_)
            assert rc == 0
        lib.qlin_dev_rows_stamps(None)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    for _ in range(30):
        g.replay()
    torch.cuda.synchronize()
    st.zero_()
    g.replay()
    torch.cuda.synchronize()
    S = st.view(ring, nbmax * 16, 8).cpu()
    prev_end = None
    print(f"== {name} N={N} K={K}", flush=True)
    for i in range(ring):
        v = S[i]
        valid = v[:, 0] > 0
        v = v[valid].double()
        if v.shape[0] == 0:  # a kernel without stamps (the fast kernel)
            print(f" launch {i}: no stamps", flush=True)
            break
        t0 = v[:, 0].min()
        rel = (v - t0) / 100.0  # us
        q = lambda c, p: torch.quantile(rel[:, c], p).item()  # noqa: E731
        span = (v[:, 5].max() - t0).item() / 100.0
        gap = (t0 - prev_end).item() / 100.0 if prev_end is not None else float("nan")
        prev_end = v[:, 5].max()
        if i >= 2:
            print(f" launch {i}: waves {v.shape[0]} span {span:.2f} gap {gap:.2f} | entry p50/p100 "
                  f"{q(0, .5):.2f}/{q(0, 1):.2f} issued p50 {q(1, .5):.2f} xpark p50/max "
                  f"{q(2, .5):.2f}/{q(2, 1):.2f} first-tile p10/p50/p90 {q(3, .1):.2f}/{q(3, .5):.2f}/"
                  f"{q(3, .9):.2f} last-tile p10/p50/p90/max {q(4, .1):.2f}/{q(4, .5):.2f}/{q(4, .9):.2f}/"
                  f"{q(4, 1):.2f} exit max {q(5, 1):.2f}", flush=True)
    if os.environ.get("STAMP_BREAKDOWN") and (S[ring - 1].view(nbmax, 16, 8)[:, :, 0] > 0).any():
        v = S[ring - 1].view(nbmax, 16, 8)
        blk = torch.arange(nbmax)[:, None].expand(nbmax, 16)
        wv = torch.arange(16)[None, :].expand(nbmax, 16)
        ok = v[:, :, 0] > 0
        t0 = v[:, :, 0][ok].min()
        last = (v[:, :, 4].double() - t0) / 100.0
        for nm_, key in (("block % 8", blk % 8), ("wave", wv), ("block // 32", blk // 32)):
            parts = []
            for k_ in range(int(key[ok].max()) + 1):
                sel = ok & (key == k_)
                if sel.any():
                    parts.append(f"{k_}:{last[sel].median().item():.2f}/{last[sel].max().item():.2f}")
            print(f"   last-tile median/max by {nm_}: " + " ".join(parts), flush=True)
    del mats, g
    torch.cuda.empty_cache()
