"""Dev: tile placement vs dequant overlap (tools/dev/gemv_lab2.hip), int4 g128 4096^2, M = 1,
ring of 64 matrices, HIP events over graph replays; stamp timelines of selected variants."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin

dev = torch.device("cuda:0")
lab = ctypes.CDLL(os.path.join(ROOT, "tools/dev/liblab2.so"))
R, N, K = 64, 4096, 4096
mats = []
for i in range(R):
    w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
    o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
    mats.append((o["qweight"], o["qsz"]))
x = torch.randn(1, K, device=dev, dtype=torch.float16)
ys = [torch.empty(1, N, device=dev, dtype=torch.float16) for _ in range(8)]
P = ctypes.c_void_p
st = lambda: P(torch.cuda.current_stream().cuda_stream)


def launch(m, y, SC, MODE, stamps=None):
    rc = lab.lab2_launch(P(m[0].data_ptr()), P(m[1].data_ptr()), P(x.data_ptr()), P(y.data_ptr()),
                         N, K, SC, MODE, P(stamps.data_ptr() if stamps is not None else 0), st())
    assert rc == 0


def timed(fn, reps=20):
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
    return e0.elapsed_time(e1) * 1e3 / reps / R


ref = qlin.gemv(x, mats[0][0], mats[0][1], None, N, K, 4, 128)
for SC in (0, 1):
    y = torch.empty(1, N, device=dev, dtype=torch.float16)
    launch(mats[0], y, SC, 0)
    torch.cuda.synchronize()
    d = (y.float() - ref.float()).abs().max().item() / ref.float().abs().max().item()
    print(f"check SC={SC}: max |lab - product| / max|y| = {d:.3g}", flush=True)
prod = timed(lambda: [qlin.gemv(x, m[0], m[1], None, N, K, 4, 128) for m in mats])
print(f"product: {prod:.3f} us", flush=True)
for SC in (0, 1, 2, 3):
    for MODE in (0, 1, 2):
        us = timed(lambda: [launch(m, ys[j % 8], SC, MODE) for j, m in enumerate(mats)])
        print(f"SC={SC} MODE={MODE}: {us:.3f} us", flush=True)
stamps = torch.zeros(4096 * 4, dtype=torch.int64, device=dev)
q = lambda a: " ".join(f"{np.percentile(a, p):6.0f}" for p in (0, 10, 50, 90, 100))
for (SC, MODE) in ((0, 0), (1, 0), (2, 0), (2, 1)):
    stamps.zero_()

    def f():
        for j, m in enumerate(mats):
            launch(m, ys[j % 8], SC, MODE, stamps if j == 32 else None)
    timed(f, reps=3)
    torch.cuda.synchronize()
    s_ = stamps.view(4096, 4).cpu().numpy().astype(np.int64)
    rel = (s_ - s_[:, 0].min()) * 10
    print(f"SC={SC} MODE={MODE} [ns: p0 p10 p50 p90 p100]")
    for i, nm in enumerate(("start", "first tile", "body end", "wave end")):
        print(f"  {nm:11s}", q(rel[:, i]))
    # per-block spread of the first-tile time (is a CU's data a burst?)
    ft = rel[:, 1].reshape(256, 16)
    print("  per-block first-tile spread (max-min) p10/p50/p90:",
          " ".join(f"{v:.0f}" for v in np.percentile(ft.max(1) - ft.min(1), (10, 50, 90))))
