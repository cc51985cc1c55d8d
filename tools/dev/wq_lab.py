"""Dev: the work-queue wide GEMV lab (tools/dev/wq_lab.hip, libwq.so) against the product's
whole-row route on the gate/up decode launch (N 28,672 x K 4,096, int4 g128, fp16 RMSNorm + SiLU*up),
each a HIP graph of dependent launches over a ring of distinct matrices (> 700 MB, beyond the
MALL).  Prints us per launch and the max difference to the product's output; STAMPS=1 adds the
per-wave stamp summary of one cold launch."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch  # noqa: E402
from quant import qlin  # noqa: E402

dev = torch.device("cuda:0")
lab = ctypes.CDLL(os.path.join(ROOT, "tools/dev/libwq.so"))
prodlib = qlin.load_library()
oldlib = ctypes.CDLL(os.path.join(ROOT, "tools/dev/libold.so")) if os.path.exists(
    os.path.join(ROOT, "tools/dev/libold.so")) else None
P, F = ctypes.c_void_p, ctypes.c_float
lab.lab_wq.argtypes = [P, P, P, P, F, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                       ctypes.c_int, P, P]
lab.lab_wqd.argtypes = lab.lab_wq.argtypes  # "wqdN": LDS-DMA ring of N chunks per wave
N, K = int(os.environ.get("N", 28672)), int(os.environ.get("K", 4096))
ep = qlin.EP_SILU_MUL
ring = max(8, -(-700_000_000 // (N * K // 2)))
mats = []
for i in range(ring):
    w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
    o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
    mats.append((o["qweight"], o["qsz"]))
    del w
x = torch.randn(1, K, device=dev, dtype=torch.float16) * 3
nw16 = (1 + 0.1 * torch.randn(K, device=dev)).half()
y0 = torch.empty(1, N // 2, device=dev, dtype=torch.float16)
y1 = torch.empty(1, N // 2, device=dev, dtype=torch.float16)
cus = torch.cuda.get_device_properties(0).multi_processor_count
variants = [v for v in os.environ.get("VARIANTS", "prod,wq840,wq841,wq820,wq480,wq481,wq440,wq441").split(",")]


def run(v, qw, qsz, y, stamps=None):
    st = P(torch.cuda.current_stream().cuda_stream)
    if v in ("prod", "old"):  # the library call itself, into the preallocated y (no copy)
        L = prodlib if v == "prod" else oldlib
        rc = L.qlin_rmsnorm_linear_ep_f16(P(qw.data_ptr()), P(qsz.data_ptr()), qlin.NORM_W16,
                                          P(x.data_ptr()), P(nw16.data_ptr()), F(1e-5), None, None,
                                          P(y.data_ptr()), ctypes.c_int64(1), ctypes.c_int64(N),
                                          ctypes.c_int64(K), 4, 128, ep, st)
        assert rc == 0, rc
        return
    fn, arg = (lab.lab_wqd, int(v[3:])) if v.startswith("wqd") else (lab.lab_wq, int(v[2:]))
    rc = fn(P(qw.data_ptr()), P(qsz.data_ptr()), P(x.data_ptr()), P(nw16.data_ptr()),
                    F(1e-5), P(y.data_ptr()), N, K, ep, arg, cus,
                    P(stamps.data_ptr() if stamps is not None else 0), st)
    assert rc == 0, rc


ref = None
res = {}
for v in variants:
    run(v, *mats[0], y1)
    torch.cuda.synchronize()
    if ref is None:
        ref = y1.clone()
    d = ((y1.float() - ref.float()).abs().max() / ref.float().abs().max()).item()

    def step(v=v):
        for qw, qsz in mats:
            run(v, qw, qsz, y1)
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
    res[v] = (round(best, 2), f"{d:.1e}")
    del g
print(f"N={N} K={K} ring={ring}: us/launch, rel diff vs {variants[0]}: {res}", flush=True)

if os.environ.get("STAMPS"):
    for v in variants:
        if v in ("prod", "old"):
            continue
        stamps = torch.zeros(cus * 8 * 8, dtype=torch.int64, device=dev)
        # cold: other matrices streamed in between
        for qw, qsz in mats[1:]:
            run(v, qw, qsz, y1)
        torch.cuda.synchronize()
        run(v, *mats[0], y1, stamps)
        torch.cuda.synchronize()
        s = stamps.view(cus, 8, 8).cpu().double()
        t0 = s[:, :, 0][s[:, :, 0] > 0].min()
        out = {}
        for k, nm in ((0, "start"), (1, "issued"), (2, "xstaged"), (4, "done"), (5, "exit")):
            col = s[:, :, k]
            col = (col[col > 0] - t0) / 100.0
            out[nm] = (round(col.median().item(), 2), round(col.max().item(), 2))
        done = (s[:, :, 4] - t0) / 100.0
        byw = {w: round(done[:, w].median().item(), 2) for w in range(8)}
        print(f"{v} stamps (median, max us): {out}  done by wave: {byw}", flush=True)
