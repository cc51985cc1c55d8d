"""Dev GEMV lab: timings of knob variants + per-wave stamp timeline (int4 g128 4096^2, M=1)."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin

dev = torch.device("cuda:0")
lab = ctypes.CDLL(os.path.join(ROOT, "tools/dev/liblab.so"))
R, N, K = 64, 4096, 4096
mats = []
for i in range(R):
    w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
    o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
    mats.append((o["qweight"], o["qsz"]))
x = torch.randn(1, K, device=dev, dtype=torch.float16)
ys = [torch.empty(1, N, device=dev, dtype=torch.float16) for _ in range(8)]
P = ctypes.c_void_p


def st():
    return P(torch.cuda.current_stream().cuda_stream)


def launch(m, y, W, PF, NT, MODE, stamps=None, RED=0, XL=0):
    rc = lab.lab_gemv_launch(P(m[0].data_ptr()), P(m[1].data_ptr()), P(x.data_ptr()),
                             P(y.data_ptr()), N, K, W, PF, NT, MODE, RED,
                             P(stamps.data_ptr() if stamps is not None else 0), st(), XL)
    assert rc == 0


out = torch.zeros(4, dtype=torch.int32, device=dev)


def launch_stream(m, stamps=None):
    rc = lab.lab_stream_launch(P(m[0].data_ptr()), ctypes.c_int64(m[0].numel() * 4),
                               P(out.data_ptr()), P(stamps.data_ptr() if stamps is not None else 0),
                               st())
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


# correctness
ref = qlin.gemv(x, mats[0][0], mats[0][1], None, N, K, 4, 128)
for (W, MODE, RED, XL) in ((16, 0, 1, 1), (16, 10, 1, 1), (8, 10, 1, 1)):
    y = torch.empty(1, N, device=dev, dtype=torch.float16)
    launch(mats[0], y, W, 2, 0, MODE, RED=RED, XL=XL)
    torch.cuda.synchronize()
    d = (y.float() - ref.float()).abs().max().item() / ref.float().abs().max().item()
    print(f"check W={W} mode{MODE} red{RED} xl{XL}: max |lab - product| / max|y| = {d:.3g}")

CONFIGS = [  # (W, PF, NT, MODE, RED, XL)
    (16, 2, 1, 0, 1, 1), (16, 2, 1, 1, 1, 1), (16, 2, 1, 10, 1, 1), (8, 4, 1, 10, 1, 1),
    (8, 2, 1, 10, 1, 1), (16, 2, 1, 3, 1, 1),
]
if os.environ.get("LAB_CONFIGS"):
    CONFIGS = [tuple(int(v) for v in c.split(",")) for c in os.environ["LAB_CONFIGS"].split(";")]
STAMP_CONFIGS = [(16, 2, 1, 10, 1, 1)]
if os.environ.get("LAB_STAMPS"):
    STAMP_CONFIGS = [tuple(int(v) for v in c.split(",")) for c in os.environ["LAB_STAMPS"].split(";")]
res = {}
res["stream"] = timed(lambda: [launch_stream(m) for m in mats])
print(f"stream: {res['stream']:.3f} us", flush=True)
for c in CONFIGS:
    W, PF, NT, MODE, RED, XL = c
    res[c] = timed(lambda: [launch(m, ys[j % 8], W, PF, NT, MODE, RED=RED, XL=XL)
                            for j, m in enumerate(mats)])
    print(f"W{W:2d} PF{PF} NT{NT} mode{MODE} red{RED} xl{XL}: {res[c]:.3f} us", flush=True)

# stamp timelines inside the ring: launch 32 of the ring carries the stamp buffer
stamps = torch.zeros(8192 * 4, dtype=torch.int64, device=dev)
q = lambda a: " ".join(f"{np.percentile(a, p):6.0f}" for p in (0, 10, 50, 90, 100))


def show(name, nw):
    s_ = stamps[: nw * 4].view(nw, 4).cpu().numpy().astype(np.int64)
    rel = (s_ - s_[:, 0].min()) * 10  # ns (100 MHz)
    print(f"{name}  [ns: p0 p10 p50 p90 p100]")
    print("  start      ", q(rel[:, 0]))
    print("  first tile ", q(rel[:, 1]))
    print("  body end   ", q(rel[:, 2]))
    print("  wave end   ", q(rel[:, 3]))


def ring_stamped(fn_stamped, fn):
    def f():
        for j, m in enumerate(mats):
            if j == 32:
                fn_stamped(j, m)
            else:
                fn(j, m)
    timed(f, reps=3)


ring_stamped(lambda j, m: launch_stream(m, stamps), lambda j, m: launch_stream(m))
torch.cuda.synchronize()
show("stream (ring)", 2048)
for c in STAMP_CONFIGS:
    W, PF, NT, MODE, RED, XL = c
    stamps.zero_()
    ring_stamped(lambda j, m: launch(m, ys[j % 8], W, PF, NT, MODE, stamps, RED, XL),
                 lambda j, m: launch(m, ys[j % 8], W, PF, NT, MODE, None, RED, XL))
    torch.cuda.synchronize()
    Kt = K // 128
    tpw = -(-Kt // W)
    show(f"W{W} PF{PF} NT{NT} mode{MODE} red{RED} xl{XL} (ring)", (N // 16) * (-(-Kt // tpw)))
