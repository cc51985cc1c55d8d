"""Does a decode GEMV run faster when its packed weights were just read by another kernel (the
MALL / Infinity Cache warm)?  Ring of R distinct packed matrices (> 256 MB in total), graph-replayed:
  cold  = gemv(W_i) for i in ring
  touch = sum(W_i.view(int32)) for i in ring (a plain streaming read, no GEMV)
  both  = touch(W_i) then gemv(W_i) for i in ring (same stream)
gemv on warm weights ~ both - touch.  (dev; decides whether a prefetch of the next launches'
weights, run beside the latency-bound attention launch, is worth building)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch  # noqa: E402

from quant import qlin  # noqa: E402

dev = torch.device("cuda:0")


def timed(fn, reps=10):
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        fn()
    for _ in range(3):
        gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def run(N, K, R):
    g = torch.Generator(device=dev).manual_seed(N)
    w = (torch.randn(N, K, device=dev, generator=g) * 0.02).half()
    o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
    qw0, sz0, fl = o["qweight"], o["qsz"], o["flags"]
    qws = [qw0.clone() for _ in range(R)]
    szs = [sz0.clone() for _ in range(R)]
    x = torch.randn(1, K, device=dev, generator=g).half()
    acc = torch.zeros(R, dtype=torch.int64, device=dev)

    def gemv(i):
        qlin.linear(x, qws[i], szs[i], None, N, K, 4, 128, fl)

    def touch(i):
        torch.sum(qws[i].view(-1), 0, out=acc[i])

    cold = timed(lambda: [gemv(i) for i in range(R)]) / R
    tch = timed(lambda: [touch(i) for i in range(R)]) / R
    both = timed(lambda: [(touch(i), gemv(i)) for i in range(R)]) / R
    mb = qw0.numel() * 4 / 1e6
    print({"N": N, "K": K, "MB": round(mb, 1), "R": R, "gemv_cold_us": round(cold, 2),
           "touch_us": round(tch, 2), "touch_then_gemv_us": round(both, 2),
           "gemv_warm_est_us": round(both - tch, 2),
           "cold_TBps": round(mb / cold, 2), "warm_TBps": round(mb / max(both - tch, 1e-3), 2)},
          flush=True)


for N, K, R in [(4096, 4096, 48), (28672, 4096, 8), (4096, 14336, 16), (6144, 4096, 32)]:
    run(N, K, R)
