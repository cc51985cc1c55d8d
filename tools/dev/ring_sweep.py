"""Dev: per-launch time of the batched streaming GEMV against the number of products per launch
(int4 g128 4096^2, one process, one warm clock, graph-replayed, best of 5 x 40 replays).  The
slope is the streaming cost per matrix; the intercept is what a launch pays once (dispatch gap,
wave ramp, tail).  Usage: python tools/dev/ring_sweep.py [bits] [group]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llama3-quantization_amd")]
import torch  # noqa: E402
from quant import qlin  # noqa: E402

bits = int(sys.argv[1]) if len(sys.argv) > 1 else 4
group = int(sys.argv[2]) if len(sys.argv) > 2 else 128
N = K = 4096
RS = [16, 32, 64, 128, 256]
dev = torch.device("cuda", 0)
lib = qlin.load_library()
Rmax = max(RS)
qw = torch.zeros((Rmax, *qlin.packed_shape(N, K, bits)), dtype=torch.int32, device=dev)
sz = torch.zeros((Rmax, *qlin.sz_shape(N, K, group)), dtype=torch.int32, device=dev)
g = torch.Generator(device=dev)
for i in range(Rmax):
    g.manual_seed(i)
    w = torch.empty(N, K, device=dev, dtype=torch.float16).normal_(0, 0.02, generator=g)
    o = qlin.quantize(w, bits, group, 0, want_xdq=False, want_params=False, pack=True)
    qw[i].copy_(o["qweight"])
    sz[i].copy_(o["qsz"])
xs = torch.randn(Rmax, 1, K, device=dev, dtype=torch.float16, generator=g)
y = torch.empty(Rmax, 1, N, device=dev, dtype=torch.float16)


def graph_for(R):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())

    def call(st):
        assert lib.qlin_gemv_batched_f16(qw.data_ptr(), qw[0].numel(), sz.data_ptr(), sz[0].numel(),
                                         0, xs.data_ptr(), K, None, 0, y.data_ptr(), N, R, 1, N, K,
                                         bits, group, st) == 0
    with torch.cuda.stream(s):
        call(s.cuda_stream)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        call(s.cuda_stream)
    torch.cuda.current_stream().wait_stream(s)
    return gr


graphs = {R: graph_for(R) for R in RS}
t0 = time.perf_counter()
while time.perf_counter() - t0 < 1.0:  # clock ramp
    graphs[64].replay()
    torch.cuda.synchronize()
best = {R: 1e9 for R in RS}
for rep in range(5):
    for R in RS:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(40):
            graphs[R].replay()
        e1.record()
        torch.cuda.synchronize()
        best[R] = min(best[R], e0.elapsed_time(e1) * 1e3 / 40)
nb = N * K * bits // 8 + N * (K // group) * 3 + 2 * K + 2 * N
for R in RS:
    print(f"R={R:4d}: {best[R]:8.2f} us per launch, {best[R] / R:6.3f} us per matrix, "
          f"{R * nb / best[R] / 1e3:7.1f} GB/s", flush=True)
# least squares over the three largest rings
import numpy as np  # noqa: E402
xs_ = np.array(RS[-3:], dtype=float)
ys_ = np.array([best[R] for R in RS[-3:]])
slope, icpt = np.polyfit(xs_, ys_, 1)
print(f"fit over R = {RS[-3:]}: {slope:.3f} us per matrix ({nb / slope / 1e3:.1f} GB/s), "
      f"intercept {icpt:.2f} us per launch", flush=True)
