"""A/B timing of the GEMV in two library builds (same process, interleaved trials).
usage: python tools/dev/ab.py <libA.so> <libB.so> [M] [bits] [group]"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin
dev = torch.device("cuda:0")
libs = [ctypes.CDLL(p) for p in sys.argv[1:3]]
M = int(sys.argv[3]) if len(sys.argv) > 3 else 1
BITS = int(sys.argv[4]) if len(sys.argv) > 4 else 4
GRP = int(sys.argv[5]) if len(sys.argv) > 5 else 128
N = K = 4096
R = 64
P = ctypes.c_void_p
mats = []
for i in range(R):
    w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
    o = qlin.quantize(w, BITS, GRP, 0, want_xdq=False, want_params=False, pack=True)
    mats.append((o["qweight"], o["qsz"], o["flags"]))
x = torch.randn(M, K, device=dev, dtype=torch.float16)
ys = [torch.empty(M, N, device=dev, dtype=torch.float16) for _ in range(4)]


def graph_for(lib):
    def f():
        st = P(torch.cuda.current_stream().cuda_stream)
        for j, m in enumerate(mats):
            rc = lib.qlin_gemv_f16(P(m[0].data_ptr()), P(m[1].data_ptr()), m[2], P(x.data_ptr()), None,
                                   P(ys[j % 4].data_ptr()), ctypes.c_int64(M), ctypes.c_int64(N),
                                   ctypes.c_int64(K), BITS, GRP, st)
            assert rc == 0
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        f()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        f()
    return g


graphs = [graph_for(l) for l in libs]
res = [[], []]
for trial in range(10):
    for i, g in enumerate(graphs):
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(20):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        res[i].append(e0.elapsed_time(e1) * 1e3 / 20 / R)
import statistics as st
for i, p in enumerate(sys.argv[1:3]):
    print(f"{os.path.basename(p):28s} median {st.median(res[i]):.3f} us  min {min(res[i]):.3f}  max {max(res[i]):.3f}")
