"""Dev ablation timings (one process, graph replays over a ring of distinct buffers)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin

dev = torch.device("cuda:0")
lib = ctypes.CDLL(os.path.join(ROOT, "tools/dev/libdev.so"))
q = qlin.load_library()
R = 64
N = K = int(os.environ.get("NK", "4096"))
BITS = int(os.environ.get("BITS", "4"))
GRP = int(os.environ.get("GRP", "128"))
mats = []
for i in range(R):
    w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
    o = qlin.quantize(w, BITS, GRP, 0, want_xdq=False, want_params=False, pack=True)
    mats.append((o["qweight"], o["qsz"], o["flags"]))
x = torch.randn(4, K, device=dev, dtype=torch.float16)
ys = [torch.empty(4, N, device=dev, dtype=torch.float16) for _ in range(8)]
out = torch.zeros(4, dtype=torch.int32, device=dev)

def timed(fn, reps=20, ring=R, streams=1):
    side = [torch.cuda.Stream(dev) for _ in range(streams)]
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        if streams == 1:
            fn(0)
        else:
            cur = torch.cuda.current_stream()
            for sd in side:
                sd.wait_stream(cur)
            for i, sd in enumerate(side):
                with torch.cuda.stream(sd):
                    fn(i + 1, streams)
            for sd in side:
                cur.wait_stream(sd)
    for _ in range(3): g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps): g.replay()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps / ring  # us per launch

def st(): return torch.cuda.current_stream().cuda_stream

def gemv_ring(M, hot=False, extra=0):
    def f(part=0, nparts=1):
        sel = mats if part == 0 else mats[part - 1::nparts]
        for j, m in enumerate(sel):
            mm = mats[0] if hot else m
            y = ys[(j + part) % len(ys)]
            rc = q.qlin_gemv_f16(mm[0].data_ptr(), mm[1].data_ptr(), mm[2] | extra, x.data_ptr(), None, y.data_ptr(), M, N, K, BITS, GRP, st())
            assert rc == 0, rc
    return f

res = {}
res["empty_512"] = timed(lambda p=0, n=1: [lib.dev_empty(512, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(st())) for m in mats])
res["stream_read_pt4"] = timed(lambda p=0, n=1: [lib.dev_stream_read(ctypes.c_void_p(m[0].data_ptr()), ctypes.c_int64(m[0].numel()*4), ctypes.c_void_p(out.data_ptr()), 4, 0, ctypes.c_void_p(st())) for m in mats])
for M in (1, 2, 4):
    res[f"gemv_M{M}"] = timed(gemv_ring(M))
res["gemv_M1_hot"] = timed(gemv_ring(1, hot=True))
for ns in (2, 4, 8):
    res[f"gemv_M1_{ns}streams"] = timed(gemv_ring(1), streams=ns)
bytes_ = N*K*BITS//8 + N*(K//GRP)*4 + 2*K + 2*N
for k, v in res.items():
    print(f"{k:24s} {v:8.3f} us   {bytes_/v/1e3:8.1f} GB/s-equiv")
