"""Dev (round 6): decode GEMV time with its weights L2-warm on the computing XCD vs MALL-warm vs
cold (tools/dev/l2pf_lab.hip).  Per shape, a ring of R distinct packed int4 g128 matrices (> 256 MB
in total), graph-replayed; per matrix i:
  cold    touch(W_{i+R/2}) then gemv(W_i)  (the same touch traffic, on other bytes)
  mall    touch(W_i, shift 1) then gemv(W_i)  (read on another XCD: Infinity-Cache-warm)
  l2      touch(W_i, shift 0) then gemv(W_i)  (read on the computing XCD)
  touch   touch alone
gemv time ~ pair - touch.  Prints one line per shape."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch  # noqa: E402

from quant import qlin  # noqa: E402

dev = torch.device("cuda:0")
lab = ctypes.CDLL(os.path.join(ROOT, "tools/dev/libl2pf.so"))
P, L, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
lab.lab_touch_rows.argtypes = [P, L, P, L, I, I, I, P, P]
sink = torch.zeros(1 << 20, dtype=torch.int32, device=dev)
NB = int(os.environ.get("TOUCH_BLOCKS", "1024"))


def timed(fn, reps=20):
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        fn()
    for _ in range(5):
        gr.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(reps):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


def run(name, N, K):
    g = torch.Generator(device=dev).manual_seed(N + K)
    w = (torch.randn(N, K, device=dev, generator=g) * 0.02).half()
    o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
    del w
    mb = (o["qweight"].numel() + o["qsz"].numel()) * 4 / 1e6
    R = max(8, int(600 / mb) // 2 * 2)
    qws = [o["qweight"].clone() for _ in range(R)]
    szs = [o["qsz"].clone() for _ in range(R)]
    x = torch.randn(1, K, device=dev, generator=g).half()
    Nt = qws[0].shape[0]
    q16 = qws[0][0].numel() // 4
    s16 = szs[0][0].numel() // 4
    st = lambda: P(torch.cuda.current_stream().cuda_stream)  # noqa: E731

    def touch(i, shift):
        lab.lab_touch_rows(P(qws[i].data_ptr()), q16, P(szs[i].data_ptr()), s16, Nt, NB, shift,
                           P(sink.data_ptr()), st())

    def gemv(i):
        qlin.gemv(x, qws[i], szs[i], None, N, K, 4, 128, o["flags"])

    res = {"route": qlin.m1_route(N, K, 4, 128), "MB": round(mb, 2), "ring": R}
    res["gemv"] = timed(lambda: [gemv(i) for i in range(R)]) / R
    res["touch"] = timed(lambda: [touch(i, 0) for i in range(R)]) / R
    for mode, fn in (("cold", lambda i: (touch((i + R // 2) % R, 0), gemv(i))),
                     ("mall", lambda i: (touch(i, 1), gemv(i))),
                     ("l2", lambda i: (touch(i, 0), gemv(i)))):
        res[mode] = timed(lambda: [fn(i) for i in range(R)]) / R - res["touch"]
    print(name, {k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()},
          flush=True)
    del qws, szs
    torch.cuda.empty_cache()


for nm, N, K in (("o_4096x4096", 4096, 4096), ("qkv_6144x4096", 6144, 4096),
                 ("down_4096x14336", 4096, 14336), ("gateup_28672x4096", 28672, 4096)):
    run(nm, N, K)
