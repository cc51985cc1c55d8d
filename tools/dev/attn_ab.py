"""Timing of fused decode-attention variants (libattn<mode>.so, see ATTN_FENCE_MODE) in HIP graphs
over a ring of distinct KV caches; also checks each against mode 0's output.  (dev)"""
import ctypes, math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
dev = torch.device("cuda:0")
P, L64, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
libs = {p: ctypes.CDLL(os.path.join(ROOT, "tools/dev", p)) for p in sys.argv[1:]}
for lib in libs.values():
    lib.qlin_attn_decode_partials_bytes.restype = ctypes.c_int64
    lib.qlin_attn_decode_partials_bytes.argtypes = [L64, I, I, L64]


def run(B, Hq, Hkv, L, R=16, reps=20):
    g = torch.Generator(device=dev).manual_seed(0)
    qs = [torch.randn(B, Hq, 128, device=dev, generator=g) for _ in range(R)]
    ks = [torch.randn(B, Hkv, L, 128, device=dev, generator=g).half() for _ in range(R)]
    vs = [torch.randn(B, Hkv, L, 128, device=dev, generator=g).half() for _ in range(R)]
    res = {}
    outs = {}
    for name, lib in libs.items():
        nb = lib.qlin_attn_decode_partials_bytes(B, Hq, Hkv, L)
        part = torch.empty(max(nb, 4) // 4, device=dev)
        cnt = torch.zeros(B * Hkv, dtype=torch.int32, device=dev)
        out = [torch.empty(B, Hq, 128, device=dev) for _ in range(R)]

        def f():
            st = P(torch.cuda.current_stream().cuda_stream)
            for i in range(R):
                rc = lib.qlin_attn_decode(P(qs[i].data_ptr()), P(ks[i].data_ptr()), P(vs[i].data_ptr()), None,
                                          P(out[i].data_ptr()), 1, L64(B), Hq, Hkv, L64(L), 128, L64(0),
                                          ctypes.c_float(math.sqrt(128)), P(part.data_ptr()), P(cnt.data_ptr()), st)
                assert rc == 0, rc
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            f()
        torch.cuda.current_stream().wait_stream(s)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            f()
        gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(reps):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) * 1e3 / reps / R, 2)
        outs[name] = out[-1].clone()
    base = next(iter(outs.values()))
    diffs = {n: float((o - base).abs().max()) for n, o in outs.items()}
    kvb = 2 * B * Hkv * L * 128 * 2
    print({"B": B, "Hq": Hq, "Hkv": Hkv, "L": L, "us": res, "kv_GBps": {n: round(kvb / t / 1e3) for n, t in res.items()},
           "maxdiff_vs_first": diffs}, flush=True)


CFGS = [(1, 32, 8, 513), (1, 32, 8, 2048), (1, 32, 8, 4096), (16, 32, 8, 2048), (64, 32, 8, 1024)]
if os.environ.get("CFGS"):  # "B,Hq,Hkv,L;..."
    CFGS = [tuple(int(x) for x in c.split(",")) for c in os.environ["CFGS"].split(";")]
for cfg in CFGS[:int(os.environ.get("NCFG", "99"))]:
    run(*cfg)
