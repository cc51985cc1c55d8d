"""Dev: kernarg preload A/B (tools/dev/kp_lab.hip): libkp.so (no preload) vs libkp_pre.so
(-mllvm -amdgpu-kernarg-preload-count=16), both variants (struct / scalar arguments) each; 64
dependent launches over a ring of 64 distinct 8 MB buffers (> MALL) in one graph, best of 5."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

dev = torch.device("cuda", 0)
P = ctypes.c_void_p
libs = {}
for nm in ("libkp.so", "libkp_pre.so"):
    L = ctypes.CDLL(os.path.join(ROOT, "tools/dev", nm))
    L.kp_launch.argtypes = [ctypes.c_int, P, P, ctypes.c_int64, P]
    libs[nm] = L
nbytes = 256 * 512 * 16 * 4
R = 64
bufs = [torch.randint(0, 1 << 30, (nbytes // 4,), dtype=torch.int32, device=dev) for _ in range(R)]
out = torch.zeros(256, dtype=torch.int32, device=dev)
res = {}
for rep in range(5):
    for nm, L in libs.items():
        for variant in (0, 1):
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())

            def run(st):
                for b in bufs:
                    assert L.kp_launch(variant, P(b.data_ptr()), P(out.data_ptr()), nbytes, P(st)) == 0
            with torch.cuda.stream(s):
                run(s.cuda_stream)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                run(s.cuda_stream)
            torch.cuda.current_stream().wait_stream(s)
            for _ in range(3):
                g.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(10):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / (10 * R)
            key = f"{nm}:{'struct' if variant == 0 else 'scalar'}"
            res[key] = min(res.get(key, 1e9), us)
for k, v in res.items():
    print(f"{k:24s} {v:6.3f} us per dependent 8 MB launch ({nbytes / v / 1e3:6.1f} GB/s)", flush=True)
