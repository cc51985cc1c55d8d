"""Launch-floor probes: empty kernels and streaming reads of one 8.4 MB matrix over a ring, by grid."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
dev = torch.device("cuda:0")
lib = ctypes.CDLL(os.path.join(ROOT, "tools/dev/libdev.so"))
P = ctypes.c_void_p
R = 64
bufs = [torch.empty(8929280 // 4, dtype=torch.int32, device=dev) for _ in range(R)]
out = torch.zeros(4, dtype=torch.int32, device=dev)


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


st = lambda: P(torch.cuda.current_stream().cuda_stream)
for (b, t) in ((1, 64), (1, 1024), (256, 64), (256, 256), (256, 1024), (512, 256), (2048, 256), (4096, 256)):
    us = timed(lambda: [lib.dev_empty_cfg(b, t, P(out.data_ptr()), st()) for _ in range(R)])
    print(f"empty  {b:5d} x {t:4d}: {us:6.3f} us", flush=True)
for (b, t) in ((256, 1024), (512, 512), (512, 1024), (1024, 256), (1024, 512), (2048, 256), (2048, 512), (4096, 256)):
    us = timed(lambda: [lib.dev_stream_cfg(P(bf.data_ptr()), ctypes.c_int64(bf.numel() * 4), b, t, P(out.data_ptr()), st()) for bf in bufs])
    print(f"stream {b:5d} x {t:4d}: {us:6.3f} us  ({8929280 / us / 1e3:7.1f} GB/s)", flush=True)
