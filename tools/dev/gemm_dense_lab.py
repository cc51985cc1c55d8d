"""Dev: large-M GEMM as dequant pre-pass + dense-B MFMA GEMM (tools/dev/gemm_dense_lab.hip) vs the
product's fused qlin_gemm_f16, int4 g128 N = K = 4096: bit-identity and TFLOP/s per M."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch  # noqa: E402
from quant import qlin  # noqa: E402

lab = ctypes.CDLL(os.path.join(ROOT, "tools/dev/libgd.so"))
P, L = ctypes.c_void_p, ctypes.c_int64
lab.lab_dequant_frag.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int, P]
lab.lab_gemm_dense.argtypes = [P, P, P, L, ctypes.c_int, ctypes.c_int, P]
lab.lab_gemm_dense3.argtypes = [P, P, P, L, ctypes.c_int, ctypes.c_int, P]
dev = torch.device("cuda:0")
N = K = 4096
w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
qw, qsz = o["qweight"], o["qsz"]
wf = torch.empty(N * K, dtype=torch.float16, device=dev)


def t_events(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    return best


for M in [int(m) for m in os.environ.get("MS", "2048,8192,65536").split(",")]:
    x = torch.empty(M, K, device=dev, dtype=torch.float16).normal_()
    y0 = qlin.gemm(x, qw, qsz, None, N, K, 4, 128, o["flags"], split=False)
    y1 = torch.empty(M, N, device=dev, dtype=torch.float16)
    st = P(torch.cuda.current_stream().cuda_stream)

    def pre():
        assert lab.lab_dequant_frag(P(qw.data_ptr()), P(qsz.data_ptr()), P(wf.data_ptr()), N, K, st) == 0

    def dense():
        assert lab.lab_gemm_dense(P(x.data_ptr()), P(wf.data_ptr()), P(y1.data_ptr()), M, N, K, st) == 0

    def dense3():
        assert lab.lab_gemm_dense3(P(x.data_ptr()), P(wf.data_ptr()), P(y1.data_ptr()), M, N, K, st) == 0

    pre()
    fl = 2.0 * M * N * K
    reps = max(3, int(2e12 // (2 * M * N * K)))
    tp = t_events(lambda: qlin.gemm(x, qw, qsz, None, N, K, 4, 128, o["flags"], split=False), reps)
    tpre = t_events(pre, 20)
    msg = f"M={M}: fused {tp*1e3:.1f} us = {fl/tp/1e9:.0f} TF; pre-pass {tpre*1e3:.1f} us"
    for nm, fn in (("dense", dense), ("dense3", dense3)):
        y1.zero_()
        fn()
        torch.cuda.synchronize()
        nd = int((y0 != y1).sum().item())
        td = t_events(fn, reps)
        msg += f"; {nm} {td*1e3:.1f} us = {fl/td/1e9:.0f} TF (+pre {fl/(td+tpre)/1e9:.0f}), {nd} differ"
    print(msg, flush=True)
    del x, y0, y1
