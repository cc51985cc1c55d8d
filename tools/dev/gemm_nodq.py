"""Dev: the product GEMM block with and without its dequant VALU (B = raw packed words, wrong
values): how much of the MFMA time the dequant costs.  int4 g128, N = K = 4096."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin
dev = torch.device("cuda:0")
lab = ctypes.CDLL(os.path.join(ROOT, "tools/dev/libgemmlab.so"))
P = ctypes.c_void_p
N = K = 4096
w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
wdq = qlin.dequant(o["qweight"], o["qsz"], N, K, 4, 128)


def timeit(fn, reps):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


for M in (2048, 8192, 65536):
    x = torch.randn(M, K, device=dev, dtype=torch.float16)
    y = torch.empty(M, N, device=dev, dtype=torch.float16)
    f = 2 * M * N * K
    st = P(torch.cuda.current_stream().cuda_stream)
    reps = 20 if M < 65536 else 5
    line = f"M={M}:"
    for bn in (256, 512):
        for nodq in (0, 1):
            t = timeit(lambda: lab.lab_gemm_nodq(P(o["qweight"].data_ptr()), P(o["qsz"].data_ptr()),
                                                 P(x.data_ptr()), P(y.data_ptr()), ctypes.c_int64(M),
                                                 N, K, bn, nodq, st), reps)
            line += f" bn{bn}{'-nodq' if nodq else ''} {f / t / 1e12:.0f}"
    t = timeit(lambda: torch.nn.functional.linear(x, wdq), reps)
    line += f" | hipBLASLt fp16 {f / t / 1e12:.0f} TF/s"
    print(line, flush=True)
