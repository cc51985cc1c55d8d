"""Dev: a few launches of one GEMM variant for rocprofv3 --pmc passes (KERNEL=prod|lab, BN, M, N, K)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin
dev = torch.device("cuda:0")
lab = ctypes.CDLL(os.path.join(ROOT, "tools/dev/libgemm32.so"))
P = ctypes.c_void_p
M, N, K = (int(os.environ.get(k, d)) for k, d in (("M", "16384"), ("N", "4096"), ("K", "4096")))
BN = int(os.environ.get("BN", "512"))
kern = os.environ.get("KERNEL", "lab")
w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
x = torch.randn(M, K, device=dev, dtype=torch.float16)
y = torch.empty(M, N, device=dev, dtype=torch.float16)
st = P(torch.cuda.current_stream().cuda_stream)
for _ in range(int(os.environ.get("REPS", "6"))):
    if kern == "lab":
        assert lab.lab_gemm32(P(o["qweight"].data_ptr()), P(o["qsz"].data_ptr()), P(x.data_ptr()),
                              P(y.data_ptr()), ctypes.c_int64(M), N, K, 4, 128, BN, st) == 0
    else:
        qlin.gemm(x, o["qweight"], o["qsz"], None, N, K, 4, 128, o["flags"], out=y) if False else \
            qlin.gemm(x, o["qweight"], o["qsz"], None, N, K, 4, 128, o["flags"])
torch.cuda.synchronize()
print("done", kern, M, N, K, BN)
