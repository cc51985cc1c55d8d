"""Run a few eager GEMV launches (for rocprofv3 counter collection)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin
dev = torch.device("cuda:0")
N = K = 4096
R = 16
mats = []
for i in range(R):
    w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
    o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
    mats.append((o["qweight"], o["qsz"], o["flags"]))
x = torch.randn(1, K, device=dev, dtype=torch.float16)
for it in range(3):
    for m in mats:
        y = qlin.gemv(x, m[0], m[1], None, N, K, 4, 128, m[2])
torch.cuda.synchronize()
print("done")
