import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin
dev = torch.device("cuda:0")
N, K, g = 256, 1024, 128
w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
o = qlin.quantize(w, 4, g, 0, want_xdq=False, want_params=False, pack=True)
for M in (1, 2, 3, 4):
    for same in (False, True):
        x = torch.randn(M, K, device=dev, dtype=torch.float16)
        if same:
            x[:] = x[0]
        ye = qlin.gemv(x, o["qweight"], o["qsz"], None, N, K, 4, g, o["flags"])
        yf = qlin.gemv(x, o["qweight"], o["qsz"], None, N, K, 4, g, o["flags"] | qlin.FAST_DEQUANT)
        err = (ye.float() - yf.float()).abs().amax(dim=1)
        print(f"M={M} same={same}: per-row max|exact-fast| = {err.tolist()}  max|y|={ye.abs().max().item():.3f}")
        if M > 1 and not same:
            # does row i of fast equal exact row j for some j? (row mixing)
            for i in range(M):
                d = [(ye[j].float() - yf[i].float()).abs().max().item() for j in range(M)]
                print("   fast row", i, "vs exact rows:", [f"{v:.3g}" for v in d])
