import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin
dev = torch.device("cuda:0")
for (N, K, g) in ((64, 32, 32), (64, 64, 32), (64, 96, 32), (64, 160, 32), (64, 256, 128), (64, 128, 128)):
    w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
    o = qlin.quantize(w, 4, g, 0, want_xdq=False, want_params=False, pack=True)
    wdq = qlin.dequant(o["qweight"], o["qsz"], N, K, 4, g, o["flags"]).float()
    bad = []
    for M in range(1, 17):
        x = torch.randn(M, K, device=dev, dtype=torch.float16)
        y = qlin.gemv(x, o["qweight"], o["qsz"], None, N, K, 4, g, o["flags"]).float()
        ref = x.float() @ wdq.t()
        err = (y - ref).abs().amax(dim=1) / ref.abs().max()
        rows = [i for i in range(M) if err[i] > 3e-3]
        if rows:
            bad.append((M, rows))
    print(N, K, g, "bad (M, rows):", bad)
