#!/usr/bin/env python3
"""Which summation order does F.linear (hipBLASLt / rocBLAS fp16) use at decode sizes?

For LLaMA3-8B decode shapes and M = 1, 2, 4: the fraction of outputs of each packed kernel that
are bit-equal to F.linear(x, W_dq), and each path's error against a float64 product.  Prints one
JSON line per case."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from quant import qlin  # noqa: E402


def stats(y, ref, y64):
    m = y64.abs().max().item()
    return {"eq_flinear": round((y == ref).float().mean().item(), 4),
            "err64_max": (y.double() - y64).abs().max().item() / m,
            "err64_mean": (y.double() - y64).abs().mean().item() / m}


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for (N, K) in [(4096, 4096), (6144, 4096), (28672, 4096), (4096, 14336)]:
        w = torch.empty(N, K, device=dev, dtype=torch.float16).normal_(0, 0.02, generator=g)
        o = qlin.quantize(w, 4, 128, 0, pack=True)
        wdq = o["x_dq"]
        for M in (1, 2, 4):
            x = torch.empty(M, K, device=dev, dtype=torch.float16).normal_(0, 1, generator=g)
            ref = F.linear(x, wdq)
            ref3 = F.linear(x[None], wdq)[0]
            y64 = x.double() @ wdq.double().T
            out = {"N": N, "K": K, "M": M, "flinear3d_eq_2d": bool(torch.equal(ref, ref3)),
                   "flinear": stats(ref, ref, y64)}
            out["fast"] = stats(qlin.gemv(x, o["qweight"], o["qsz"], None, N, K, 4, 128,
                                          o["flags"]), ref, y64)
            out["chain"] = stats(qlin.gemv_batched(x, o["qweight"][None], o["qsz"][None], None,
                                                   N, K, 4, 128, o["flags"])[0], ref, y64)
            out["gemm_nosplit"] = stats(qlin.gemm(x, o["qweight"], o["qsz"], None, N, K, 4, 128,
                                                  o["flags"], split=False), ref, y64)
            # fp32 F.linear on the same fp16 operands, rounded once (an order-free reference)
            out["fp32_flinear"] = stats(F.linear(x.float(), wdq.float()).half(), ref, y64)
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
