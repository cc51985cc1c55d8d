#!/usr/bin/env python3
"""Dev: recover the summation order of F.linear (hipBLASLt fp16, fp32 accumulation) at decode
sizes (M = 1), so the packed GEMV can reproduce the reference fake-quant path bit for bit.

Model of one v_mfma_f32_16x16x{KS}_f16 step: acc = fp32(acc + sum of KS exact products) (products
of fp16 are exact; the KS-term sum taken in fp64, one rounding when added).  Validated first on our
own k-ordered MFMA chain (qlin.gemv_batched, 16x16x32), then hypotheses for hipBLASLt's kernels
(MT16x16x256 / MT64x16x256 / MT16x16x512, WG16_4_4: LocalSplitU = 4) are scored by the fraction of
outputs bit-equal to F.linear.  Prints one JSON line per shape."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from quant import qlin  # noqa: E402


def steps(x, w, ks):
    """[N, K/ks] fp64 exact-ish partial dots of ks consecutive k."""
    N, K = w.shape
    p = w.double() * x.double()[None, :]
    return p.view(N, K // ks, ks).sum(-1)


def chain(d, order):
    acc = torch.zeros(d.shape[0], dtype=torch.float32, device=d.device)
    for s in order:
        acc = (acc.double() + d[:, s]).float()
    return acc


def lsu(d, depth_steps, lsu_n, assign, reduce="seq"):
    """LocalSplitU: per iteration of depth_steps MFMA steps, wave w takes the steps assign(w);
    each wave's chain runs over the iterations in order; partials reduced per `reduce`."""
    n_it = d.shape[1] // depth_steps
    parts = []
    for w in range(lsu_n):
        order = [it * depth_steps + s for it in range(n_it) for s in assign(w)]
        parts.append(chain(d, order))
    if reduce == "seq":
        acc = parts[0]
        for p in parts[1:]:
            acc = acc + p
    elif reduce == "rev":
        acc = parts[-1]
        for p in reversed(parts[:-1]):
            acc = acc + p
    else:  # pairwise
        acc = (parts[0] + parts[1]) + (parts[2] + parts[3])
    return acc


def eq(a, ref):
    return round((a.half() == ref).float().mean().item(), 5)


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for (N, K) in [(4096, 4096), (1024, 4096), (14336, 4096), (28672, 4096), (4096, 14336)]:
        w = torch.empty(N, K, device=dev, dtype=torch.float16).normal_(0, 0.02, generator=g)
        o = qlin.quantize(w, 4, 128, 0, pack=True)
        wdq = o["x_dq"]
        x = torch.empty(1, K, device=dev, dtype=torch.float16).normal_(0, 1, generator=g)
        ref = F.linear(x, wdq)[0]
        ours_chain = qlin.gemv_batched(x, o["qweight"][None], o["qsz"][None], None, N, K, 4, 128,
                                       o["flags"])[0][0]
        out = {"N": N, "K": K}
        for ks in (32, 16):
            d = steps(x[0], wdq, ks)
            ns = d.shape[1]
            c = chain(d, range(ns))
            out[f"emu_chain{ks}_vs_ours_chain"] = eq(c, ours_chain)
            out[f"emu_chain{ks}_vs_flinear"] = eq(c, ref)
            for du in (256, 512):
                dst = du // ks  # MFMA steps per iteration
                per = dst // 4
                hyps = {
                    "contig": lambda w_, per=per: range(w_ * per, (w_ + 1) * per),
                    "strided": lambda w_, per=per: range(w_, 4 * per, 4),
                }
                for hn, asg in hyps.items():
                    for red in ("seq", "rev", "pair"):
                        out[f"lsu4_du{du}_k{ks}_{hn}_{red}"] = eq(lsu(d, dst, 4, asg, red), ref)
        best = max((v, k) for k, v in out.items() if k.startswith("lsu4") or k.endswith("flinear"))
        out["best"] = best
        print(json.dumps(out), flush=True)
        del w, o, wdq


if __name__ == "__main__":
    main()
