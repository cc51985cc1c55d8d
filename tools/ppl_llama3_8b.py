#!/usr/bin/env python3
"""Full-size LLaMA3-8B-architecture perplexity parity and eval-window timing (BASELINE metric's
"LLaMA3-8B PPL delta"; main.py:102-154 evaluate loop).

There are no checkpoints or datasets offline, so the model is random-init (N(0, 0.02^2) linears,
N(0, 1) embeddings) with the exact LLaMA3-8B shapes (32 layers, hidden 4096, inter 14336, 32/8
heads, vocab 128,256) and the "text" is seeded random tokens.  RTN int4 g128 exactly as
omniquant() with epochs == 0, then:
  fake-quant: the reference's eval path (weight = W_dq, dense fp16 F.linear);
  packed:     the same layers after pack_quant_linears (gfx950 dequant-GEMM kernels), optionally
              with fused q/k/v + gate/up launches, and then also the fused prefill-attention
              kernel (fp32, online softmax: equal to the reference attention to fp32 rounding).
Reports PPL of both, their relative delta, the max relative logit difference on the first
window, and ms per 2048-token window (HIP events, after one warm-up window).  Prints one JSON line.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))

import torch  # noqa: E402

from models.quant_llama import (build_random_quant_llama, nll_from_logits, quant_args,  # noqa: E402
                                rtn_quantize_)
from quant.utils import pack_quant_linears  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--windows", type=int, default=3)
    ap.add_argument("--seqlen", type=int, default=2048)
    ap.add_argument("--wbits", type=int, default=4)
    ap.add_argument("--group", type=int, default=128)
    a = ap.parse_args()
    from transformers import LlamaConfig
    cfg = LlamaConfig(hidden_size=4096, intermediate_size=14336, num_attention_heads=32,
                      num_key_value_heads=8, num_hidden_layers=a.layers, vocab_size=128256,
                      max_position_embeddings=8192, rms_norm_eps=1e-5, rope_theta=500000.0)
    dev = torch.device("cuda:0")
    t0 = time.time()
    model = build_random_quant_llama(cfg, quant_args(a.wbits, a.group), seed=3, device=dev,
                                     dtype=torch.float16)
    rtn_quantize_(model)
    print(f"built + RTN-quantized {a.layers} layers in {time.time() - t0:.1f}s", file=sys.stderr,
          flush=True)
    g = torch.Generator(device=dev).manual_seed(2024)
    testenc = torch.randint(0, cfg.vocab_size, (1, a.windows * a.seqlen), device=dev, generator=g)

    @torch.no_grad()
    def run(tag):
        nlls, first = [], None
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        ms = []
        for i in range(a.windows):
            batch = testenc[:, i * a.seqlen:(i + 1) * a.seqlen]
            torch.cuda.synchronize()
            e0.record()
            logits = model(batch)
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
            nlls.append(nll_from_logits(logits, batch))
            if i == 0:
                first = logits[0, :256].float().clone()
            del logits
        ppl = torch.exp(torch.stack(nlls).sum() / (a.windows * a.seqlen)).item()
        print(f"{tag}: ppl {ppl:.6f}, ms/window {ms}", file=sys.stderr, flush=True)
        return ppl, first, (sum(ms[1:]) / max(1, len(ms) - 1)) if len(ms) > 1 else ms[0]

    ppl_fq, lg_fq, ms_fq = run("fake-quant (dense F.linear on W_dq)")
    for layer in model.layers:
        pack_quant_linears(layer)
    torch.cuda.empty_cache()
    ppl_pk, lg_pk, ms_pk = run("packed")
    for layer in model.layers:
        layer.fuse_packed_projections()
    ppl_fu, lg_fu, ms_fu = run("packed + fused projections")
    for layer in model.layers:
        layer.fuse_packed_projections(prefill_attention=True)
    ppl_fa, lg_fa, ms_fa = run("packed + fused projections + fused prefill attention")
    rel = lambda x, y: ((x.double() - y.double()).abs().max() / y.double().abs().max()).item()
    out = {
        "what": "LLaMA3-8B-architecture (random init) PPL parity, packed vs fake-quant",
        "layers": a.layers, "windows": a.windows, "seqlen": a.seqlen,
        "wbits": a.wbits, "group": a.group, "data": "synthetic tokens, random-init weights",
        "ppl_fake_quant": ppl_fq, "ppl_packed": ppl_pk, "ppl_packed_fused": ppl_fu,
        "ppl_rel_delta": abs(ppl_pk - ppl_fq) / ppl_fq,
        "ppl_rel_delta_fused": abs(ppl_fu - ppl_fq) / ppl_fq,
        "nll_per_token_delta": abs(math.log(ppl_pk) - math.log(ppl_fq)),
        "logits_rel_err_packed": rel(lg_pk, lg_fq),
        "logits_rel_err_fused": rel(lg_fu, lg_fq),
        "ms_per_window_fake_quant": round(ms_fq, 2), "ms_per_window_packed": round(ms_pk, 2),
        "ms_per_window_packed_fused": round(ms_fu, 2),
        "ppl_packed_fused_attn": ppl_fa,
        "ppl_rel_delta_fused_attn": abs(ppl_fa - ppl_fq) / ppl_fq,
        "logits_rel_err_fused_attn": rel(lg_fa, lg_fq),
        "ms_per_window_packed_fused_attn": round(ms_fa, 2),
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
