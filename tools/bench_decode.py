#!/usr/bin/env python3
"""Decode-step timing of one LLaMA3-8B-shaped QuantLlamaDecoderLayer (hidden 4096, inter 14336,
32 heads / 8 KV heads), RTN int4 g128 packed, batch 1, one new token over a KV cache of L tokens:
dense fake-quant (F.linear on W_dq, the reference eval path) vs packed, unfused vs fused q/k/v +
gate/up.  Random weights; per-layer time from HIP events over graph replays of R distinct layers
(weights beyond the 256 MB MALL).  Prints one JSON line."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))

import torch  # noqa: E402

from models.quant_llama import (causal_mask, quant_args, random_llama_layer,  # noqa: E402
                                rtn_quantize_)
from models.int_llama_layer import QuantLlamaDecoderLayer  # noqa: E402
from quant.utils import pack_quant_linears  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--kv", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from transformers import LlamaConfig
    cfg = LlamaConfig(hidden_size=4096, intermediate_size=14336, num_attention_heads=32,
                      num_key_value_heads=8, num_hidden_layers=a.layers, vocab_size=128256,
                      max_position_embeddings=8192, rms_norm_eps=1e-5, rope_theta=500000.0)
    dev = torch.device("cuda:0")
    args = quant_args(4, 128)
    layers = [QuantLlamaDecoderLayer(cfg, random_llama_layer(cfg, 100 + i, dev, torch.float16), args)
              for i in range(a.layers)]

    class Stack(torch.nn.Module):
        def __init__(self, ls):
            super().__init__()
            self.layers = torch.nn.ModuleList(ls)
    st = Stack(layers)
    rtn_quantize_(st)  # fake-quant state (weight = W_dq)
    hd = cfg.hidden_size // cfg.num_attention_heads
    g = torch.Generator(device=dev).manual_seed(0)
    past = [(torch.randn(1, cfg.num_key_value_heads, a.kv, hd, device=dev, dtype=torch.float16, generator=g),
             torch.randn(1, cfg.num_key_value_heads, a.kv, hd, device=dev, dtype=torch.float16, generator=g))
            for _ in range(a.layers)]
    x = torch.randn(1, 1, cfg.hidden_size, device=dev, dtype=torch.float16, generator=g)
    mask = torch.zeros(1, 1, 1, a.kv + 1, device=dev, dtype=torch.float16)
    pos = torch.tensor([[a.kv]], device=dev)

    cache = {"use": False}

    def step():
        h = x
        for layer, pkv in zip(st.layers, past):
            h = layer(h, attention_mask=mask, position_ids=pos, past_key_value=pkv,
                      use_cache=cache["use"])[0]
        return h

    def timed():
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s), torch.no_grad():
            step()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s), torch.no_grad():  # capture on the warm-up stream
            out = step()
        torch.cuda.current_stream().wait_stream(s)
        for _ in range(3):
            gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(a.reps):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.reps / a.layers, out.clone()

    res = {}
    res["fake_quant_dense_us"], y_fq = timed()
    for layer in st.layers:
        pack_quant_linears(layer)
    res["packed_us"], y_pk = timed()
    for layer in st.layers:
        layer.fuse_packed_projections()
    res["packed_fused_us"], y_fu = timed()
    # + the KV append into preallocated caches (kv_cache mode: RoPE writes the new k / v rows in
    # place of the reference's two torch.cat copies of the cache)
    for i, layer in enumerate(st.layers):
        layer.fuse_packed_projections(kv_cache=True)
        past[i] = layer.self_attn.adopt_kv_cache(past[i])
    cache["use"] = True
    res["packed_fused_kv_cache_us"], y_kv = timed()
    params = sum(m.in_features * m.out_features for l in st.layers for m in l.modules()
                 if hasattr(m, "qweight") and m.__class__.__name__ == "QuantLinear") / a.layers
    wbytes = params * 0.5 + params / 128 * 3
    out = {"what": "LLaMA3-8B-shaped decoder layer decode step, int4 g128, batch 1",
           "kv_len": a.kv, "layers_timed": a.layers, "weight_bytes_per_layer": int(wbytes),
           **{k: (round(v, 2) if isinstance(v, float) and "err" not in k else v)
              for k, v in res.items()},
           "fused_weight_GBps": round(wbytes / res["packed_fused_us"] / 1e3, 1),
           "rel_err_packed_vs_fake_quant": float((y_pk.float() - y_fq.float()).abs().max()
                                                 / y_fq.float().abs().max()),
           # fused = fused projections (bit-identical) + fused decode attention (fp32 summation
           # order differs from the bmm), so the comparison is a relative error, not equality
           "rel_err_fused_vs_unfused": float((y_fu.float() - y_pk.float()).abs().max()
                                             / y_pk.float().abs().max()),
           "fused_kv_cache_weight_GBps": round(wbytes / res["packed_fused_kv_cache_us"] / 1e3, 1),
           "kv_cache_equal_to_cat": bool(torch.equal(y_kv, y_fu)),
           "est_32_layer_token_ms": round(res["packed_fused_us"] * 32 / 1e3, 3),
           "est_32_layer_token_ms_kv_cache": round(res["packed_fused_kv_cache_us"] * 32 / 1e3, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
