#!/usr/bin/env python3
"""Dev: where a decode-engine step spends its time.  Runs the engine (libqlin_gfx950_trace.so,
built with DECODE_TRACE=1: the IO wave stamps 14 events per layer with the 100 MHz wall clock)
on LLaMA3-8B-shaped random layers and prints, per event, the median / max over CUs of the time
since the step's first stamp (us), for the first and a middle layer.  Usage:
  QLIN_LIBRARY=llama3-quantization_amd/csrc/libqlin_gfx950_trace.so python tools/dev/decode_trace.py
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))

import torch  # noqa: E402

from models.decode_engine import DecodeEngine  # noqa: E402
from models.quant_llama import build_random_quant_llama, quant_args, rtn_quantize_  # noqa: E402

EVENTS = ["start", "qkv_staged", "qkv_published", "qkv_done(attn CUs)", "attn_done(attn CUs)",
          "attn_merged", "o_staged", "o_published", "o_done", "gu_staged", "gu_published",
          "gu_done", "dn_staged", "dn_published", "attn: qkv loaded+rope", "attn: new row in LDS",
          "attn: scores", "attn: softmax", "attn: pv", "attn: partial counted",
          "s0: qkv first", "s0: qkv last", "s0: o first", "s0: o last", "s0: gu first",
          "s0: gu last", "s0: dn first", "s0: dn last"]
KEV = len(EVENTS)


def up256(v):
    return (v + 255) // 256 * 256


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--kv", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from transformers import LlamaConfig
    H, I, Hq, Hkv, D = 4096, 14336, 32, 8, 128
    cfg = LlamaConfig(hidden_size=H, intermediate_size=I, num_attention_heads=Hq,
                      num_key_value_heads=Hkv, num_hidden_layers=a.layers, vocab_size=1000,
                      max_position_embeddings=8192, rms_norm_eps=1e-5, rope_theta=500000.0)
    dev = torch.device("cuda:0")
    model = build_random_quant_llama(cfg, quant_args(4, 128), seed=3, device=dev,
                                     dtype=torch.float16)
    rtn_quantize_(model, pack=True)
    g = torch.Generator(device=dev).manual_seed(0)
    past = []
    for layer in model.layers:
        layer.fuse_packed_projections(kv_cache=True)
        kv = (torch.randn(1, Hkv, a.kv, D, device=dev, dtype=torch.float16, generator=g),
              torch.randn(1, Hkv, a.kv, D, device=dev, dtype=torch.float16, generator=g))
        past.append(layer.self_attn.adopt_kv_cache(kv))
    eng = DecodeEngine(model.layers)
    assert eng.reason is None, eng.reason
    x = torch.randn(1, 1, H, device=dev, dtype=torch.float16, generator=g)
    pos = torch.tensor([[a.kv]], device=dev)
    for _ in range(3):
        eng.step(x, pos, past)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(a.reps):
        eng.step(x, pos, past)
    e1.record()
    torch.cuda.synchronize()
    step_us = e0.elapsed_time(e1) * 1e3 / a.reps
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    nl, L = a.layers, a.kv + 1
    S = -(-L // 64)
    grp = Hq // Hkv
    off = up256((1 + nl * (4 * 8 + 1 + Hkv)) * 4)
    off += up256((H + 2 * Hkv * D) * 2) + 3 * up256(H * 2) + up256(I * 2)
    off += up256(Hkv * S * grp * (D + 2) * 4)
    ws = eng._ws
    if ws.numel() < off + nl * KEV * ncu * 8:  # a library built without DECODE_TRACE
        print(json.dumps({"step_us": round(step_us, 2), "per_layer_us": round(step_us / nl, 2),
                          "status": eng.status(), "trace": None}))
        return
    ws[off:off + nl * KEV * ncu * 8].zero_()
    eng.step(x, pos, past)
    torch.cuda.synchronize()
    tr = ws[off:off + nl * KEV * ncu * 8].view(torch.int64).view(nl, KEV, ncu).cpu().double()
    t0 = tr[0, 0].min()
    us = (tr - t0) / 100.0  # 100 MHz -> us
    out = {"step_us": round(step_us, 2), "per_layer_us": round(step_us / nl, 2),
           "status": eng.status()}
    for l in sorted({0, nl // 2, nl - 1}):
        rows = {}
        for e, name in enumerate(EVENTS):
            v = us[l, e]
            v = v[tr[l, e] > 0]
            if v.numel():
                rows[name] = [round(v.median().item(), 2), round(v.max().item(), 2)]
        out[f"layer{l}"] = rows
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
