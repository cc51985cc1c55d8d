"""Full-width parity (north_star: logits within 1e-3 relative of the reference fake-quant path) at
LLaMA3-8B shapes: hidden 4096, intermediate 14336, 32 query / 8 KV heads, vocab 128,256, four
decoder layers (reference models/int_llama_layer.py:103-179 and :213-267, quant/int_linear.py:62).

Three-way comparison.  Every fp16 path is measured against a float64 evaluation of the same layer
mathematics on the same W_dq, KV cache and input (``_ref64_*`` below: no intermediate roundings):
  fake_quant          the reference's path: dense fp16 F.linear on W_dq + the reference's torch glue;
  fake_quant_f32lin   the SAME reference arithmetic with F.linear run on fp32 copies of the fp16
                      operands (another summation order of the same fp32-accumulated products,
                      rounded to fp16 the same way): the order-sensitivity floor of the stack;
  packed              the gfx950 packed linears (QuantLinear packed mode), reference torch glue;
  fused_*             the fused packed layer (fuse_packed_projections) — decode with the KV cache
                      appended in place; prefill with the fused attention kernel.
On random-init stacks an fp16 ulp flip anywhere is amplified layer after layer, so two correct
fp16 paths — the reference against itself with another F.linear order included — differ from each
other by more than 1e-3 of max |logit|.  The criteria are therefore:
  * no packed path is measurably less accurate against fp64 than the reference's own fp16
    arithmetic (err_vs_fp64 <= 1.25 x fake_quant's + 1e-4);
  * its distance to the fake-quant logits stays within the distance between the reference and
    its own reordered twin (<= max(1e-3, 1.5 x floor)).
Numbers are written to $QLIN_PARITY_OUT (profiles/r3_decode_parity.json, r3_prefill_parity.json)."""
import json
import math
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from models.int_llama_layer import _rope_theta  # noqa: E402
from models.quant_llama import (build_random_quant_llama, causal_mask, quant_args,  # noqa: E402
                                rtn_quantize_)
from quant.int_linear import QuantLinear  # noqa: E402
from quant.utils import pack_quant_linears  # noqa: E402

LAYERS = 4
KV = 512


def _cfg():
    from transformers import LlamaConfig
    return LlamaConfig(hidden_size=4096, intermediate_size=14336, num_attention_heads=32,
                       num_key_value_heads=8, num_hidden_layers=LAYERS, vocab_size=128256,
                       max_position_embeddings=8192, rms_norm_eps=1e-5, rope_theta=500000.0)


def _rms64(x, w, eps):
    return w * (x / torch.sqrt((x * x).mean(-1, keepdim=True) + eps))


def _rope64(x, pos, theta):
    """x [..., S, d] (or [..., d] with a scalar pos); pos float64 [S] or a float."""
    d = x.shape[-1]
    inv = 1.0 / (theta ** (torch.arange(0, d, 2, dtype=torch.float64, device=x.device) / d))
    pos = torch.as_tensor(pos, dtype=torch.float64, device=x.device)
    f = pos[..., None] * inv if pos.dim() else pos * inv
    emb = torch.cat((f, f), -1)
    x1, x2 = x[..., : d // 2], x[..., d // 2:]
    return x * emb.cos() + torch.cat((-x2, x1), -1) * emb.sin()


def _mlp64(layer, h, eps):
    mlp = layer.mlp
    y = _rms64(h, layer.post_attention_layernorm.weight.double(), eps)
    g, u = y @ mlp.gate_proj.weight.double().T, y @ mlp.up_proj.weight.double().T
    return h + (g * torch.sigmoid(g) * u) @ mlp.down_proj.weight.double().T


def _ref64_decode(layer, h, past, pos, cfg):
    """One decode step of QuantLlamaDecoderLayer in float64 on the layer's W_dq (exact math)."""
    at = layer.self_attn
    W = lambda lin: lin.weight.double()  # noqa: E731  (fake-quant state: weight == W_dq)
    eps = cfg.rms_norm_eps
    H, Hkv = cfg.num_attention_heads, cfg.num_key_value_heads
    D = cfg.hidden_size // H
    x = _rms64(h, layer.input_layernorm.weight.double(), eps)
    q = (x @ W(at.q_proj).T).view(H, D)
    k = (x @ W(at.k_proj).T).view(Hkv, D)
    v = (x @ W(at.v_proj).T).view(Hkv, D)
    q, k = _rope64(q, pos, _rope_theta(cfg)), _rope64(k, pos, _rope_theta(cfg))
    K = torch.cat([past[0][0].double(), k[:, None]], 1)  # [Hkv, L, D]
    V = torch.cat([past[1][0].double(), v[:, None]], 1)
    Kq = K.repeat_interleave(H // Hkv, 0)
    Vq = V.repeat_interleave(H // Hkv, 0)
    s = torch.einsum("hd,hld->hl", q, Kq) / math.sqrt(D)
    a = torch.einsum("hl,hld->hd", torch.softmax(s, -1), Vq).reshape(-1)
    return _mlp64(layer, h + a @ W(at.o_proj).T, eps)


def _ref64_window(layer, h, cfg):
    """One causal window [S, H] through QuantLlamaDecoderLayer in float64 (positions 0..S-1)."""
    at = layer.self_attn
    W = lambda lin: lin.weight.double()  # noqa: E731
    eps = cfg.rms_norm_eps
    H, Hkv = cfg.num_attention_heads, cfg.num_key_value_heads
    D = cfg.hidden_size // H
    S = h.shape[0]
    x = _rms64(h, layer.input_layernorm.weight.double(), eps)
    q = (x @ W(at.q_proj).T).view(S, H, D).transpose(0, 1)      # [H, S, D]
    k = (x @ W(at.k_proj).T).view(S, Hkv, D).transpose(0, 1)
    v = (x @ W(at.v_proj).T).view(S, Hkv, D).transpose(0, 1)
    pos = torch.arange(S, dtype=torch.float64, device=h.device)
    q, k = _rope64(q, pos, _rope_theta(cfg)), _rope64(k, pos, _rope_theta(cfg))
    k = k.repeat_interleave(H // Hkv, 0)
    v = v.repeat_interleave(H // Hkv, 0)
    s = q @ k.transpose(1, 2) / math.sqrt(D)
    s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=h.device).triu(1), -math.inf)
    a = (torch.softmax(s, -1) @ v).transpose(0, 1).reshape(S, H * D)
    return _mlp64(layer, h + a @ W(at.o_proj).T, eps)


def _rel(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max()).item()


def _f32_linear(x, w, b=None):
    """F.linear on fp32 copies of the fp16 operands, rounded to fp16: the reference arithmetic
    (fp16 products, fp32 accumulation, one rounding) in another summation order."""
    return F.linear(x.float(), w.float(), None if b is None else b.float()).to(x.dtype)


def _reorder_reference(model, on):
    for m in model.modules():
        if isinstance(m, QuantLinear) and not m.packed:
            m.fwd_func = _f32_linear if on else F.linear


def _judge(rep, paths, ref_name="fake_quant", floor_name="fake_quant_f32lin"):
    fq = rep[ref_name]["logits_err_vs_fp64"]
    floor = rep[floor_name]["logits_rel_vs_fake_quant"]
    rep["criteria"] = {"err_vs_fp64_max": 1.25 * fq + 1e-4,
                       "rel_vs_fake_quant_max": max(1e-3, 1.5 * floor),
                       "order_floor": floor}
    out = os.environ.get("QLIN_PARITY_OUT")
    if out:
        with open(out, "w") as f:
            json.dump(rep, f, indent=1)
    print(json.dumps(rep))
    assert fq < 1e-2, rep
    for name in paths:
        if name in (ref_name, floor_name):
            continue
        r = rep[name]
        assert r["logits_err_vs_fp64"] <= rep["criteria"]["err_vs_fp64_max"], (name, rep)
        assert r["logits_rel_vs_fake_quant"] <= rep["criteria"]["rel_vs_fake_quant_max"], (name, rep)


@torch.no_grad()
def test_full_width_decode_three_way():
    cfg = _cfg()
    dev = torch.device("cuda")
    model = build_random_quant_llama(cfg, quant_args(4, 128), seed=21, device=dev,
                                     dtype=torch.float16)
    rtn_quantize_(model)  # fake-quant state: weight == W_dq, dense F.linear (the reference path)
    g = torch.Generator(device=dev).manual_seed(3)
    D = cfg.hidden_size // cfg.num_attention_heads
    past = [(torch.randn(1, cfg.num_key_value_heads, KV, D, device=dev, dtype=torch.float16,
                         generator=g),
             torch.randn(1, cfg.num_key_value_heads, KV, D, device=dev, dtype=torch.float16,
                         generator=g)) for _ in range(LAYERS)]
    x = torch.randn(1, 1, cfg.hidden_size, device=dev, dtype=torch.float16, generator=g)
    mask = torch.zeros(1, 1, 1, KV + 1, device=dev, dtype=torch.float16)
    pos = torch.tensor([[KV]], device=dev)

    h64 = x[0, 0].double()
    for layer, pkv in zip(model.layers, past):
        h64 = _ref64_decode(layer, h64, pkv, float(KV), cfg)
    logits64 = _rms64(h64, model.norm.weight.double(), cfg.rms_norm_eps) @ \
        model.lm_head.weight.double().T

    def run(kv_cache=False):
        h = x
        for i, layer in enumerate(model.layers):
            pkv = past[i]
            if kv_cache:
                pkv = layer.self_attn.adopt_kv_cache(pkv)
            h = layer(h, attention_mask=mask, position_ids=pos, past_key_value=pkv,
                      use_cache=kv_cache)[0]
        return h[0, 0], model.head(h)[0, 0]

    paths = {"fake_quant": run()}
    _reorder_reference(model, True)
    paths["fake_quant_f32lin"] = run()
    _reorder_reference(model, False)
    for layer in model.layers:
        pack_quant_linears(layer)
    paths["packed"] = run()
    for layer in model.layers:
        layer.fuse_packed_projections(kv_cache=True)
    paths["fused_kv_cache"] = run(kv_cache=True)
    from models.decode_engine import DecodeEngine
    eng = DecodeEngine(model.layers)
    if eng.reason is None:
        views = [layer.self_attn.adopt_kv_cache(pkv) for layer, pkv in zip(model.layers, past)]
        h, _ = eng.step(x, pos, views, mask)
        assert eng.status() == 0
        paths["decode_engine"] = (h[0, 0], model.head(h)[0, 0])

    rep = {"layers": LAYERS, "kv_len": KV + 1,
           "shapes": "LLaMA3-8B (4096 / 14336 / 32q 8kv / 128256), int4 g128, batch 1"}
    for name, (h, lg) in paths.items():
        rep[name] = {"logits_err_vs_fp64": _rel(lg, logits64), "hidden_err_vs_fp64": _rel(h, h64),
                     "logits_rel_vs_fake_quant": _rel(lg, paths["fake_quant"][1]),
                     "hidden_rel_vs_fake_quant": _rel(h, paths["fake_quant"][0])}
    _judge(rep, paths)


@torch.no_grad()
def test_full_width_prefill_three_way():
    """A 256-token causal window (positions 0..255) through the same four full-width layers:
    fake-quant, its reordered twin, packed (MFMA GEMM), and packed + fused layer + the fused
    prefill-attention kernel (opt-in mode, DESIGN.md §4 qlin_attn_prefill)."""
    cfg = _cfg()
    dev = torch.device("cuda")
    S = 256
    model = build_random_quant_llama(cfg, quant_args(4, 128), seed=22, device=dev,
                                     dtype=torch.float16)
    rtn_quantize_(model)
    g = torch.Generator(device=dev).manual_seed(4)
    x = torch.randn(1, S, cfg.hidden_size, device=dev, dtype=torch.float16, generator=g)
    mask = causal_mask(1, S, torch.float16, dev)
    pos = torch.arange(S, device=dev)[None]

    h64 = x[0].double()
    for layer in model.layers:
        h64 = _ref64_window(layer, h64, cfg)
    logits64 = _rms64(h64, model.norm.weight.double(), cfg.rms_norm_eps) @ \
        model.lm_head.weight.double().T

    def run():
        h = x
        for layer in model.layers:
            h = layer(h, attention_mask=mask, position_ids=pos)[0]
        return h[0], model.head(h)[0]

    paths = {"fake_quant": run()}
    _reorder_reference(model, True)
    paths["fake_quant_f32lin"] = run()
    _reorder_reference(model, False)
    for layer in model.layers:
        pack_quant_linears(layer)
    paths["packed"] = run()
    for layer in model.layers:
        layer.fuse_packed_projections(prefill_attention=True)
    paths["fused_prefill_attention"] = run()
    rep = {"layers": LAYERS, "window": S,
           "shapes": "LLaMA3-8B (4096 / 14336 / 32q 8kv / 128256), int4 g128, causal window"}
    for name, (h, lg) in paths.items():
        rep[name] = {"logits_err_vs_fp64": _rel(lg, logits64), "hidden_err_vs_fp64": _rel(h, h64),
                     "logits_rel_vs_fake_quant": _rel(lg, paths["fake_quant"][1]),
                     "hidden_rel_vs_fake_quant": _rel(h, paths["fake_quant"][0])}
    _judge(rep, paths)
