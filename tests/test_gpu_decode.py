"""Full-width decode parity (north_star: logits within 1e-3 relative of the reference fake-quant
path), at LLaMA3-8B shapes: hidden 4096, intermediate 14336, 32 query / 8 KV heads, vocab 128,256,
four decoder layers, one new token over a 512-row KV cache (reference models/int_llama_layer.py:
103-179 and :213-267, quant/int_linear.py:62).

Three-way comparison.  Every fp16 path (the reference's fake-quant path = dense F.linear on W_dq
with the reference's torch glue; the packed gfx950 path; the fused packed layer with the KV cache
appended in place) is measured against a float64 evaluation of the same layer mathematics on the
same W_dq, KV cache and input (``_ref64`` below: no intermediate roundings).  On random-init
stacks an fp16 ulp flip anywhere is amplified layer after layer, so two correct fp16 paths can
differ from each other by more than their own error; the criterion is that no packed path is
measurably less accurate than the reference arithmetic it replaces, and the pairwise distance to
the fake-quant path is reported beside it (profiles/r3_decode_parity.json)."""
import json
import math
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

from models.int_llama_layer import _rope_theta  # noqa: E402
from models.quant_llama import build_random_quant_llama, quant_args, rtn_quantize_  # noqa: E402
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
    d = x.shape[-1]
    inv = 1.0 / (theta ** (torch.arange(0, d, 2, dtype=torch.float64, device=x.device) / d))
    f = pos * inv
    emb = torch.cat((f, f))
    x1, x2 = x[..., : d // 2], x[..., d // 2:]
    return x * emb.cos() + torch.cat((-x2, x1), -1) * emb.sin()


def _ref64_layer(layer, h, past, pos, cfg):
    """One decode step of QuantLlamaDecoderLayer in float64 on the layer's W_dq (exact math)."""
    at, mlp = layer.self_attn, layer.mlp
    W = lambda lin: lin.weight.double()  # noqa: E731  (fake-quant state: weight == W_dq)
    eps = cfg.rms_norm_eps
    H, Hkv, D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.hidden_size // cfg.num_attention_heads
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
    h = h + a @ W(at.o_proj).T
    y = _rms64(h, layer.post_attention_layernorm.weight.double(), eps)
    g, u = y @ W(mlp.gate_proj).T, y @ W(mlp.up_proj).T
    return h + (g * torch.sigmoid(g) * u) @ W(mlp.down_proj).T


def _rel(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max()).item()


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

    # float64 evaluation of the same stack (W_dq, cache, input), logits through norm + lm_head
    h64 = x[0, 0].double()
    for layer, pkv in zip(model.layers, past):
        h64 = _ref64_layer(layer, h64, pkv, float(KV), cfg)
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

    paths = {}
    paths["fake_quant"] = run()
    for layer in model.layers:
        pack_quant_linears(layer)
    paths["packed"] = run()
    for layer in model.layers:
        layer.fuse_packed_projections(kv_cache=True)
    paths["fused_kv_cache"] = run(kv_cache=True)

    rep = {"layers": LAYERS, "kv_len": KV, "shapes": "LLaMA3-8B (4096 / 14336 / 32q 8kv / 128256)"}
    for name, (h, lg) in paths.items():
        rep[name] = {"logits_err_vs_fp64": _rel(lg, logits64), "hidden_err_vs_fp64": _rel(h, h64),
                     "logits_rel_vs_fake_quant": _rel(lg, paths["fake_quant"][1]),
                     "hidden_rel_vs_fake_quant": _rel(h, paths["fake_quant"][0])}
    out = os.environ.get("QLIN_PARITY_OUT")
    if out:
        with open(out, "w") as f:
            json.dump(rep, f, indent=1)
    print(json.dumps(rep))
    fq = rep["fake_quant"]["logits_err_vs_fp64"]
    assert fq < 1e-2, rep
    for name in paths:
        if name == "fake_quant":
            continue
        r = rep[name]
        # no packed path is measurably less accurate than the reference's own fp16 arithmetic
        assert r["logits_err_vs_fp64"] <= 1.25 * fq + 1e-4, (name, rep)
        # and it stays within the north-star distance of the fake-quant logits
        assert r["logits_rel_vs_fake_quant"] < 1e-3, (name, rep)
