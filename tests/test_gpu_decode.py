"""Full-width parity (north_star: logits within 1e-3 relative of the reference fake-quant path) at
LLaMA3-8B shapes: hidden 4096, intermediate 14336, 32 query / 8 KV heads, vocab 128,256
(reference models/int_llama_layer.py:103-179 and :213-267, quant/int_linear.py:62,
quant/omni_norm.py:52-63).

Every fp16 path runs the same random-init stack on the same W_dq, KV cache and input:
  fake_quant          the reference's path: dense fp16 F.linear on W_dq + the reference's torch glue;
  fake_quant_f32lin   the SAME reference arithmetic with F.linear run on fp32 copies of the fp16
                      operands (the same fp32-accumulated products in another summation order,
                      rounded to fp16 the same way): the reference against itself, the order floor;
  packed              the gfx950 packed linears (QuantLinear packed mode), reference torch glue;
  fused_*             the fused packed layer (fuse_packed_projections) — decode with the KV cache
                      appended in place (RMSNorm inside the q/k/v and gate/up launches, attention +
                      RoPE + append in one launch, residual / SiLU epilogues); prefill with the
                      fused prefill-attention kernel.
Logits are formed from each path's final hidden state by a float64 head (the model's RMSNorm and
lm_head in fp64), so fp16 rounding of the logits themselves does not dominate the comparison, and
are compared with the fake-quant path's: max |diff| / max |logit| (``max``), the 99th percentile
of |diff| / max |logit| (``p99``) and top-1 agreement.  A float64 evaluation of the same layer
mathematics (no intermediate roundings) anchors accuracy.

On random-init stacks an fp16 ulp flip anywhere is amplified layer after layer: the reference
differs from its own reordered twins by more than 1e-3 of max |logit|.  The twins run the SAME
reference arithmetic (fp16 products of the same W_dq and activations, one fp16 rounding of every
linear output) with only the summation order of F.linear changed:
  fake_quant_f32lin   F.linear on fp32 copies (hipBLASLt's fp32 kernel order);
  fake_quant_ksplit   the same in two K halves added in fp32 (another association);
  fake_quant_f64acc   the sum accumulated in float64 (the exactly rounded order).
The order floor is the largest distance of a twin to the fake-quant logits (each twin's own
distance is reported beside it, and every path's ratio to the single hipBLASLt twin
``fake_quant_f32lin`` too).

The bar (declared before these runs), over >= 8 seeds per
4-layer case (4 seeds for the 32-layer window), for every packed / fused path:
  * ratio of its max logit distance to the max-of-twins floor: median <= 1.0, max <= 1.1;
  * ratio of its float64 error to the reference's own float64 error: median <= 1.05.
The p99 ratios are reported beside them.  Numbers are written to $QLIN_PARITY_OUT*
(profiles/r6_decode_parity.json, r6_prefill_parity.json, r6_prefill32_parity.json)."""
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
SEEDS = (21, 31, 41, 51, 61, 71, 81, 91)
SEEDS32 = (21, 31, 41, 51)
BAR_MAX = 1.1         # max over seeds of the max-distance ratio to the max-of-twins floor
BAR_MEDIAN = 1.0      # median over seeds of that ratio
BAR_FP64_MEDIAN = 1.05  # median over seeds of (float64 error / the reference's own)


def _cfg(layers=LAYERS):
    from transformers import LlamaConfig
    return LlamaConfig(hidden_size=4096, intermediate_size=14336, num_attention_heads=32,
                       num_key_value_heads=8, num_hidden_layers=layers, vocab_size=128256,
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


def _head64(model, h, cfg):
    """The model's RMSNorm + lm_head in float64 on a final hidden state."""
    return _rms64(h.double(), model.norm.weight.double(), cfg.rms_norm_eps) @ \
        model.lm_head.weight.double().T


def _stats(lg, ref):
    """max / p99 of |lg - ref| relative to max |ref|, and top-1 agreement (fraction of rows)."""
    d = (lg - ref).abs().reshape(-1)
    scale = ref.abs().max()
    k = max(1, int(math.ceil(0.99 * d.numel())))
    p99 = d.float().kthvalue(k).values.double() if d.numel() > 1 else d.max()
    top1 = (lg.reshape(-1, lg.shape[-1]).argmax(-1) == ref.reshape(-1, ref.shape[-1]).argmax(-1))
    return {"max": (d.max() / scale).item(), "p99": (p99 / scale).item(),
            "top1": top1.double().mean().item()}


def _f32_linear(x, w, b=None):
    """F.linear on fp32 copies of the fp16 operands, rounded to fp16: the reference arithmetic
    (fp16 products, fp32 accumulation, one rounding) in another summation order."""
    return F.linear(x.float(), w.float(), None if b is None else b.float()).to(x.dtype)


def _ksplit_linear(x, w, b=None):
    """The same with K summed as two halves added in fp32 (another association)."""
    h = x.shape[-1] // 2
    y = F.linear(x[..., :h].float(), w[:, :h].float()) + F.linear(x[..., h:].float(), w[:, h:].float())
    return (y if b is None else y + b.float()).to(x.dtype)


def _f64acc_linear(x, w, b=None):
    """The same accumulated in float64 (the exactly rounded sum of the fp16 products)."""
    return F.linear(x.double(), w.double(), None if b is None else b.double()).to(x.dtype)


TWINS = {"fake_quant_f32lin": _f32_linear, "fake_quant_ksplit": _ksplit_linear,
         "fake_quant_f64acc": _f64acc_linear}


def _reorder_reference(model, fn):
    for m in model.modules():
        if isinstance(m, QuantLinear) and not m.packed:
            m.fwd_func = fn


def _progress(*a):
    print("[parity]", *a, flush=True)  # a long full-width case shows it is alive


def _report(seed, paths, model, cfg, ref64_h):
    logits64 = _head64(model, ref64_h, cfg)
    ref = _head64(model, paths["fake_quant"], cfg)
    rep = {"seed": seed}
    for name, h in paths.items():
        lg = _head64(model, h, cfg)
        r = {"logits_err_vs_fp64": _stats(lg, logits64)["max"],
             "hidden_err_vs_fp64": ((h.double() - ref64_h).abs().max()
                                    / ref64_h.abs().max()).item()}
        r.update({f"logits_{k}_vs_fake_quant": v for k, v in _stats(lg, ref).items()})
        r["hidden_rel_vs_fake_quant"] = ((h.double() - paths["fake_quant"].double()).abs().max()
                                         / paths["fake_quant"].double().abs().max()).item()
        rep[name] = r
    return rep


def _judge(reps, ref_name="fake_quant", out_env=None, known_misses=()):
    """Per path, over the seeds: the ratio of its max (and p99) logit distance to the fake-quant
    logits against the max-of-twins order floor and against the single hipBLASLt twin, and of
    its float64 error against the reference's own; the bar (module docstring) on the median and
    max of those ratios."""
    import statistics
    ratios = {}
    for rep in reps:
        fq = rep[ref_name]
        fmax = max(rep[t]["logits_max_vs_fake_quant"] for t in TWINS)
        fp99 = max(rep[t]["logits_p99_vs_fake_quant"] for t in TWINS)
        rep["criteria"] = {"order_floor_max": fmax, "order_floor_p99": fp99,
                           "reference_fp64_err": fq["logits_err_vs_fp64"],
                           "order_floor_twins_max": {t: rep[t]["logits_max_vs_fake_quant"]
                                                     for t in TWINS}}
        for name, r in rep.items():
            if name in (ref_name, "criteria", "seed") or name in TWINS or not isinstance(r, dict):
                continue
            r["ratio_max_to_floor"] = r["logits_max_vs_fake_quant"] / fmax
            r["ratio_p99_to_floor"] = r["logits_p99_vs_fake_quant"] / fp99
            r["ratio_max_to_f32lin_twin"] = (r["logits_max_vs_fake_quant"] /
                                             rep["fake_quant_f32lin"]["logits_max_vs_fake_quant"])
            r["ratio_fp64_to_reference"] = r["logits_err_vs_fp64"] / fq["logits_err_vs_fp64"]
            ratios.setdefault(name, []).append(r)
    summary, failures = {}, []
    for name, rs_ in ratios.items():
        col = lambda k: [r[k] for r in rs_]  # noqa: E731
        sm = {k: {"median": statistics.median(col(k)), "max": max(col(k)), "min": min(col(k))}
              for k in ("ratio_max_to_floor", "ratio_p99_to_floor", "ratio_max_to_f32lin_twin",
                        "ratio_fp64_to_reference")}
        sm["top1_min"] = min(col("logits_top1_vs_fake_quant"))
        summary[name] = sm
        if sm["ratio_max_to_floor"]["median"] > BAR_MEDIAN:
            failures.append((name, "median ratio_max_to_floor", sm["ratio_max_to_floor"]["median"]))
        if sm["ratio_max_to_floor"]["max"] > BAR_MAX:
            failures.append((name, "max ratio_max_to_floor", sm["ratio_max_to_floor"]["max"]))
        if sm["ratio_fp64_to_reference"]["median"] > BAR_FP64_MEDIAN:
            failures.append((name, "median ratio_fp64_to_reference",
                             sm["ratio_fp64_to_reference"]["median"]))
    missed = [f for f in failures if (f[0], f[1]) in known_misses]
    failures = [f for f in failures if (f[0], f[1]) not in known_misses]
    doc = {"bar": {"ratio_max_to_floor": f"median <= {BAR_MEDIAN}, max <= {BAR_MAX}",
                   "ratio_fp64_to_reference": f"median <= {BAR_FP64_MEDIAN}",
                   "declared": "before the runs (VERDICT r4 item 2; DESIGN.md §2)"},
           "n_seeds": len(reps), "summary": summary, "failures": failures,
           "known_misses": missed, "seeds": reps}
    out = os.environ.get(out_env or "QLIN_PARITY_OUT")
    if out:
        with open(out, "w") as f:
            json.dump(doc, f, indent=1)
    print(json.dumps({"summary": summary, "failures": failures, "known_misses": missed}))
    for rep in reps:
        assert rep[ref_name]["logits_err_vs_fp64"] < 1e-2, rep
    assert not failures, failures


def _decode_seed(seed):
    cfg = _cfg()
    dev = torch.device("cuda")
    model = build_random_quant_llama(cfg, quant_args(4, 128), seed=seed, device=dev,
                                     dtype=torch.float16)
    rtn_quantize_(model)  # fake-quant state: weight == W_dq, dense F.linear (the reference path)
    g = torch.Generator(device=dev).manual_seed(seed + 1)
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

    def run(kv_cache=False):
        h = x
        for i, layer in enumerate(model.layers):
            pkv = past[i]
            if kv_cache:
                pkv = layer.self_attn.adopt_kv_cache(pkv)
            h = layer(h, attention_mask=mask, position_ids=pos, past_key_value=pkv,
                      use_cache=kv_cache)[0]
        return h[0, 0]

    def run_dyn_len():
        """The device-length launches generate(graphs=True) captures and replays: the cache
        length read from a device tensor, the attention grid sized for a generation 64 tokens
        longer, no host-side mask / past (models/pipeline.py _layers_step_len)."""
        h = x
        length = torch.tensor([KV + 1], dtype=torch.int32, device=dev)
        for i, layer in enumerate(model.layers):
            at = layer.self_attn
            at.adopt_kv_cache(past[i], rows=KV + 65)
            at._dyn_len, at._dyn_max = length, KV + 65
            try:
                h = layer(h, attention_mask=None, position_ids=pos, past_key_value=None,
                          use_cache=False)[0]
            finally:
                at._dyn_len = at._dyn_max = None
        return h[0, 0]

    paths = {"fake_quant": run()}
    for name, fn in TWINS.items():
        _reorder_reference(model, fn)
        paths[name] = run()
    _reorder_reference(model, F.linear)
    for layer in model.layers:
        pack_quant_linears(layer)
    paths["packed"] = run()
    for layer in model.layers:
        layer.fuse_packed_projections(kv_cache=True)
    paths["fused_kv_cache"] = run(kv_cache=True)
    paths["fused_device_len"] = run_dyn_len()
    _progress("decode seed", seed, "paths done")
    rep = _report(seed, paths, model, cfg, h64)
    rep.update(layers=LAYERS, kv_len=KV + 1,
               shapes="LLaMA3-8B (4096 / 14336 / 32q 8kv / 128256), int4 g128, batch 1")
    del model
    torch.cuda.empty_cache()
    return rep


@torch.no_grad()
def test_full_width_decode_three_way():
    _judge([_decode_seed(s) for s in SEEDS])


def _prefill_seed(seed, layers, S):
    cfg = _cfg(layers)
    dev = torch.device("cuda")
    model = build_random_quant_llama(cfg, quant_args(4, 128), seed=seed, device=dev,
                                     dtype=torch.float16)
    rtn_quantize_(model)
    g = torch.Generator(device=dev).manual_seed(seed + 1)
    x = torch.randn(1, S, cfg.hidden_size, device=dev, dtype=torch.float16, generator=g)
    mask = causal_mask(1, S, torch.float16, dev)
    pos = torch.arange(S, device=dev)[None]

    h64 = x[0].double()
    for layer in model.layers:
        h64 = _ref64_window(layer, h64, cfg)
    _progress("prefill seed", seed, "layers", layers, "fp64 done")

    def run():
        h = x
        for layer in model.layers:
            h = layer(h, attention_mask=mask, position_ids=pos)[0]
        return h[0]

    paths = {"fake_quant": run()}
    for name, fn in TWINS.items():
        _reorder_reference(model, fn)
        paths[name] = run()
    _reorder_reference(model, F.linear)
    for layer in model.layers:
        pack_quant_linears(layer)
    paths["packed"] = run()
    for layer in model.layers:
        layer.fuse_packed_projections()
    paths["fused"] = run()
    for layer in model.layers:
        layer.fuse_packed_projections(prefill_attention=True)
    paths["fused_prefill_attention"] = run()
    _progress("prefill seed", seed, "paths done")
    rep = _report(seed, paths, model, cfg, h64)
    rep.update(layers=layers, window=S,
               shapes="LLaMA3-8B (4096 / 14336 / 32q 8kv / 128256), int4 g128, causal window")
    del model
    torch.cuda.empty_cache()
    return rep


@torch.no_grad()
def test_full_width_prefill_three_way():
    """A 256-token causal window (positions 0..255) through four full-width layers: fake-quant,
    its reordered twins, packed (MFMA GEMM), the fused layer, and the fused layer + the fused
    prefill-attention kernel (opt-in mode, DESIGN.md §4 qlin_attn_prefill)."""
    _judge([_prefill_seed(s, LAYERS, 256) for s in SEEDS], out_env="QLIN_PARITY_OUT_PREFILL")


@torch.no_grad()
def test_full_depth_prefill_attention_mode():
    """The opt-in prefill-attention mode through all 32 LLaMA3-8B layers (a 128-token window):
    amplified over 32 random layers, its distance to the fake-quant logits is held to the
    reference's own order floor at the same depth — every criterion of the declared bar, no
    exemption (round 5's 1.110 miss is gone with the reference-order softmax: exact row max,
    x fp32(1 / sqrt(d)), libm expf, three-term fp16 operands; csrc/qlin_attn_prefill.hip)."""
    _judge([_prefill_seed(s, 32, 128) for s in SEEDS32], out_env="QLIN_PARITY_OUT_PREFILL32")
