"""Generate golden vectors by running the REFERENCE implementation (survey container only).

Run from the repo root:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
Needs ``/root/reference`` (SilviaUvA/LLaMA3-Quantization @ 2025-01-03).  The reference is imported
read-only; nothing of it is copied: only seeded inputs and the reference's outputs are written, as
``.npz`` files (no pickles) next to this script.  The GPU box never runs this script.

Cases (SURVEY.md §8c "Golden vectors to generate"):
  q_*      UniformAffineQuantizer (quant/quantizer.py:23-165) weight + activation cases
  lin_*    QuantLinear.forward (quant/int_linear.py:48-65)
  mm_*     QuantMatMul (quant/int_matmul.py:7-43) with per-token act quant
  llama_*  QuantLlamaDecoderLayer (models/int_llama_layer.py:191-267), fp32 forward of RTN int4
           g128 weights quantized in fp16 (harness-only transformers-4.37.2 RoPE shim, see below)
  opt_*    QuantOPTDecoderLayer (models/int_opt_layer.py:230-340), int8 per-channel (W8A16, W8A8)
Layer weights are NOT stored: they are regenerated from numpy seeds by ``layer_weights`` (shared
with the tests through ``tests/golden/golden_common.py``); the W_dq of every linear is pinned by a
sha256 of its fp16 bytes.
"""
import hashlib
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
REF = os.environ.get("REFERENCE_ROOT", "/root/reference")
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from golden_common import (LLAMA_CFG, OPT_CFG, layer_weights, llama_inputs,  # noqa: E402
                           opt_inputs, special_weight)

from quant.quantizer import UniformAffineQuantizer  # noqa: E402  (reference)
from quant.int_linear import QuantLinear  # noqa: E402  (reference)
from quant.int_matmul import QuantMatMul  # noqa: E402  (reference)


def t2n(t):
    return t.detach().cpu().numpy()


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def save(name, **arrs):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrs.items()})
    print("wrote", path, {k: getattr(np.asarray(v), "shape", None) for k, v in arrs.items()})


# ------------------------------------------------------------------------------------------------
# 1. UniformAffineQuantizer weight cases
# ------------------------------------------------------------------------------------------------
WEIGHT_CASES = [
    # name, shape, dtype, params, lwc factor dtype (None = no lwc)
    ("q_w4g128_f16", (64, 512), "f16", dict(n_bits=4, group_size=128), None),
    ("q_w3g64_f16", (64, 512), "f16", dict(n_bits=3, group_size=64), None),
    ("q_w2g64_f16", (64, 512), "f16", dict(n_bits=2, group_size=64), None),
    ("q_w8pc_f16", (64, 512), "f16", dict(n_bits=8, group_size=None), None),
    ("q_w4pc_f16_k4096", (16, 4096), "f16", dict(n_bits=4, group_size=None), None),
    ("q_w4g128_sym_f16", (64, 512), "f16", dict(n_bits=4, group_size=128, symmetric=True), None),
    ("q_w4g128_nozp_f16", (64, 512), "f16", dict(n_bits=4, group_size=128, disable_zero_point=True), None),
    ("q_w8g128_nozp_f16", (64, 512), "f16", dict(n_bits=8, group_size=128, disable_zero_point=True), None),
    ("q_w4g128_lwc16_f16", (64, 512), "f16", dict(n_bits=4, group_size=128, lwc=True), "f16"),
    ("q_w4g128_lwc32_f16", (64, 512), "f16", dict(n_bits=4, group_size=128, lwc=True), "f32"),
    ("q_w4g128_f32", (64, 512), "f32", dict(n_bits=4, group_size=128), None),
    ("q_w3g64_symlwc_def_f16", (32, 200), "f16", dict(n_bits=3, group_size=64, symmetric=True, lwc=True), "f16"),
]


def weight_case(name, shape, dt, params, lwc_dt, seed):
    W = special_weight(shape, seed)  # numpy fp32 with special groups in rows 0..5
    tdt = torch.float16 if dt == "f16" else torch.float32
    Wt = torch.from_numpy(W).to(tdt)
    q = UniformAffineQuantizer(**params, dynamic_method="per_channel", shape=Wt.shape)
    extra = {}
    if lwc_dt is not None:
        rs = np.random.RandomState(seed + 1000)
        up = (4.0 + rs.randn(*q.upbound_factor.shape) * 1.5).astype(np.float32)
        low = (4.0 + rs.randn(*q.lowbound_factor.shape) * 1.5).astype(np.float32)
        fdt = torch.float16 if lwc_dt == "f16" else torch.float32
        with torch.no_grad():
            q.upbound_factor.data = torch.from_numpy(up).to(fdt)
            q.lowbound_factor.data = torch.from_numpy(low).to(fdt)
        extra = dict(lwc_up=t2n(q.upbound_factor), lwc_low=t2n(q.lowbound_factor))
    with torch.no_grad():
        Wdq = q(Wt)
    out = dict(w=t2n(Wt), w_dq=t2n(Wdq), scale=t2n(q.scale),
               deficiency=np.int64(q.deficiency), **extra)
    if q.round_zero_point is not None:
        out["zp"] = t2n(q.round_zero_point)
    for k, v in params.items():
        out["p_" + k] = np.asarray(-1 if v is None else v)
    save(name, **out)


# ------------------------------------------------------------------------------------------------
# 2. activation (per-token) cases
# ------------------------------------------------------------------------------------------------
def act_cases():
    rs = np.random.RandomState(7)
    for bits, dt in ((8, torch.float16), (4, torch.float16), (8, torch.float32)):
        x = torch.from_numpy(rs.randn(2, 8, 512).astype(np.float32) * 2.0).to(dt)
        x[0, 0, :] = 0.0  # all-zero token: scale clamps to CLIPMIN
        q = UniformAffineQuantizer(n_bits=bits, per_channel_axes=[], symmetric=False,
                                   dynamic_method="per_token")
        with torch.no_grad():
            xq = q(x)
        tag = "f16" if dt == torch.float16 else "f32"
        save(f"q_a{bits}tok_{tag}", x=t2n(x), x_dq=t2n(xq), scale=t2n(q.scale),
             zp=t2n(q.round_zero_point), p_n_bits=np.asarray(bits))


# ------------------------------------------------------------------------------------------------
# 3. QuantLinear forward
# ------------------------------------------------------------------------------------------------
def linear_cases():
    rs = np.random.RandomState(11)
    for dt, tag in ((torch.float16, "f16"), (torch.float32, "f32")):
        lin = torch.nn.Linear(512, 96, bias=True)
        with torch.no_grad():
            lin.weight.copy_(torch.from_numpy(rs.randn(96, 512).astype(np.float32) * 0.02))
            lin.bias.copy_(torch.from_numpy(rs.randn(96).astype(np.float32) * 0.1))
        lin = lin.to(dt)
        ql = QuantLinear(lin, dict(n_bits=4, group_size=128, dynamic_method="per_channel",
                                   per_channel_axes=[0]),
                         dict(n_bits=8, dynamic_method="per_token"))
        ql.set_quant_state(weight_quant=True, act_quant=False)
        x1 = torch.from_numpy(rs.randn(1, 1, 512).astype(np.float32)).to(dt)
        x8 = torch.from_numpy(rs.randn(1, 8, 512).astype(np.float32)).to(dt)
        with torch.no_grad():
            y1 = ql(x1)
            y8 = ql(x8)
            ql.set_quant_state(weight_quant=True, act_quant=True)
            y8a = ql(x8)
        save(f"lin_w4g128_{tag}", w=t2n(lin.weight), b=t2n(lin.bias), x1=t2n(x1), x8=t2n(x8),
             y1=t2n(y1), y8=t2n(y8), y8_a8=t2n(y8a))


def matmul_cases():
    rs = np.random.RandomState(13)
    qp = dict(n_bits=8, per_channel_axes=[], symmetric=False, dynamic_method="per_token")
    mm = QuantMatMul(qp, qp, matmul_func=torch.matmul)
    x1 = torch.from_numpy(rs.randn(1, 2, 16, 64).astype(np.float32))
    x2 = torch.from_numpy(rs.randn(1, 2, 64, 16).astype(np.float32))
    with torch.no_grad():
        y = mm(x1, x2)
        mm.set_quant_state(False, True)
        y_q = mm(mm.quant_x1(x1), mm.quant_x2(x2))
    save("mm_a8_f32", x1=t2n(x1), x2=t2n(x2), y=t2n(y), y_a8=t2n(y_q))


# ------------------------------------------------------------------------------------------------
# 4. layers
# ------------------------------------------------------------------------------------------------
class _Args:
    pass


def make_args(wbits, group, abits):
    a = _Args()
    a.weight_quant_params = dict(n_bits=wbits, per_channel_axes=[0], symmetric=False,
                                 dynamic_method="per_channel", group_size=group, lwc=False,
                                 disable_zero_point=False)
    act = dict(n_bits=abits, per_channel_axes=[], symmetric=False, dynamic_method="per_token")
    a.act_quant_params = dict(act)
    a.q_quant_params = dict(act)
    a.k_quant_params = dict(act)
    a.v_quant_params = dict(act)
    a.p_quant_params = dict(n_bits=16, metric="fix0to1")
    return a


class Rotary437(torch.nn.Module):
    """Harness-only restatement of the transformers-4.37.2 LlamaRotaryEmbedding call contract
    that the reference layer expects (``rotary_emb(x, seq_len=)`` -> cos, sin [S, D])."""

    def __init__(self, dim, max_pos, base):
        super().__init__()
        inv_freq = 1.0 / (base ** (torch.arange(0, dim, 2).float() / dim))
        t = torch.arange(max_pos, dtype=torch.float32)
        emb = torch.cat((torch.outer(t, inv_freq),) * 2, dim=-1)
        self.register_buffer("cos_cached", emb.cos(), persistent=False)
        self.register_buffer("sin_cached", emb.sin(), persistent=False)

    def forward(self, x, seq_len=None):
        return self.cos_cached[:seq_len].to(x.dtype), self.sin_cached[:seq_len].to(x.dtype)


def _rotate_half(x):
    x1 = x[..., : x.shape[-1] // 2]
    x2 = x[..., x.shape[-1] // 2:]
    return torch.cat((-x2, x1), dim=-1)


def apply_rotary_437(q, k, cos, sin, position_ids, unsqueeze_dim=1):
    cos = cos[position_ids].unsqueeze(unsqueeze_dim)
    sin = sin[position_ids].unsqueeze(unsqueeze_dim)
    return (q * cos) + (_rotate_half(q) * sin), (k * cos) + (_rotate_half(k) * sin)


def quantize_layer_fp16(qlayer):
    """omniquant.py:296-314 with epochs == 0: .half() -> smooth_and_quant_inplace (no LET) ->
    register_scales_and_zeros; then back to fp32 for the golden forward."""
    from quant.utils import register_scales_and_zeros, smooth_and_quant_inplace
    qlayer.half()
    args = _Args()
    args.let = False
    qlayer.let = False
    smooth_and_quant_inplace(qlayer, args, True)
    register_scales_and_zeros(qlayer)
    hashes = {}
    for name, m in qlayer.named_modules():
        if isinstance(m, QuantLinear):
            hashes["sha_" + name.replace(".", "_")] = np.asarray(sha(t2n(m.weight)))
    qlayer.float()
    return hashes


def llama_case():
    from transformers import LlamaConfig
    from transformers.models.llama.modeling_llama import LlamaDecoderLayer
    import models.int_llama_layer as ref_llama
    cfg = LlamaConfig(**LLAMA_CFG)
    cfg._attn_implementation = "eager"
    hf = LlamaDecoderLayer(cfg, layer_idx=0)
    W = layer_weights("llama", LLAMA_CFG, seed=2024)
    with torch.no_grad():
        for name, arr in W.items():
            dict(hf.named_parameters())[name].copy_(torch.from_numpy(arr))
    head_dim = cfg.hidden_size // cfg.num_attention_heads
    hf.self_attn.rotary_emb = Rotary437(head_dim, LLAMA_CFG["max_position_embeddings"], LLAMA_CFG["rope_theta"])
    ref_llama.apply_rotary_pos_emb = apply_rotary_437
    x, mask, pos = llama_inputs(LLAMA_CFG, seed=99)
    out = {}
    for wbits, group in ((4, 128), (16, None)):
        q = ref_llama.QuantLlamaDecoderLayer(cfg, hf, make_args(wbits, group, 16))
        hashes = quantize_layer_fp16(q) if wbits < 16 else {}
        with torch.no_grad():
            y = q(torch.from_numpy(x), attention_mask=torch.from_numpy(mask),
                  position_ids=torch.from_numpy(pos))[0]
        tag = f"w{wbits}"
        out["y_" + tag] = t2n(y)
        out.update({k + "_" + tag: v for k, v in hashes.items()})
    save("llama_layer_fp32", x=x, mask=mask, pos=pos, **out)


def opt_case():
    from transformers import OPTConfig
    from transformers.models.opt.modeling_opt import OPTDecoderLayer
    from models.int_opt_layer import QuantOPTDecoderLayer
    from quant.utils import set_quant_state
    cfg = OPTConfig(**OPT_CFG)
    cfg._attn_implementation = "eager"
    hf = OPTDecoderLayer(cfg, layer_idx=0)
    W = layer_weights("opt", OPT_CFG, seed=125)
    with torch.no_grad():
        params = dict(hf.named_parameters())
        for name, arr in W.items():
            params[name].copy_(torch.from_numpy(arr))
    x, mask = opt_inputs(OPT_CFG, seed=5)
    out = {}
    for abits in (16, 8):
        q = QuantOPTDecoderLayer(cfg, hf, make_args(8, None, abits))
        hashes = quantize_layer_fp16(q)
        set_quant_state(q, weight_quant=False, act_quant=abits < 16)
        with torch.no_grad():
            y = q(torch.from_numpy(x), attention_mask=torch.from_numpy(mask))[0]
        tag = f"w8a{abits}"
        out["y_" + tag] = t2n(y)
        out.update({k + "_" + tag: v for k, v in hashes.items()})
    save("opt_layer_fp32", x=x, mask=mask, **out)


if __name__ == "__main__":
    torch.manual_seed(0)
    for i, (name, shape, dt, params, lwc_dt) in enumerate(WEIGHT_CASES):
        weight_case(name, shape, dt, params, lwc_dt, seed=100 + i)
    act_cases()
    linear_cases()
    matmul_cases()
    llama_case()
    opt_case()
