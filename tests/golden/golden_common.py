"""Seeded inputs shared by the golden generator (make_golden.py) and the tests.

Pure numpy: the tests regenerate exactly the weights/inputs the reference saw without importing
the reference.  Test infrastructure only.
"""
import numpy as np

# reduced-width LLaMA3-shaped layer: head_dim 128, GQA 2:1, theta 500000 (LLaMA3)
LLAMA_CFG = dict(hidden_size=256, intermediate_size=512, num_attention_heads=2,
                 num_key_value_heads=1, rope_theta=500000.0, max_position_embeddings=64,
                 rms_norm_eps=1e-5, hidden_act="silu", vocab_size=512)
LLAMA_T = 16

# OPT-125M-width layer (hidden 768, 12 heads, FFN 3072, biased linears)
OPT_CFG = dict(hidden_size=768, ffn_dim=3072, num_attention_heads=12, enable_bias=True,
               do_layer_norm_before=True, attention_dropout=0.0, dropout=0.0,
               word_embed_proj_dim=768, max_position_embeddings=64, vocab_size=512)
OPT_T = 16


def special_weight(shape, seed):
    """W ~ N(0, 0.02^2) with hand-made hard groups in the first rows (first 64 columns):
    row 0 all-positive (zp < 0), row 1 all-zero (range 0 -> CLIPMIN scale), row 2 constant 0.5
    (x/s saturates), row 3 constant 1.0 (x/s overflows fp16 -> NaN through round_ste), row 4 a
    narrow range far from 0 (|zp| clamps at 1e4 -> wide zeros), row 5 large outliers."""
    rs = np.random.RandomState(seed)
    W = (rs.randn(*shape) * 0.02).astype(np.float32)
    n = min(64, shape[1])
    if shape[0] >= 6:
        W[0, :n] = np.abs(W[0, :n]) + 0.01
        W[1, :n] = 0.0
        W[2, :n] = 0.5
        W[3, :n] = 1.0
        W[4, :n] = 1.0 + rs.rand(n).astype(np.float32) * 1e-3
        W[5, :n] *= 50.0
    return W


def _llama_specs(c):
    H, I = c["hidden_size"], c["intermediate_size"]
    hd = H // c["num_attention_heads"]
    KV = c["num_key_value_heads"] * hd
    return [
        ("self_attn.q_proj.weight", (H, H), "w"),
        ("self_attn.k_proj.weight", (KV, H), "w"),
        ("self_attn.v_proj.weight", (KV, H), "w"),
        ("self_attn.o_proj.weight", (H, H), "w"),
        ("mlp.gate_proj.weight", (I, H), "w"),
        ("mlp.up_proj.weight", (I, H), "w"),
        ("mlp.down_proj.weight", (H, I), "w"),
        ("input_layernorm.weight", (H,), "n"),
        ("post_attention_layernorm.weight", (H,), "n"),
    ]


def _opt_specs(c):
    H, F = c["hidden_size"], c["ffn_dim"]
    s = []
    for p in ("k_proj", "v_proj", "q_proj", "out_proj"):
        s += [(f"self_attn.{p}.weight", (H, H), "w"), (f"self_attn.{p}.bias", (H,), "b")]
    s += [("self_attn_layer_norm.weight", (H,), "n"), ("self_attn_layer_norm.bias", (H,), "b"),
          ("fc1.weight", (F, H), "w"), ("fc1.bias", (F,), "b"),
          ("fc2.weight", (H, F), "w"), ("fc2.bias", (H,), "b"),
          ("final_layer_norm.weight", (H,), "n"), ("final_layer_norm.bias", (H,), "b")]
    return s


def layer_weights(kind, cfg, seed):
    """name -> float32 array for every parameter of one decoder layer (HF parameter names)."""
    specs = _llama_specs(cfg) if kind == "llama" else _opt_specs(cfg)
    rs = np.random.RandomState(seed)
    out = {}
    for name, shape, k in specs:
        r = rs.randn(*shape).astype(np.float32)
        if k == "w":
            out[name] = r * np.float32(0.05)
        elif k == "n":
            out[name] = np.float32(1.0) + r * np.float32(0.1)
        else:
            out[name] = r * np.float32(0.02)
    return out


def causal_mask(T):
    m = np.zeros((1, 1, T, T), dtype=np.float32)
    m[0, 0][np.triu_indices(T, 1)] = np.finfo(np.float32).min
    return m


def llama_inputs(cfg, seed, T=LLAMA_T):
    rs = np.random.RandomState(seed)
    x = rs.randn(1, T, cfg["hidden_size"]).astype(np.float32)
    return x, causal_mask(T), np.arange(T, dtype=np.int64)[None, :]


def opt_inputs(cfg, seed, T=OPT_T):
    rs = np.random.RandomState(seed)
    x = rs.randn(1, T, cfg["hidden_size"]).astype(np.float32)
    return x, causal_mask(T)
