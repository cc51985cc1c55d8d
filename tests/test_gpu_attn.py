"""GPU parity of the fused decode-attention kernel (qlin_attn_decode) against the reference
layer's own fp32 formulation (models/int_llama_layer.py:137-165 of the reference: repeat_kv, QK^T,
/ sqrt(d), + mask, clamp at finfo.min, softmax, PV) computed with PyTorch in float64."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from quant import qlin  # noqa: E402


def _ref(q, k, v, mask):
    B, Hq, _, D = q.shape
    g = Hq // k.shape[1]
    kk = k.double().repeat_interleave(g, dim=1)
    vv = v.double().repeat_interleave(g, dim=1)
    w = q.double() @ kk.transpose(2, 3) / math.sqrt(D)
    if mask is not None:
        w = w + mask.double()
        w = torch.clamp_min(w, torch.finfo(torch.float32).min)
    p = torch.softmax(w, dim=-1)
    return p @ vv


@pytest.mark.parametrize("B,Hq,Hkv,L", [(1, 32, 8, 513), (1, 32, 8, 1), (2, 8, 8, 77),
                                        (1, 16, 2, 4096), (3, 4, 4, 300), (1, 64, 8, 1000),
                                        (40, 32, 8, 4096), (2, 32, 8, 31), (1, 8, 8, 2049)])
@pytest.mark.parametrize("masked", [False, True])
def test_attn_decode_matches_reference(B, Hq, Hkv, L, masked):
    g = torch.Generator(device="cuda").manual_seed(B * 1000 + L)
    q = torch.randn(B, Hq, 1, 128, device="cuda", generator=g) * 0.5
    k = torch.randn(B, Hkv, L, 128, device="cuda", generator=g).half()
    v = torch.randn(B, Hkv, L, 128, device="cuda", generator=g).half()
    mask = None
    if masked:
        mask = torch.zeros(B, 1, 1, L, device="cuda", dtype=torch.float16)
        mask[..., : L // 3] = torch.finfo(torch.float16).min  # a padded prefix
    out = qlin.attn_decode(q, k, v, mask, math.sqrt(128))
    ref = _ref(q, k, v, mask)
    err = (out.double() - ref).abs().max().item()
    assert err <= 1e-5 * max(1.0, ref.abs().max().item()), err
    # fp16 output = the fp32 result rounded once (the layer's .to(fp16) before o_proj)
    out16 = qlin.attn_decode(q, k, v, mask, math.sqrt(128), out_dtype=torch.float16)
    assert out16.dtype == torch.float16 and torch.equal(out16, out.half())


def test_attn_decode_split_counters_reset_under_graph_replay():
    """The split-L merge counts blocks in on a workspace counter that the last block resets: back
    to back eager calls and graph replays must give the same result every time."""
    g = torch.Generator(device="cuda").manual_seed(7)
    q = torch.randn(1, 32, 1, 128, device="cuda", generator=g)
    k = torch.randn(1, 8, 1500, 128, device="cuda", generator=g).half()
    v = torch.randn(1, 8, 1500, 128, device="cuda", generator=g).half()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        first = qlin.attn_decode(q, k, v, None, math.sqrt(128))
        again = qlin.attn_decode(q, k, v, None, math.sqrt(128))
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            out = qlin.attn_decode(q, k, v, None, math.sqrt(128))
        for _ in range(3):
            gr.replay()
    torch.cuda.synchronize()
    assert torch.equal(first, again)
    assert torch.equal(first, out)
    ref = _ref(q, k, v, None)
    assert (first.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()


def test_attn_decode_rejects_unsupported():
    q = torch.randn(1, 32, 1, 64, device="cuda")
    k = torch.randn(1, 8, 10, 64, device="cuda").half()
    assert not qlin.attn_decode_supported(q, k)
    with pytest.raises(ValueError):
        qlin.attn_decode(q, k, k, None, 8.0)


def test_layer_decode_kernel_matches_torch_path():
    """A packed LLaMA layer decode step (one token over a KV cache) with the fused kernel vs the
    reference formulation: same hidden state to fp16 rounding."""
    from transformers import LlamaConfig
    from models.int_llama_layer import QuantLlamaDecoderLayer
    from models.quant_llama import quant_args, random_llama_layer
    cfg = LlamaConfig(hidden_size=1024, intermediate_size=2816, num_attention_heads=8,
                      num_key_value_heads=2, num_hidden_layers=1, vocab_size=100,
                      max_position_embeddings=2048, rms_norm_eps=1e-5, rope_theta=500000.0)
    layer = QuantLlamaDecoderLayer(cfg, random_llama_layer(cfg, 3, "cuda", torch.float16),
                                   quant_args(4, 128))
    layer.half()
    layer.smooth_and_quant_inplace()
    layer.register_scales_and_zeros()
    from quant.utils import pack_quant_linears
    pack_quant_linears(layer)
    L = 700
    gen = torch.Generator(device="cuda").manual_seed(1)
    past = (torch.randn(1, 2, L, 128, device="cuda", generator=gen).half(),
            torch.randn(1, 2, L, 128, device="cuda", generator=gen).half())
    x = torch.randn(1, 1, 1024, device="cuda", generator=gen).half()
    mask = torch.zeros(1, 1, 1, L + 1, device="cuda", dtype=torch.float16)
    pos = torch.tensor([[L]], device="cuda")
    with torch.no_grad():
        ref = layer(x, attention_mask=mask, position_ids=pos, past_key_value=past)[0]
        layer.self_attn.decode_kernel = True
        got = layer(x, attention_mask=mask, position_ids=pos, past_key_value=past)[0]
    rel = ((got.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
    assert rel < 2e-3, rel
