"""Model-level north-star criterion on GPU: a random-init LLaMA-architecture stack, RTN int4 g128,
run once through the reference's fake-quant path (weight = W_dq, dense F.linear) and once through
the packed gfx950 kernels on identical fp16 inputs.  Logits must agree within 1e-3 relative (to
max |logit|) and the perplexity within 1e-3 relative.  Covers the GEMV (one token) and the
MFMA GEMM (a window) dispatch."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from models.quant_llama import (build_random_quant_llama, eval_ppl, quant_args,  # noqa: E402
                                rtn_quantize_)
from quant import qlin  # noqa: E402
from quant.int_linear import QuantLinear  # noqa: E402
from quant.utils import pack_quant_linears  # noqa: E402


def _cfg(layers=4):
    from transformers import LlamaConfig
    return LlamaConfig(hidden_size=512, intermediate_size=1408, num_attention_heads=8,
                       num_key_value_heads=2, num_hidden_layers=layers, vocab_size=1000,
                       max_position_embeddings=256, rms_norm_eps=1e-5, rope_theta=500000.0)


def _rel(a, b):
    a = a.double()
    b = b.double()
    return ((a - b).abs().max() / b.abs().max()).item()


@pytest.mark.parametrize("wbits,group", [(4, 128), (3, 64), (2, 64)])
def test_packed_logits_match_fake_quant(wbits, group):
    cfg = _cfg()
    model = build_random_quant_llama(cfg, quant_args(wbits, group), seed=11, device="cuda",
                                     dtype=torch.float16)
    rtn_quantize_(model)  # fake-quant state: weight == W_dq, dense F.linear
    g = torch.Generator(device="cuda").manual_seed(5)
    toks = {T: torch.randint(0, cfg.vocab_size, (1, T), device="cuda", generator=g)
            for T in (1, 3, 37, 128)}
    with torch.no_grad():
        ref = {T: model(x).float() for T, x in toks.items()}
    for layer in model.layers:
        pack_quant_linears(layer)
    assert all(m.packed for layer in model.layers for m in layer.modules()
               if isinstance(m, QuantLinear))
    with torch.no_grad():
        got = {T: model(x).float() for T, x in toks.items()}
    for T in toks:
        assert _rel(got[T], ref[T]) < 1e-3, (T, _rel(got[T], ref[T]))


def test_packed_ppl_matches_fake_quant():
    cfg = _cfg(layers=3)
    model = build_random_quant_llama(cfg, quant_args(4, 128), seed=12, device="cuda",
                                     dtype=torch.float16)
    rtn_quantize_(model)
    g = torch.Generator(device="cuda").manual_seed(9)
    testenc = torch.randint(0, cfg.vocab_size, (1, 4 * 128), device="cuda", generator=g)
    ppl_fq = eval_ppl(model, testenc, seqlen=128)
    for layer in model.layers:
        pack_quant_linears(layer)
    ppl_pk = eval_ppl(model, testenc, seqlen=128)
    assert np.isfinite(ppl_fq) and abs(ppl_pk - ppl_fq) / ppl_fq < 1e-3, (ppl_fq, ppl_pk)


def test_fused_layer_matches_unfused():
    """fuse_packed_projections(): q/k/v and gate/up (+ SiLU·mul) as one launch each, residual
    adds in the o_proj / down_proj epilogues (all bit-identical per element), RMSNorm and RoPE
    as single kernels (RoPE bit-exact; RMSNorm's sum of squares in another order: one fp16 ulp
    here and there), decode attention kernel — logits within 1e-3 relative."""
    cfg = _cfg(layers=2)
    model = build_random_quant_llama(cfg, quant_args(4, 128), seed=13, device="cuda",
                                     dtype=torch.float16)
    rtn_quantize_(model, pack=True)
    g = torch.Generator(device="cuda").manual_seed(6)
    toks = [torch.randint(0, cfg.vocab_size, (1, T), device="cuda", generator=g)
            for T in (1, 5, 70)]
    with torch.no_grad():
        ref = [model(x) for x in toks]
        for layer in model.layers:
            layer.fuse_packed_projections()
        got = [model(x) for x in toks]
    for a, b in zip(got, ref):
        assert _rel(a, b) < 1e-3, _rel(a, b)


def test_fused_layer_w4a8_matches_unfused():
    """W4A8 (per-token 8-bit activations, the reference's act_quant_params): the fused layer
    runs the act quantizers inside the packed launches — logits equal the unfused packed path
    (act quantizer kernel, then the packed linear) within 1e-3 relative."""
    cfg = _cfg(layers=2)
    model = build_random_quant_llama(cfg, quant_args(4, 128, abits=8), seed=14, device="cuda",
                                     dtype=torch.float16)
    rtn_quantize_(model, pack=True)
    assert all(m.use_act_quant for layer in model.layers for m in layer.modules()
               if isinstance(m, QuantLinear))
    g = torch.Generator(device="cuda").manual_seed(7)
    toks = [torch.randint(0, cfg.vocab_size, (1, T), device="cuda", generator=g)
            for T in (1, 9, 80)]
    with torch.no_grad():
        ref = [model(x) for x in toks]
        for layer in model.layers:
            layer.fuse_packed_projections()
        assert model.layers[0].mlp.fused()
        got = [model(x) for x in toks]
    for a, b in zip(got, ref):
        assert _rel(a, b) < 1e-3, _rel(a, b)


def test_fused_prefill_attention_matches_reference_attention():
    """fuse_packed_projections(prefill_attention=True): multi-token windows take the fused
    prefill-attention kernel (causal mask verified on the host, key blocks past the diagonal
    skipped) — logits within 1e-3 relative of the reference attention path, and the PPL within
    1e-4 relative."""
    from transformers import LlamaConfig
    cfg = LlamaConfig(hidden_size=1024, intermediate_size=2816, num_attention_heads=8,
                      num_key_value_heads=2, num_hidden_layers=2, vocab_size=1000,
                      max_position_embeddings=256, rms_norm_eps=1e-5, rope_theta=500000.0)
    model = build_random_quant_llama(cfg, quant_args(4, 128), seed=15, device="cuda",
                                     dtype=torch.float16)
    rtn_quantize_(model, pack=True)
    g = torch.Generator(device="cuda").manual_seed(8)
    toks = [torch.randint(0, cfg.vocab_size, (1, T), device="cuda", generator=g)
            for T in (2, 70, 200)]
    testenc = torch.randint(0, cfg.vocab_size, (1, 4 * 64), device="cuda", generator=g)
    with torch.no_grad():
        for layer in model.layers:
            layer.fuse_packed_projections()
        ref = [model(x) for x in toks]
        ppl_ref = eval_ppl(model, testenc, seqlen=64)
        for layer in model.layers:
            layer.fuse_packed_projections(prefill_attention=True)
        assert model.layers[0].self_attn.prefill_kernel
        calls = []
        orig = qlin.attn_prefill
        qlin.attn_prefill = lambda *a, **k: calls.append(1) or orig(*a, **k)
        try:
            got = [model(x) for x in toks]
        finally:
            qlin.attn_prefill = orig
        assert len(calls) == 2 * len(toks)  # every layer of every window took the kernel
        ppl = eval_ppl(model, testenc, seqlen=64)
    for a, b in zip(got, ref):
        assert _rel(a, b) < 1e-3, _rel(a, b)
    assert abs(ppl - ppl_ref) / ppl_ref < 1e-4, (ppl, ppl_ref)
