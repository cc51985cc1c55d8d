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
            out.zero_()
            gr.replay()
            torch.cuda.synchronize()
            assert torch.equal(first, out)
    torch.cuda.synchronize()
    assert torch.equal(first, again)
    ref = _ref(q, k, v, None)
    assert (first.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()


def test_attn_decode_interleaved_shapes_and_layers():
    """Many launches of different lengths (split counts) and batch shapes back to back on one
    stream sharing its merge counters, each checked against the float64 reference (every launch
    leaves the counters zero for the next)."""
    g = torch.Generator(device="cuda").manual_seed(11)
    cases = []
    for L in (513, 1500, 77, 513, 4096, 1500, 600, 513):
        B = 1 if L != 77 else 3
        q = torch.randn(B, 32, 1, 128, device="cuda", generator=g)
        k = torch.randn(B, 8, L, 128, device="cuda", generator=g).half()
        v = torch.randn(B, 8, L, 128, device="cuda", generator=g).half()
        cases.append((q, k, v))
    for rep in range(3):
        outs = [qlin.attn_decode(q, k, v, None, math.sqrt(128)) for q, k, v in cases]
        for (q, k, v), o in zip(cases, outs):
            ref = _ref(q, k, v, None)
            assert (o.double() - ref).abs().max().item() <= 1e-5 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("B,L,rows", [(1, 513, 1024), (2, 77, 80), (1, 4096, 4104)])
def test_attn_decode_reads_cache_views(B, L, rows):
    """k / v as row-prefix views of [B, Hkv, rows, D] cache buffers (the kv_cache mode) are read
    in place: the same result, bit for bit, as on contiguous copies."""
    g = torch.Generator(device="cuda").manual_seed(L)
    q = torch.randn(B, 32, 1, 128, device="cuda", generator=g)
    kb = torch.randn(B, 8, rows, 128, device="cuda", generator=g).half()
    vb = torch.randn(B, 8, rows, 128, device="cuda", generator=g).half()
    k, v = kb[:, :, :L], vb[:, :, :L]
    assert qlin._cache_head_stride(k, v) == rows * 128
    mask = torch.zeros(B, 1, 1, L, device="cuda", dtype=torch.float16)
    got = qlin.attn_decode(q, k, v, mask, math.sqrt(128))
    ref = qlin.attn_decode(q, k.contiguous(), v.contiguous(), mask, math.sqrt(128))
    assert torch.equal(got, ref)


@pytest.mark.parametrize("B,Hq,Hkv,kv0,rows,masked", [(1, 32, 8, 512, 1024, True),
                                                     (1, 32, 8, 0, 256, False),
                                                     (2, 16, 4, 77, 80, True),
                                                     (1, 8, 1, 4095, 4096, False),
                                                     (3, 8, 8, 300, 512, True)])
def test_attn_decode_rope_equals_two_launches(B, Hq, Hkv, kv0, rows, masked):
    """qlin_attn_decode_rope (RoPE + KV append + decode attention in one launch) = qlin_rope_kv_f16
    then qlin_attn_decode, bit for bit: output and the written cache row."""
    from models.int_llama_layer import LlamaRotaryEmbedding437
    D = 128
    g = torch.Generator(device="cuda").manual_seed(kv0 + 7 * B)
    qkv = (torch.randn(B, 1, (Hq + 2 * Hkv) * D, device="cuda", generator=g) * 2).half()
    q, k, v = torch.split(qkv, [Hq * D, Hkv * D, Hkv * D], dim=-1)
    rot = LlamaRotaryEmbedding437(D, 8192, 500000.0, device="cuda").half()
    cos, sin = rot.cos_cached.float().contiguous(), rot.sin_cached.float().contiguous()
    pos = torch.full((B, 1), kv0, device="cuda", dtype=torch.int64)
    kc = torch.randn(B, Hkv, rows, D, device="cuda", generator=g).half()
    vc = torch.randn(B, Hkv, rows, D, device="cuda", generator=g).half()
    kc2, vc2 = kc.clone(), vc.clone()
    mask = None
    if masked:
        mask = torch.zeros(B, 1, 1, kv0 + 1, device="cuda", dtype=torch.float16)
        mask[..., : kv0 // 4] = torch.finfo(torch.float16).min
    got = qlin.attn_decode_rope(q, k, v, cos, sin, pos, Hq, Hkv, D, kc, vc, kv0, mask,
                                math.sqrt(D))
    qr = qlin.rope_kv(q, k, v, cos, sin, pos, Hq, Hkv, D, kc2, vc2, kv0)
    ref = qlin.attn_decode(qr, kc2[:, :, :kv0 + 1], vc2[:, :, :kv0 + 1], mask, math.sqrt(D))
    assert torch.equal(kc, kc2) and torch.equal(vc, vc2)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("B,Hq,Hkv,kv0,cap", [(1, 32, 8, 512, 513), (1, 32, 8, 100, 1024),
                                               (2, 16, 4, 77, 300), (1, 8, 1, 2000, 4096)])
def test_attn_decode_rope_len_matches(B, Hq, Hkv, kv0, cap):
    """qlin_attn_decode_rope_len (cache length read on the device, grid sized for the capacity):
    at length == capacity bit-identical to qlin_attn_decode_rope, below it the same attention to
    fp32 rounding (the rows split by the capacity's chunk); the new cache row written the same."""
    from models.int_llama_layer import LlamaRotaryEmbedding437
    D = 128
    g = torch.Generator(device="cuda").manual_seed(kv0 + cap)
    qkv = (torch.randn(B, 1, (Hq + 2 * Hkv) * D, device="cuda", generator=g) * 2).half()
    q, k, v = torch.split(qkv, [Hq * D, Hkv * D, Hkv * D], dim=-1)
    rot = LlamaRotaryEmbedding437(D, 8192, 500000.0, device="cuda").half()
    cos, sin = rot.cos_cached.float().contiguous(), rot.sin_cached.float().contiguous()
    pos = torch.full((B, 1), kv0, device="cuda", dtype=torch.int64)
    kc = torch.randn(B, Hkv, cap, D, device="cuda", generator=g).half()
    vc = torch.randn(B, Hkv, cap, D, device="cuda", generator=g).half()
    kc2, vc2 = kc.clone(), vc.clone()
    length = torch.tensor([kv0 + 1], dtype=torch.int32, device="cuda")
    got = qlin.attn_decode_rope_len(q, k, v, cos, sin, pos, Hq, Hkv, D, kc, vc, length)
    ref = qlin.attn_decode_rope(q, k, v, cos, sin, pos, Hq, Hkv, D, kc2, vc2, kv0, None,
                                math.sqrt(D))
    assert torch.equal(kc[:, :, :kv0 + 1], kc2[:, :, :kv0 + 1])
    assert torch.equal(vc[:, :, :kv0 + 1], vc2[:, :, :kv0 + 1])
    if kv0 + 1 == cap:
        assert torch.equal(got, ref)
    else:
        assert (got - ref).abs().max().item() <= 1e-5 * max(1.0, ref.abs().max().item())


def test_attn_decode_rope_len_bounds():
    """The device-length attention sizes its grid for ``max_len`` (the longest length the captured
    steps will reach) and refuses caches / lengths past ATTN_MAX_L rows instead of clamping (a
    clamped length would attend over a prefix and rewrite row ATTN_MAX_L - 1); with max_len the
    grid of a large-capacity cache covers exactly the steps' lengths."""
    from models.int_llama_layer import LlamaRotaryEmbedding437
    B, Hq, Hkv, D = 1, 32, 8, 128
    g = torch.Generator(device="cuda").manual_seed(3)
    qkv = (torch.randn(B, 1, (Hq + 2 * Hkv) * D, device="cuda", generator=g) * 2).half()
    q, k, v = torch.split(qkv, [Hq * D, Hkv * D, Hkv * D], dim=-1)
    rot = LlamaRotaryEmbedding437(D, 8192, 500000.0, device="cuda").half()
    cos, sin = rot.cos_cached.float().contiguous(), rot.sin_cached.float().contiguous()
    big = qlin.ATTN_MAX_L + 256
    kc = torch.randn(B, Hkv, big, D, device="cuda", generator=g).half()
    vc = torch.randn(B, Hkv, big, D, device="cuda", generator=g).half()
    kv0 = 700
    pos = torch.full((B, 1), kv0, device="cuda", dtype=torch.int64)
    length = torch.tensor([kv0 + 1], dtype=torch.int32, device="cuda")
    with pytest.raises(ValueError):  # capacity past ATTN_MAX_L and no max_len
        qlin.attn_decode_rope_len(q, k, v, cos, sin, pos, Hq, Hkv, D, kc, vc, length)
    with pytest.raises(ValueError):
        qlin.attn_decode_rope_len(q, k, v, cos, sin, pos, Hq, Hkv, D, kc, vc, length,
                                  max_len=qlin.ATTN_MAX_L + 1)
    kc2, vc2 = kc.clone(), vc.clone()
    got = qlin.attn_decode_rope_len(q, k, v, cos, sin, pos, Hq, Hkv, D, kc, vc, length,
                                    max_len=kv0 + 1)
    ref = qlin.attn_decode_rope(q, k, v, cos, sin, pos, Hq, Hkv, D, kc2, vc2, kv0, None,
                                math.sqrt(D))
    assert torch.equal(got, ref)  # max_len == length: the per-step launch's split, same bits
    assert torch.equal(kc, kc2) and torch.equal(vc, vc2)


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


def test_layer_kv_cache_mode_matches_cat():
    """fuse_packed_projections(kv_cache=True): a prefill then decode steps with use_cache append
    into the module's cache buffers (qlin_rope_kv_f16) instead of torch.cat — identical hidden
    states and identical past_key_value contents at every step."""
    from transformers import LlamaConfig
    from models.int_llama_layer import QuantLlamaDecoderLayer
    from models.quant_llama import quant_args, random_llama_layer
    from quant.utils import pack_quant_linears
    cfg = LlamaConfig(hidden_size=1024, intermediate_size=2816, num_attention_heads=8,
                      num_key_value_heads=2, num_hidden_layers=1, vocab_size=100,
                      max_position_embeddings=2048, rms_norm_eps=1e-5, rope_theta=500000.0)
    layers = []
    for kv in (False, True):
        layer = QuantLlamaDecoderLayer(cfg, random_llama_layer(cfg, 5, "cuda", torch.float16),
                                       quant_args(4, 128))
        layer.half()
        layer.smooth_and_quant_inplace()
        layer.register_scales_and_zeros()
        pack_quant_linears(layer)
        layer.fuse_packed_projections(kv_cache=kv)
        layers.append(layer)
    gen = torch.Generator(device="cuda").manual_seed(2)
    T0, steps = 300, 4
    xs = torch.randn(1, T0 + steps, 1024, device="cuda", generator=gen).half()
    pasts = [None, None]
    with torch.no_grad():
        for i in range(steps + 1):
            lo, hi = (0, T0) if i == 0 else (T0 + i - 1, T0 + i)
            x = xs[:, lo:hi]
            L = hi
            mask = torch.zeros(1, 1, hi - lo, L, device="cuda", dtype=torch.float16)
            if i == 0:
                mask[0, 0] = torch.triu(torch.full((T0, T0), torch.finfo(torch.float16).min,
                                                   device="cuda"), 1).half()
            pos = torch.arange(lo, hi, device="cuda")[None]
            outs = []
            for j, layer in enumerate(layers):
                o = layer(x, attention_mask=mask, position_ids=pos, past_key_value=pasts[j],
                          use_cache=True)
                outs.append(o[0])
                pasts[j] = o[-1]
            assert torch.equal(outs[0], outs[1]), i
            assert torch.equal(pasts[0][0], pasts[1][0]) and torch.equal(pasts[0][1], pasts[1][1]), i
    # the kv_cache layer's past is a view of its own buffer (no per-step copy of the cache)
    assert pasts[1][0].data_ptr() == layers[1].self_attn._kv[0].data_ptr()


def _causal_mask(B, S, L, dtype=torch.float16, pad=None):
    """HF-style additive 4D mask [B, 1, S, L]: query i (key position L - S + i) sees keys <= its
    position; ``pad`` left-pads batch b's first pad[b] keys as well (non-causal pattern)."""
    i = torch.arange(S, device="cuda")[:, None]
    j = torch.arange(L, device="cuda")[None, :]
    m = torch.zeros(B, 1, S, L, device="cuda", dtype=dtype)
    m[:, 0][:, j.expand(S, L) > (L - S) + i.expand(S, L)] = torch.finfo(dtype).min
    if pad is not None:
        for b, p in enumerate(pad):
            m[b, 0, :, :p] = torch.finfo(dtype).min
    return m


@pytest.mark.parametrize("B,Hq,Hkv,S,L", [(1, 32, 8, 128, 128), (1, 32, 8, 257, 257),
                                          (1, 8, 8, 100, 137), (2, 16, 4, 65, 65),
                                          (1, 16, 2, 33, 100), (1, 8, 1, 200, 200),
                                          (1, 4, 4, 1, 40), (1, 32, 8, 2048, 2048)])
@pytest.mark.parametrize("mask_kind", ["causal", "causal_f32", "none"])
def test_attn_prefill_matches_reference(B, Hq, Hkv, S, L, mask_kind):
    """Fused prefill attention (qlin_attn_prefill, fp32 arithmetic on the matrix cores) vs the
    reference formulation in float64; causal masks take the block-skipping path."""
    g = torch.Generator(device="cuda").manual_seed(B * 7919 + S * 31 + L)
    q = torch.randn(B, Hq, S, 128, device="cuda", generator=g) * 0.5
    k = torch.randn(B, Hkv, L, 128, device="cuda", generator=g).half()
    v = torch.randn(B, Hkv, L, 128, device="cuda", generator=g).half()
    mask = None
    if mask_kind != "none":
        mask = _causal_mask(B, S, L, torch.float32 if mask_kind == "causal_f32" else torch.float16)
        assert qlin.mask_is_causal(mask, S, L) == 2  # the pure pattern: applied, never read
    out = qlin.attn_prefill(q, k, v, mask, math.sqrt(128))
    ref = _ref(q, k, v, mask).transpose(1, 2)
    err = (out.double() - ref).abs().max().item()
    assert err <= 1e-5 * max(1.0, ref.abs().max().item()), err
    out16 = qlin.attn_prefill(q, k, v, mask, math.sqrt(128), out_dtype=torch.float16)
    assert out16.dtype == torch.float16 and torch.equal(out16, out.half())


def _ref32(q, k, v, mask):
    """The reference's own fp32 attention core (models/int_llama_layer.py:137-165: repeat_kv,
    fp32 bmm, / sqrt(d), + mask, max(., finfo.min), fp32 softmax, fp32 bmm) run by torch."""
    B, Hq, _, D = q.shape
    g = Hq // k.shape[1]
    kk = k.float().repeat_interleave(g, dim=1)
    vv = v.float().repeat_interleave(g, dim=1)
    w = torch.matmul(q, kk.transpose(2, 3)) / math.sqrt(D)
    if mask is not None:
        w = w + mask
        w = torch.max(w, torch.tensor(torch.finfo(torch.float32).min, device=w.device))
    p = torch.nn.functional.softmax(w, dim=-1, dtype=torch.float32)
    return torch.matmul(p, vv)


@pytest.mark.parametrize("S,L,mask_kind", [(128, 128, "causal"), (2048, 2048, "causal"),
                                           (300, 813, "causal"), (257, 257, "none"),
                                           (150, 150, "padded")])
def test_attn_prefill_reference_order_accuracy(S, L, mask_kind):
    """Round 6: with the reference-order softmax (exact row max, x fp32
    1 / sqrt(d), libm expf) and exact three-term operands, the kernel is as accurate as the
    reference's own fp32 path: its float64 error at most 1.5x the torch fp32 reference's own
    float64 error (max over the output, relative to max |out|), and its fp16-rounded output (the
    layer casts the attention output to fp16 before o_proj) equal to the fp16 rounding of the
    exact (float64) result on at least as many elements as the reference's own fp32 path's
    (within 0.02 %).  (The first run of this test also asked >= 99.9 % fp16 equality with the
    reference's fp32 path; measured 99.46-99.68 % while the kernel was closer to float64 than the
    reference on every case — the reference's own fp32 rounding flips fp16 outputs at that rate,
    so that criterion measured the reference's error, not the kernel's)"""
    B, Hq, Hkv = 1, 32, 8
    g = torch.Generator(device="cuda").manual_seed(S * 131 + L)
    # LLaMA-like score spread: q . k / sqrt(d) of a few units
    q = torch.randn(B, Hq, S, 128, device="cuda", generator=g) * 1.5
    k = torch.randn(B, Hkv, L, 128, device="cuda", generator=g).half()
    v = torch.randn(B, Hkv, L, 128, device="cuda", generator=g).half()
    mask = None
    if mask_kind != "none":
        mask = _causal_mask(B, S, L, torch.float16, pad=[7] if mask_kind == "padded" else None)
    out = qlin.attn_prefill(q, k, v, mask, math.sqrt(128)).double()
    r32 = _ref32(q, k, v, mask).transpose(1, 2).double()
    r64 = _ref(q, k, v, mask).transpose(1, 2)
    scale = r64.abs().max().item()
    e_k = (out - r64).abs().max().item() / scale
    e_r = (r32 - r64).abs().max().item() / scale
    exact16 = r64.half()
    same_k = (out.half() == exact16).double().mean().item()
    same_r = (r32.half() == exact16).double().mean().item()
    same_kr = (out.half() == r32.half()).double().mean().item()
    print(f"S={S} L={L} {mask_kind}: kernel fp64 err {e_k:.3e}, reference fp32 err {e_r:.3e}, "
          f"fp16 = exact: kernel {same_k:.6f} reference {same_r:.6f}; kernel = reference "
          f"{same_kr:.6f}")
    assert e_k <= 1.5 * e_r + 1e-9, (e_k, e_r)
    assert same_k >= same_r - 2e-4, (same_k, same_r)


def test_attn_prefill_padding_mask_is_not_causal():
    """Left padding on top of the causal pattern keeps every key block (non-causal path), and a
    fully masked padded query row reproduces the reference's softmax over finfo.min scores."""
    B, Hq, Hkv, S = 2, 8, 2, 150
    g = torch.Generator(device="cuda").manual_seed(5)
    q = torch.randn(B, Hq, S, 128, device="cuda", generator=g)
    k = torch.randn(B, Hkv, S, 128, device="cuda", generator=g).half()
    v = torch.randn(B, Hkv, S, 128, device="cuda", generator=g).half()
    mask = _causal_mask(B, S, S, pad=[0, 70])
    assert qlin.mask_is_causal(mask, S, S) == 0
    out = qlin.attn_prefill(q, k, v, mask, math.sqrt(128))
    ref = _ref(q, k, v, mask).transpose(1, 2)
    # rows 0..69 of batch 1 see no open key: their scores are qk / sqrt(d) - 65504 quantised to
    # the fp32 grid there (~0.004), so the kernel and an fp32 reference agree only loosely
    live = torch.ones(B, S, dtype=torch.bool, device="cuda")
    live[1, :70] = False
    d = (out.double() - ref).abs().amax(dim=(2, 3))
    assert d[live].max().item() <= 1e-5 * ref.abs().max().item()
    assert d[~live].max().item() <= 2e-2 * ref.abs().max().item()
    # a causal-looking mask that is broadcast over the batch
    mask1 = _causal_mask(1, S, S)
    out = qlin.attn_prefill(q, k, v, mask1, math.sqrt(128))
    ref = _ref(q, k, v, mask1).transpose(1, 2)
    assert (out.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()


def test_attn_prefill_rejects_unsupported():
    q = torch.randn(1, 32, 8, 64, device="cuda")
    k = torch.randn(1, 8, 8, 64, device="cuda").half()
    assert not qlin.attn_prefill_supported(q, k)
    q = torch.randn(1, 32, 9, 128, device="cuda")
    k = torch.randn(1, 8, 8, 128, device="cuda").half()  # L < S
    assert not qlin.attn_prefill_supported(q, k)
    with pytest.raises(ValueError):
        qlin.attn_prefill(q, k, k, None, 8.0)
    lib = qlin.load_library()
    p = 16
    # mask-reading causal mode without a mask, bad mode, odd group size
    assert lib.qlin_attn_prefill(p, p, p, None, 0, 0, 1, p, 0, 1, 8, 8, 4, 4, 128, 11.3, None) == 1
    assert lib.qlin_attn_prefill(p, p, p, p, 0, 0, 3, p, 0, 1, 8, 8, 4, 4, 128, 11.3, None) == 1
    assert lib.qlin_attn_prefill(p, p, p, None, 0, 0, 0, p, 0, 1, 24, 8, 4, 4, 128, 11.3, None) == 1
