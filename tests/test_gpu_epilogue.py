"""GPU: the packed linear's fused output epilogues (qlin_linear_ep_f16) against the unfused
launches they replace — residual add (bit-exact) and SiLU·mul over interleaved gate/up rows
(QuantLlamaMLP's act_fn(gate) * up on the fp16 F.linear outputs)."""
import numpy as np
import pytest
import torch

from helpers import rand_weight, rand_x, t

pytestmark = pytest.mark.gpu

from quant import qlin  # noqa: E402

MS = (1, 3, 16, 40, 300)


def _packed(N, K, seed, bits=4, group=128):
    o = qlin.quantize(t(rand_weight(N, K, seed)), bits, group, 0, want_xdq=False,
                      want_params=False, pack=True)
    return o["qweight"], o["qsz"], o["flags"]


@pytest.mark.parametrize("M", MS)
def test_residual_epilogue_bit_exact(M):
    N, K = 384, 1024
    qw, qsz, fl = _packed(N, K, 1)
    x = t(rand_x(M, K, 2))
    r = t(rand_x(M, N, 3))
    bias = t((np.random.RandomState(4).randn(N) * 0.1).astype(np.float16))
    ref = r + qlin.linear(x, qw, qsz, bias, N, K, 4, 128, fl)
    got = qlin.linear_ep(x, qw, qsz, bias, N, K, 4, 128, fl, epilogue=qlin.EP_RESIDUAL, residual=r)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("M", MS)
@pytest.mark.parametrize("bits,group", [(4, 128), (3, 64)])
def test_silu_mul_epilogue(M, bits, group):
    I, K = 528, 1024  # 33 tiles of 16 rows
    qg, sg, fg = _packed(I, K, 5, bits, group)
    qu, su, fu = _packed(I, K, 6, bits, group)
    x = t(rand_x(M, K, 7))
    gate = qlin.linear(x, qg, sg, None, I, K, bits, group, fg)
    up = qlin.linear(x, qu, su, None, I, K, bits, group, fu)
    ref = torch.nn.functional.silu(gate) * up
    qw, qsz = qlin.interleave_gate_up(qg, sg, qu, su)
    got = qlin.linear_ep(x, qw, qsz, None, 2 * I, K, bits, group, fg | fu,
                         epilogue=qlin.EP_SILU_MUL)
    assert got.shape == ref.shape
    # identical accumulators; silu is torch's fp32 x / (1 + exp(-x)) rounded to fp16 — allow the
    # rare one-ulp difference should the two exp implementations round differently
    diff = (got.float() - ref.float()).abs()
    ulp = ref.float().abs().clamp_min(6.1e-5) * 2.0 ** -10
    assert bool((diff <= ulp).all()), float(diff.max())
    assert (diff > 0).float().mean().item() < 1e-3


def test_epilogue_argument_checks():
    lib = qlin.load_library()
    qw, qsz, fl = _packed(32, 128, 8)
    x = t(rand_x(1, 128, 9))
    y = torch.empty(1, 32, dtype=torch.float16, device="cuda")
    P = lambda a: a.data_ptr()
    ep = lib.qlin_linear_ep_f16
    assert ep(P(qw), P(qsz), fl, P(x), None, None, P(y), 1, 32, 128, 4, 128, qlin.EP_RESIDUAL,
              0, 0, None, 0, None) == 1  # residual missing
    assert ep(P(qw), P(qsz), fl, P(x), None, None, P(y), 1, 24, 128, 4, 128, qlin.EP_SILU_MUL,
              0, 0, None, 0, None) == 1  # N % 16
    assert ep(P(qw), P(qsz), fl, P(x), None, None, P(y), 1, 32, 128, 4, 128, 7,
              0, 0, None, 0, None) == 1  # unknown epilogue


@pytest.mark.parametrize("rows,H", [(1, 4096), (7, 4096), (3, 768), (5, 14336), (64, 4096)])
def test_rmsnorm_kernel_matches_mirror(rows, H):
    from quant.omni_norm import OmniLlamaRMSNorm
    rs = np.random.RandomState(rows + H)
    x = t((rs.randn(1, rows, H) * 3).astype(np.float16))
    w = torch.nn.Module()
    w.weight = torch.nn.Parameter(t((1 + 0.1 * rs.randn(H)).astype(np.float16)), requires_grad=False)
    norm = OmniLlamaRMSNorm(w, eps=1e-5)
    ref = norm(x)
    norm.use_kernel = True
    got = norm(x)
    diff = (got.float() - ref.float()).abs()
    # same fp32 arithmetic; the sum of squares runs in another order than torch's reduction
    assert bool((diff <= ref.float().abs() * 2.0 ** -10 + 1e-7).all()), float(diff.max())
    assert (diff > 0).float().mean().item() < 0.02


@pytest.mark.parametrize("B,S,strided", [(1, 1, True), (1, 37, True), (3, 5, False), (2, 64, True),
                                         (2, 9, "odd")])
def test_rope_kernel_bit_exact(B, S, strided):
    """Row kernel (aligned rows) and, for "odd" (rows starting at an odd element, not 8-B
    aligned), the per-element kernel: both bit-exact with the reference's apply_rotary_pos_emb."""
    from models.int_llama_layer import LlamaRotaryEmbedding437, apply_rotary_pos_emb
    Hq, Hkv, D = 8, 2, 128
    rs = np.random.RandomState(B * 100 + S)
    qkv = t((rs.randn(B, S, (Hq + 2 * Hkv) * D + 1) * 2).astype(np.float16))
    if strided == "odd":
        qkv = qkv[..., 1:]
    else:
        qkv = qkv[..., :-1]
    q, k, _ = torch.split(qkv, [Hq * D, Hkv * D, Hkv * D], dim=-1)
    if not strided:
        q, k = q.contiguous(), k.contiguous()
    rot = LlamaRotaryEmbedding437(D, 256, 500000.0, device="cuda").half()  # cache in fp16, as after layer.half()
    pos = torch.stack([torch.arange(S) + 11 * b for b in range(B)]).cuda()
    qs = q.reshape(B, S, Hq, D).transpose(1, 2).type(torch.float32)
    ks = k.reshape(B, S, Hkv, D).transpose(1, 2)
    cos, sin = rot(ks, seq_len=int(pos.max()) + 1)
    ref_q, ref_k = apply_rotary_pos_emb(qs, ks, cos, sin, pos)
    got_q, got_k = qlin.rope(q, k, rot.cos_cached.float().contiguous(),
                             rot.sin_cached.float().contiguous(), pos, Hq, Hkv, D)
    assert got_q.dtype == torch.float32 and got_k.dtype == torch.float16
    assert torch.equal(got_q, ref_q.contiguous())
    assert torch.equal(got_k, ref_k.contiguous())


@pytest.mark.parametrize("B,S,kv0,rows", [(1, 1, 0, 8), (1, 1, 511, 512), (2, 7, 20, 64),
                                          (3, 1, 33, 40)])
def test_rope_kv_appends_into_cache(B, S, kv0, rows):
    """qlin_rope_kv_f16 = qlin_rope_f16 + the reference's torch.cat of the KV cache: the rotated
    k and the v rows land at cache rows kv0 .. kv0 + S - 1 bit for bit; no other row changes."""
    from models.int_llama_layer import LlamaRotaryEmbedding437
    Hq, Hkv, D = 8, 2, 128
    rs = np.random.RandomState(B * 1000 + S + kv0)
    qkv = t((rs.randn(B, S, (Hq + 2 * Hkv) * D) * 2).astype(np.float16))
    q, k, v = torch.split(qkv, [Hq * D, Hkv * D, Hkv * D], dim=-1)
    rot = LlamaRotaryEmbedding437(D, 1024, 500000.0, device="cuda").half()
    cos, sin = rot.cos_cached.float().contiguous(), rot.sin_cached.float().contiguous()
    pos = torch.stack([torch.arange(S) + kv0 + b for b in range(B)]).cuda()
    kc = t(rs.randn(B, Hkv, rows, D).astype(np.float16))
    vc = t(rs.randn(B, Hkv, rows, D).astype(np.float16))
    kc0, vc0 = kc.clone(), vc.clone()
    got_q = qlin.rope_kv(q, k, v, cos, sin, pos, Hq, Hkv, D, kc, vc, kv0)
    ref_q, ref_k = qlin.rope(q, k, cos, sin, pos, Hq, Hkv, D)
    assert torch.equal(got_q, ref_q)
    assert torch.equal(kc[:, :, kv0:kv0 + S], ref_k)
    assert torch.equal(vc[:, :, kv0:kv0 + S], v.reshape(B, S, Hkv, D).transpose(1, 2))
    keep = torch.ones(rows, dtype=torch.bool)
    keep[kv0:kv0 + S] = False
    assert torch.equal(kc[:, :, keep], kc0[:, :, keep]) and torch.equal(vc[:, :, keep], vc0[:, :, keep])
    with pytest.raises(ValueError):
        qlin.rope_kv(q, k, v, cos, sin, pos, Hq, Hkv, D, kc, vc, rows - S + 1)


@pytest.mark.parametrize("M", (1, 2, 5, 16, 33, 200))
@pytest.mark.parametrize("abits,aflags", [(8, 0), (4, 0), (6, 1), (8, 2)])
def test_fused_act_quant_matches_two_launches(M, abits, aflags):
    """qlin_linear_ep_f16 with act_bits: per-token fake-quant of x fused into the GEMV (M <= 64)
    or run by the quantizer kernel into the workspace (M > 64) — bit-identical to the reference
    order act_quantizer(x) (quantizer kernel, itself bit-exact with the reference) then the
    packed linear."""
    N, K = (272, 1024) if M != 2 else (16400, 256)  # N > 16384: the quantizer + GEMV leg
    qw, qsz, fl = _packed(N, K, 11)
    x = t((np.random.RandomState(M + abits).randn(M, K) * 2).astype(np.float16))
    xdq = qlin.quantize(x, abits, K, aflags, want_params=False)["x_dq"]
    ref = qlin.linear(xdq, qw, qsz, None, N, K, 4, 128, fl)
    got = qlin.linear_ep(x, qw, qsz, None, N, K, 4, 128, fl, act_bits=abits, act_flags=aflags)
    assert torch.equal(got, ref)


def test_quantlinear_act_quant_fused_path(golden):
    """QuantLinear (packed, W4 + per-token A8) equals the two-launch path on the reference's own
    A8 activation fixture."""
    from quant.int_linear import QuantLinear
    g = golden("q_a8tok_f16")
    x = t(g["x"])
    K = x.shape[-1]
    lin = torch.nn.Linear(K, 64, bias=False).cuda().half()
    with torch.no_grad():
        lin.weight.copy_(t(rand_weight(64, K, 3)))
    ql = QuantLinear(lin, dict(n_bits=4, group_size=min(128, K), dynamic_method="per_channel",
                               per_channel_axes=[0]),
                     dict(n_bits=8, per_channel_axes=[], symmetric=False,
                          dynamic_method="per_token")).cuda()
    ql.pack_from_weight()
    ql.set_quant_state(weight_quant=False, act_quant=True)
    got = ql(x)
    ref = qlin.linear(t(g["x_dq"]).reshape(-1, K), ql.qweight, ql.qsz, None, 64, K, 4, ql.group,
                      ql.qflags).reshape(got.shape)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("mask", ["f16", "f32", "none", "bcast"])
def test_attn_scores_pass_bit_exact(mask):
    """/ sqrt(d) + mask + torch.max(w, finfo.min) in one in-place pass == the reference's three
    torch ops (models/int_llama_layer.py:143-157)."""
    import math
    B, H, T, L = 2, 4, 37, 40
    w = torch.randn(B, H, T, L, device="cuda") * 50
    w[0, 0, 0, :3] = torch.tensor([float("nan"), float("-inf"), -3e38])
    m = None
    if mask != "none":
        mm = torch.full((T, L), torch.finfo(torch.float16).min).triu(1 + L - T)
        m = mm[None, None].expand(B if mask != "bcast" else 1, 1, T, L).contiguous()
        m = m.to("cuda", torch.float16 if mask == "f16" else torch.float32)
        if mask == "bcast":
            m = m.expand(B, 1, T, L)
    ref = w / math.sqrt(128)
    if m is not None:
        ref = (ref + m).clamp_min(torch.finfo(torch.float32).min)
    got = qlin.attn_scores_(w.clone(), m, math.sqrt(128))
    assert torch.equal(torch.nan_to_num(got, nan=7.0), torch.nan_to_num(ref, nan=7.0))
    assert torch.isnan(got[0, 0, 0, 0])


@pytest.mark.parametrize("N,K,bits,group,ep", [(6144, 4096, 4, 128, "none"),
                                               (4096, 4096, 4, 128, "residual"),
                                               (2 * 2816, 1024, 4, 128, "silu"),
                                               (1024, 2048, 3, 64, "none"),
                                               (512, 1024, 2, 32, "residual"),
                                               (28672, 4096, 4, 128, "silu")])
def test_rmsnorm_linear_matches_two_launches(N, K, bits, group, ep):
    """qlin_rmsnorm_linear_ep_f16 (one token row: every block reduces the sum of squares, rounds
    RN16(w * (x * r)) as the reference's norm output and multiplies that) against the two launches
    it replaces (qlin_rmsnorm_f16, then the packed linear): the same rounding point, the sum of
    squares in another fp32 order (an fp16 ulp of the normed x may move) — outputs within 2e-3 of
    max |y|, and no less accurate against a float64 evaluation of the norm + linear on the same
    W_dq than the two launches."""
    qw, qsz, fl = _packed(N, K, 21, bits, group)
    rs = np.random.RandomState(N + K)
    x = t((rs.randn(1, 1, K) * 3).astype(np.float16))
    w = torch.tensor((1 + 0.1 * rs.randn(K)).astype(np.float32), device="cuda")
    epc = {"none": qlin.EP_NONE, "residual": qlin.EP_RESIDUAL, "silu": qlin.EP_SILU_MUL}[ep]
    ny = N // 2 if ep == "silu" else N
    res = t(rs.randn(1, 1, ny).astype(np.float16)) if ep == "residual" else None
    assert qlin.rmsnorm_linear_supported(1, N, K, bits, group)
    xn = qlin.rmsnorm(x, w, 1e-5)
    ref = qlin.linear_ep(xn, qw, qsz, None, N, K, bits, group, fl, epilogue=epc, residual=res)
    got = qlin.rmsnorm_linear_ep(x, w, 1e-5, qw, qsz, None, N, K, bits, group, fl, epilogue=epc,
                                 residual=res)
    assert got.shape == ref.shape
    scale = ref.float().abs().max().item()
    assert (got.float() - ref.float()).abs().max().item() <= 2e-3 * scale
    # float64: RMSNorm (fp32 statistics as the reference) and the product on the exact W_dq
    wdq = qlin.dequant(qw, qsz, N, K, bits, group, fl).double()
    x64 = x.double().reshape(-1)
    xn = w.double() * x64 * torch.rsqrt((x64 * x64).mean() + 1e-5)
    y64 = xn @ wdq.T
    if ep == "silu":
        g, u = y64.view(-1, 2, 8)[:, 0].reshape(-1), y64.view(-1, 2, 8)[:, 1].reshape(-1)
        y64 = g * torch.sigmoid(g) * u
    if res is not None:
        y64 = y64 + res.double().reshape(-1)
    err = lambda a: (a.double().reshape(-1) - y64).abs().max().item()  # noqa: E731
    assert err(got) <= 1.25 * err(ref) + 1e-3 * scale, (err(got), err(ref))


@pytest.mark.parametrize("xs,ws,outliers", [(1e-3, 1.0, False), (1e3, 1.0, True),
                                            (1.0, 20.0, True), (30.0, 1.0, True)])
def test_rmsnorm_linear_extreme_scales(xs, ws, outliers):
    """The fused norm + linear where fp16 is tight: tiny inputs (normed values near the fp16
    subnormals before the rsqrt), huge inputs with massive-activation channels, enlarged norm
    weights (LET smoothing folds scales into them): finite and within 2e-3 of max |y| of the two
    launches, whose rounding point (RN16(w * (x * r)), quant/omni_norm.py:54-63) it shares."""
    N, K = 4096, 4096
    qw, qsz, fl = _packed(N, K, 23, 4, 128)
    rs = np.random.RandomState(7)
    xv = rs.randn(K) * xs
    if outliers:
        xv[rs.choice(K, 6, replace=False)] *= 40.0
    xv = np.clip(xv, -6e4, 6e4)
    x = t(xv.astype(np.float16).reshape(1, 1, K))
    w = torch.tensor(((1 + 0.1 * rs.randn(K)) * ws).astype(np.float32), device="cuda")
    xn = qlin.rmsnorm(x, w, 1e-5)
    ref = qlin.linear_ep(xn, qw, qsz, None, N, K, 4, 128, fl)
    got = qlin.rmsnorm_linear_ep(x, w, 1e-5, qw, qsz, None, N, K, 4, 128, fl)
    assert torch.isfinite(got).all() and torch.isfinite(ref).all()
    scale = ref.float().abs().max().item()
    assert (got.float() - ref.float()).abs().max().item() <= 2e-3 * scale


@pytest.mark.parametrize("N,K,bits,group,ep,offset", [(28672, 4096, 4, 128, "silu", 0),   # whole-row
                                                      (28672, 4096, 4, 128, "silu", 2),   # unaligned
                                                      (6144, 4096, 4, 128, "none", 0),    # fast
                                                      (4096, 14336, 4, 128, "residual", 0),  # rows
                                                      (512, 1024, 2, 32, "residual", 0),
                                                      (1024, 2048, 3, 64, "none", 0)])
def test_rmsnorm_linear_fp16_norm_weight(N, K, bits, group, ep, offset):
    """QLIN_NORM_W16: the module's fp16 norm weight read as fp16 gives the output of its fp32 copy
    bit for bit on every M = 1 route (the whole-row, fast and rows kernels; a weight only 4-B
    aligned leaves the whole-row kernel, which reads 16-B chunks)."""
    qw, qsz, fl = _packed(N, K, 29, bits, group)
    rs = np.random.RandomState(N + K + offset)
    x = t((rs.randn(1, 1, K) * 3).astype(np.float16))
    w16 = torch.tensor((1 + 0.1 * rs.randn(K + offset)).astype(np.float16), device="cuda")[offset:]
    epc = {"none": qlin.EP_NONE, "residual": qlin.EP_RESIDUAL, "silu": qlin.EP_SILU_MUL}[ep]
    ny = N // 2 if ep == "silu" else N
    res = t(rs.randn(1, 1, ny).astype(np.float16)) if ep == "residual" else None
    # the fp32 copy at the same offset (8-B aligned at offset 2): the same route as w16
    w32 = torch.cat([torch.zeros(offset, device="cuda"), w16.float()])[offset:]
    ref = qlin.rmsnorm_linear_ep(x, w32, 1e-5, qw, qsz, None, N, K, bits, group, fl,
                                 epilogue=epc, residual=res)
    got = qlin.rmsnorm_linear_ep(x, w16, 1e-5, qw, qsz, None, N, K, bits, group, fl,
                                 epilogue=epc, residual=res)
    assert torch.equal(got, ref)


def test_rmsnorm_linear_rejects_unsupported():
    qw, qsz, fl = _packed(256, 1024, 5)
    w = torch.ones(1024, device="cuda")
    assert not qlin.rmsnorm_linear_supported(2, 256, 1024, 4, 128)  # one token row only
    assert not qlin.rmsnorm_linear_supported(1, 256, 1000, 4, 40)   # K % 128
    x2 = t(np.ones((2, 1024), np.float16))
    with pytest.raises(ValueError):
        qlin.rmsnorm_linear_ep(x2, w, 1e-5, qw, qsz, None, 256, 1024, 4, 128, fl)
