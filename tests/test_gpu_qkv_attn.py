"""The fused input-RMSNorm + q/k/v + RoPE + KV append + decode attention launch
(``qlin_qkv_attn_decode_f16``, csrc/qlin_decode_fused.hip) against the two launches it replaces —
``qlin_rmsnorm_linear_ep_f16`` (q/k/v) then ``qlin_attn_decode_rope`` / ``_rope_len`` — and against
a float64 evaluation of the reference attention (models/int_llama_layer.py:113-165).

The q/k/v rows it writes and the cache row it appends are bit-identical to the two launches (the
same GEMV body and RoPE arithmetic); the attention output agrees to fp32 rounding (its rows split
into 64-row chunks, the two-launch path's by its own split choice) and is held to the float64
reference like the two-launch path."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from quant import qlin  # noqa: E402

H, HQ, HKV, D = 4096, 32, 8, 128
N = (HQ + 2 * HKV) * D


def _rope():
    from models.int_llama_layer import LlamaRotaryEmbedding437
    rot = LlamaRotaryEmbedding437(D, 8192, 500000.0, device="cuda").half()
    return rot.cos_cached.float().contiguous(), rot.sin_cached.float().contiguous()


def _case(bits, group, seed, hqq=False):
    g = torch.Generator(device="cuda").manual_seed(seed)
    w = (torch.randn(N, H, device="cuda", generator=g) * 0.02).half()
    o = qlin.quantize(w, bits, group, 0, want_xdq=False, want_params=False, pack=True)
    qw, qsz, fl = o["qweight"], o["qsz"], o["flags"]
    if hqq:
        sc, zi = qlin.split_sz(qsz, N)
        qsz = qlin.join_sz_float(sc, zi.to(torch.float16) + 0.375)
        fl = qlin.FLOAT_ZERO
    x = (torch.randn(1, 1, H, device="cuda", generator=g) * 1.5).half()
    nw = (1.0 + 0.1 * torch.randn(H, device="cuda", generator=g)).half()
    return qw, qsz, fl, x, nw, g


def _ref64(qkv, kc, vc, L, pos, cos, sin, mask):
    """The reference attention of the step in float64 from the q/k/v rows (RoPE with the fp16
    cos / sin as the reference casts them; k rounded to fp16 after RoPE as the cache holds it)."""
    q, k, v = torch.split(qkv.double().reshape(-1), [HQ * D, HKV * D, HKV * D])
    c = cos[pos].half().double()
    s_ = sin[pos].half().double()

    def rot(x):
        x1, x2 = x[..., : D // 2], x[..., D // 2:]
        return x * c + torch.cat((-x2, x1), -1) * s_
    q = rot(q.view(HQ, D))
    K = kc[0, :, :L].double().clone()
    V = vc[0, :, :L].double().clone()
    K[:, L - 1] = rot(k.view(HKV, D)).half().double()
    V[:, L - 1] = v.view(HKV, D)
    Kq, Vq = K.repeat_interleave(HQ // HKV, 0), V.repeat_interleave(HQ // HKV, 0)
    sc = torch.einsum("hd,hld->hl", q, Kq) / math.sqrt(D)
    if mask is not None:
        sc = sc + mask.reshape(1, L).double()
    return torch.einsum("hl,hld->hd", torch.softmax(sc, -1), Vq)


@pytest.mark.parametrize("bits,group,hqq", [(4, 128, False), (2, 64, False), (3, 64, True),
                                            (8, 128, False), (4, 32, False)])
@pytest.mark.parametrize("kv0,rows,masked", [(512, 1024, False), (0, 256, False), (63, 128, True),
                                             (64, 128, False), (1999, 2048, True),
                                             (4095, 4096, False)])
def test_qkv_attn_equals_two_launches(bits, group, hqq, kv0, rows, masked):
    cos, sin = _rope()
    qw, qsz, fl, x, nw, g = _case(bits, group, 1000 * bits + kv0 + group, hqq)
    L = kv0 + 1
    kc = torch.randn(1, HKV, rows, D, device="cuda", generator=g).half()
    vc = torch.randn(1, HKV, rows, D, device="cuda", generator=g).half()
    kc2, vc2 = kc.clone(), vc.clone()
    pos = torch.tensor([[kv0]], device="cuda")
    mask = None
    if masked:
        mask = torch.zeros(1, 1, 1, L, device="cuda", dtype=torch.float16)
        mask[..., : kv0 // 3] = torch.finfo(torch.float16).min
    assert qlin.qkv_attn_supported(HQ, HKV, D, H, bits, group, fl, L)
    out, qkv = qlin.qkv_attn_decode(x, nw, 1e-5, qw, qsz, fl, bits, group, cos, sin, pos, HQ, HKV,
                                    D, kc, vc, kv0=kv0, mask=mask)
    ref_qkv = qlin.rmsnorm_linear_ep(x, nw, 1e-5, qw, qsz, None, N, H, bits, group, fl)
    assert torch.equal(qkv, ref_qkv)  # the same GEMV body, stores handed off as pairs
    q, k, v = torch.split(ref_qkv, [HQ * D, HKV * D, HKV * D], dim=-1)
    ref = qlin.attn_decode_rope(q, k, v, cos, sin, pos, HQ, HKV, D, kc2, vc2, kv0, mask,
                                math.sqrt(D), out_dtype=torch.float16)
    assert torch.equal(kc, kc2) and torch.equal(vc, vc2)  # the appended row and nothing else
    r64 = _ref64(ref_qkv, kc2, vc2, L, kv0, cos, sin, mask)
    scale = r64.abs().max().item()
    e_f = (out[0, :, 0].double() - r64).abs().max().item() / scale
    e_t = (ref[0, :, 0].double() - r64).abs().max().item() / scale
    # both are the fp32 attention rounded once to fp16 (half an fp16 ulp relative: 4.9e-4)
    assert e_f <= 1e-3 and e_t <= 1e-3, (e_f, e_t)
    assert (out.float() - ref.float()).abs().max().item() <= 1e-3 * max(1.0, scale)


def test_qkv_attn_device_length_graph_replay():
    """The device-length form (graph-replayed decode steps): one capture, several replays with
    the length and position advanced on the device, each equal to the host-length launch of the
    same step bit for bit (same 64-row split), the cache rows appended step by step."""
    cos, sin = _rope()
    qw, qsz, fl, x, nw, g = _case(4, 128, 77)
    cap, kv0 = 600, 500
    kc = torch.randn(1, HKV, cap, D, device="cuda", generator=g).half()
    vc = torch.randn(1, HKV, cap, D, device="cuda", generator=g).half()
    kc2, vc2 = kc.clone(), vc.clone()
    length = torch.tensor([kv0 + 1], dtype=torch.int32, device="cuda")
    pos = torch.tensor([[kv0]], device="cuda")
    xs = (torch.randn(4, 1, 1, H, device="cuda", generator=g) * 1.5).half()
    xin = xs[0].clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        qlin.qkv_attn_decode(xin, nw, 1e-5, qw, qsz, fl, 4, 128, cos, sin, pos, HQ, HKV, D,
                             kc, vc, length=length, max_len=cap)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            out, _ = qlin.qkv_attn_decode(xin, nw, 1e-5, qw, qsz, fl, 4, 128, cos, sin, pos, HQ,
                                          HKV, D, kc, vc, length=length, max_len=cap)
    torch.cuda.current_stream().wait_stream(s)
    for step in range(4):
        xin.copy_(xs[step])
        length.fill_(kv0 + 1 + step)
        pos.fill_(kv0 + step)
        graph.replay()
        ref, _ = qlin.qkv_attn_decode(xs[step], nw, 1e-5, qw, qsz, fl, 4, 128, cos, sin, pos, HQ,
                                      HKV, D, kc2, vc2, kv0=kv0 + step)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), step
        assert torch.equal(kc[:, :, :kv0 + step + 1], kc2[:, :, :kv0 + step + 1]), step
        assert torch.equal(vc[:, :, :kv0 + step + 1], vc2[:, :, :kv0 + step + 1]), step


def test_qkv_attn_counters_left_zero_and_rejects():
    """Every call leaves the merge and hand-off counters zero (graph replays need no memset);
    shapes the launch does not take are refused, never launched."""
    cos, sin = _rope()
    qw, qsz, fl, x, nw, g = _case(4, 128, 5)
    kc = torch.randn(1, HKV, 256, D, device="cuda", generator=g).half()
    vc = torch.randn(1, HKV, 256, D, device="cuda", generator=g).half()
    pos = torch.tensor([[200]], device="cuda")
    for _ in range(3):
        qlin.qkv_attn_decode(x, nw, 1e-5, qw, qsz, fl, 4, 128, cos, sin, pos, HQ, HKV, D, kc, vc,
                             kv0=200)
    torch.cuda.synchronize()
    cnt = qlin._attn_counters(torch.device("cuda", torch.cuda.current_device()), 2 * HKV)
    assert int(cnt[: 2 * HKV].abs().sum()) == 0
    assert not qlin.qkv_attn_supported(32, 32, 128, 4096, 4, 128, 0, 100)  # MHA: two launches
    assert not qlin.qkv_attn_supported(HQ, HKV, 128, 4096, 4, 128, 0, 5000)  # beyond 4096 rows
    with pytest.raises(ValueError):
        qlin.qkv_attn_decode(x, nw.float(), 1e-5, qw, qsz, fl, 4, 128, cos, sin, pos, HQ, HKV, D,
                             kc, vc, kv0=200)
