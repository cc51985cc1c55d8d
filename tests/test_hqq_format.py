"""HQQ weight format (BASELINE configs[3]): the product's unpacker and converter
(quant/hqq.py) against the oracle's restated hqq Quantizer / BitPack (oracle/hqq_format.py).
hqq is neither installed nor vendored: PARITY UNPINNED against the real library — these tests pin
the two restatements to each other and the fp16 dequant identity, nothing more."""
import numpy as np
import pytest
import torch

from helpers import assert_close_to_ref, bit_equal, n, rand_weight, rand_x, t
from oracle import hqq_format as OH
from oracle import quant_oracle as O
from quant import hqq


@pytest.mark.parametrize("nbits", [2, 3, 4, 8])
@pytest.mark.parametrize("rows", [40, 37])
def test_bitpack_roundtrip(nbits, rows):
    if nbits in (2, 4) and rows % 4:
        pytest.skip("hqq's u8 packers need rows divisible by the codes per byte")
    rs = np.random.RandomState(nbits * rows)
    W = rs.randint(0, 2 ** nbits, size=(rows, 64)).astype(np.uint8)
    P = OH.pack(W, nbits)
    assert np.array_equal(OH.unpack(P, nbits)[:rows], W)
    got = hqq.unpack(torch.from_numpy(P), nbits)[:rows]
    assert np.array_equal(got.numpy(), W)


def test_quantize_restatement_bounds():
    w = rand_weight(64, 256, seed=1)
    for nbits in (2, 3, 4, 8):
        W_q, s, z, shape = OH.quantize(w, nbits, 64, axis=1)
        assert W_q.shape == (64 * 256 // 64, 64) and W_q.max() <= 2 ** nbits - 1
        w_r = OH.dequantize(OH.pack(W_q, nbits), s, z, nbits, 64, shape)
        # RTN error bound: half a step of each group (plus fp16 rounding of scale / zero)
        step = s.astype(np.float32).reshape(64, 4).repeat(64, axis=1)
        assert np.all(np.abs(w_r.astype(np.float32) - w.astype(np.float32)) <= 0.75 * step + 1e-3)


def test_unsupported_meta_rejected():
    W_q = torch.zeros(8, 64, dtype=torch.uint8)
    meta = dict(nbits=4, group_size=64, shape=(4, 256), axis=0, scale=torch.ones(16),
                zero=torch.zeros(16))
    with pytest.raises(NotImplementedError):
        hqq.hqq_to_qlin(W_q, meta)
    meta.update(axis=1)
    del meta["zero"]
    with pytest.raises(NotImplementedError):
        hqq.hqq_to_qlin(W_q, meta)
    meta.update(zero=torch.zeros(16), group_size=48)
    with pytest.raises(ValueError):
        hqq.hqq_to_qlin(W_q, meta)


def _hqq_linear(N, K, nbits, group, seed, round_zero=False):
    w = rand_weight(N, K, seed=seed)
    W_q, s, z, shape = OH.quantize(w, nbits, group, axis=1, round_zero=round_zero)
    packed = OH.pack(W_q, nbits)
    meta = dict(nbits=nbits, group_size=group, shape=shape, axis=1, packing=OH.PACKING[nbits],
                scale=torch.from_numpy(s.reshape(-1, 1)), zero=torch.from_numpy(z.reshape(-1, 1)))
    ref_w = OH.dequantize(packed, s, z, nbits, group, shape)
    return torch.from_numpy(packed), meta, ref_w


@pytest.mark.gpu
@pytest.mark.parametrize("nbits,group", [(4, 64), (3, 64), (2, 64), (4, 128), (8, 128), (2, 32)])
def test_hqq_conversion_dequant_bit_exact(nbits, group):
    """Converted layer's W_dq == hqq's fp16 ((W_q - zero) * scale) bit for bit; GEMV and GEMM
    (QLIN_FLOAT_ZERO kernels) match x @ W^T in fp64."""
    N, K = 400, 1024
    W_q, meta, ref_w = _hqq_linear(N, K, nbits, group, seed=nbits + group)
    ql = hqq.packed_quant_linear(W_q, meta)
    assert ql.qflags & 16
    assert bit_equal(n(ql.dequantized_weight()), ref_w)
    for M in (1, 5, 16, 40, 300):
        x = rand_x(M, K, seed=M)
        y = ql(t(x).unsqueeze(0))[0]
        assert_close_to_ref(n(y), O.linear_ref(x, ref_w), what=f"int{nbits} g{group} M={M}")


@pytest.mark.gpu
def test_hqq_round_zero_and_view_as_float():
    N, K, nbits, group = 64, 512, 4, 128
    W_q, meta, ref_w = _hqq_linear(N, K, nbits, group, seed=7, round_zero=True)
    meta["view_as_float"] = True
    ql = hqq.packed_quant_linear(W_q.view(torch.float16), meta)
    assert bit_equal(n(ql.dequantized_weight()), ref_w)


@pytest.mark.gpu
def test_pack_codes_matches_oracle_packer():
    from quant import qlin
    rs = np.random.RandomState(3)
    for bits in (2, 3, 4, 8):
        N, K = 40, 96 + 128  # ragged: last row tile and last k-tile partial
        u = rs.randint(0, 2 ** bits, size=(N, K)).astype(np.uint8)
        qw = qlin.pack_codes(t(u), bits)
        ref = O.pack_qweight(u.astype(np.uint32), bits)
        assert np.array_equal(n(qw).view(np.uint32), ref.reshape(n(qw).shape)), bits


@pytest.mark.gpu
@pytest.mark.parametrize("nbits,N,K", [(3, 28672, 4096), (2, 4096, 14336)])
def test_hqq_conversion_llama_widths(nbits, N, K):
    """configs[3] at LLaMA3-8B widths: an HQQ int3 gate/up-wide matrix (28,672 x 4,096, the
    work-queue route at one token) and an int2 down-shaped matrix (4,096 x 14,336, the long-K
    rows route), g64: the converted W_dq is hqq's fp16 ((W_q - zero) * scale) bit for bit, and
    the decode (M = 1) and a 16-row product match x @ W_dq^T in fp64."""
    from quant import qlin
    group = 64
    W_q, meta, ref_w = _hqq_linear(N, K, nbits, group, seed=nbits * 7 + 1)
    ql = hqq.packed_quant_linear(W_q, meta)
    assert ql.qflags & 16
    assert bit_equal(n(ql.dequantized_weight()), ref_w)
    assert qlin.m1_route(N, K, nbits, group) in (qlin.M1_WHOLE_ROW, qlin.M1_ROWS)
    for M in (1, 16):
        x = rand_x(M, K, seed=M + nbits)
        y = ql(t(x).unsqueeze(0))[0]
        assert_close_to_ref(n(y), O.linear_ref(x, ref_w), what=f"hqq int{nbits} {N}x{K} M={M}")


@pytest.mark.gpu
@pytest.mark.parametrize("nbits,N", [(3, 512), (2, 528)])
def test_hqq_batched_bit_identical_to_gemm(nbits, N):
    """configs[3]'s batched rings with hqq's fp16 zeros (the streaming kernel's float-zero
    instances; even and odd tile-row counts): every product bit-identical to qlin_gemm_f16 unsplit
    and close to x @ W_dq^T in fp64."""
    from quant import qlin
    K, group, B = 2048, 64, 3
    convs, refs = [], []
    for b in range(B):
        W_q, meta, ref_w = _hqq_linear(N, K, nbits, group, seed=100 * nbits + b)
        convs.append(hqq.hqq_to_qlin(W_q.cuda(), {k: (v.cuda() if torch.is_tensor(v) else v)
                                                     for k, v in meta.items()}))
        refs.append(ref_w)
    fl = convs[0]["flags"]
    assert fl & qlin.FLOAT_ZERO
    qw = torch.stack([c["qweight"] for c in convs])
    qsz = torch.stack([c["qsz"] for c in convs])
    x = np.stack([rand_x(1, K, seed=7 + b) for b in range(B)])
    y = qlin.gemv_batched(t(x), qw, qsz, None, N, K, nbits, group, fl)
    for b in range(B):
        yb = qlin.gemm(t(x[b]), qw[b], qsz[b], None, N, K, nbits, group, fl, split=False)
        assert bit_equal(n(y[b]), n(yb)), f"problem {b}"
        assert_close_to_ref(n(y[b]), O.linear_ref(x[b], refs[b]), what=f"hqq batched b{nbits} {b}")
