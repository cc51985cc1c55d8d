"""Pin the CPU oracle (oracle/quant_oracle.py) against the reference's own outputs.

The golden vectors were produced by running the reference's quant/quantizer.py, quant/int_linear.py
and quant/int_matmul.py (tests/golden/make_golden.py).  Everything here is bit-exact except the
F.linear / matmul outputs, whose accumulation order is the reference BLAS's.
"""
import numpy as np
import pytest

from conftest import load_golden
from oracle import quant_oracle as O

WEIGHT_CASES = ["q_w4g128_f16", "q_w3g64_f16", "q_w2g64_f16", "q_w8pc_f16", "q_w4pc_f16_k4096",
                "q_w4g128_sym_f16", "q_w4g128_nozp_f16", "q_w8g128_nozp_f16",
                "q_w4g128_lwc16_f16", "q_w4g128_lwc32_f16", "q_w4g128_f32",
                "q_w3g64_symlwc_def_f16"]


def params(g):
    p = dict(n_bits=int(g["p_n_bits"]))
    gs = int(g["p_group_size"]) if "p_group_size" in g else -1
    p["group_size"] = None if gs < 0 else gs
    p["symmetric"] = bool(g.get("p_symmetric", False))
    p["disable_zero_point"] = bool(g.get("p_disable_zero_point", False))
    return p


def bit_equal(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape and a.dtype == b.dtype, (a.shape, b.shape, a.dtype, b.dtype)
    return np.array_equal(a.view(np.uint8), b.view(np.uint8)) or \
        np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("name", WEIGHT_CASES)
def test_quantizer_bit_exact(name):
    g = load_golden(name)
    p = params(g)
    w_dq, scale, zp, _ = O.quantize(g["w"], p["n_bits"], p["group_size"], p["symmetric"],
                                    p["disable_zero_point"], g.get("lwc_up"), g.get("lwc_low"),
                                    int(g["deficiency"]))
    assert bit_equal(scale, g["scale"])
    if "zp" in g:
        assert bit_equal(zp, g["zp"])
    else:
        assert zp is None
    assert bit_equal(w_dq, g["w_dq"]), f"{name}: {np.sum(w_dq != g['w_dq'])} mismatches"


def test_golden_exercises_hard_groups():
    g = load_golden("q_w3g64_f16")
    assert np.isnan(g["w_dq"][3, :64]).all()          # x/s overflow -> NaN via round_ste
    assert (g["zp"] < 0).any()                        # all-positive group
    assert g["zp"].min() == -1e4                      # clamped wide zero point
    assert (g["scale"] == np.float16(1e-5)).any()     # CLIPMIN


@pytest.mark.parametrize("name", ["q_a8tok_f16", "q_a4tok_f16", "q_a8tok_f32"])
def test_act_per_token_bit_exact(name):
    g = load_golden(name)
    x_dq, scale, zp, _ = O.quantize(g["x"], int(g["p_n_bits"]), None)
    assert bit_equal(scale, g["scale"]) and bit_equal(zp, g["zp"])
    assert bit_equal(x_dq, g["x_dq"])


@pytest.mark.parametrize("bits", [2, 3, 4, 8])
@pytest.mark.parametrize("shape", [(7, 256), (16, 128), (33, 96), (48, 4096)])
def test_pack_roundtrip(bits, shape):
    rs = np.random.RandomState(bits)
    u = rs.randint(0, 2 ** bits, size=shape).astype(np.uint32)
    qw = O.pack_qweight(u, bits)
    assert qw.shape == O.tiled_shape(*shape, bits) and qw.dtype == np.uint32
    np.testing.assert_array_equal(O.unpack_qweight(qw, bits, *shape), u)


def _f16(v):
    return float(np.array([v & 0xFFFF], dtype=np.uint16).view(np.float16)[0])


MAGIC = {1024: 0x64006400, 256: 0x5C005C00, 64: 0x54005400, 16: 0x4C004C00}


def kernel_extract(words, bits, s):
    """The GEMV kernel's unpack of k-step s of one lane piece (qlin_common.h), simulated bit for bit:
    returns the 8 fp16 values (off_j + u_j) and the offsets off_j."""
    w = [int(x) for x in words]
    pairs = []
    if bits == 4:
        ws = w[s]
        for sh, mask, off in ((0, 0x000F000F, 1024), (0, 0x00F000F0, 64), (8, 0x000F000F, 1024),
                              (8, 0x00F000F0, 64)):
            pairs.append((((ws >> sh) & mask) | MAGIC[off], off))
    elif bits == 8:
        for ww in (w[2 * s], w[2 * s + 1]):
            for sh in (0, 8):
                pairs.append((((ww >> sh) & 0x00FF00FF) | MAGIC[1024], 1024))
    else:
        ws = w[s >> 1] >> (8 * (s & 1))
        hs = ((w[2] >> O.RHO3[s]) | (w[2] << (32 - O.RHO3[s]))) & 0xFFFFFFFF if bits == 3 else 0
        for p, off in enumerate((1024, 256, 64, 16)):
            v = (ws & (0x00030003 << (2 * p))) | MAGIC[off]
            if bits == 3:
                v |= hs & (0x00040004 << (2 * p))
            pairs.append((v, off))
    vals, offs = [], []
    for v, off in pairs:
        vals += [_f16(v), _f16(v >> 16)]
        offs += [off, off]
    return vals, offs


@pytest.mark.parametrize("bits", [2, 3, 4, 8])
def test_magic_unpack_known_answer(bits):
    """Every code of every lane piece decodes to exactly off + u with the kernel's bit operations,
    and lane l = n + 16q, step s, element j is the code of row n at k = 32s + 8q + j."""
    rs = np.random.RandomState(100 + bits)
    N, K = 16, 128
    u = rs.randint(0, 2 ** bits, size=(N, K)).astype(np.uint32)
    qw = O.pack_qweight(u, bits)[0, 0]
    for lane in range(64):
        n, q = lane & 15, lane >> 4
        for s in range(4):
            vals, offs = kernel_extract(qw[lane], bits, s)
            for j in range(8):
                assert vals[j] - offs[j] == u[n, 32 * s + 8 * q + j], (lane, s, j)


@pytest.mark.parametrize("name", ["q_w4g128_f16", "q_w3g64_f16", "q_w2g64_f16", "q_w8pc_f16",
                                  "q_w4g128_sym_f16", "q_w4g128_nozp_f16", "q_w8g128_nozp_f16",
                                  "q_w4g128_lwc16_f16"])
def test_dequant_packed_matches_reference(name):
    """packed (qweight, fp16 scales, int zeros) -> W_dq reproduces the reference W_dq bit-exactly
    (NaN rows excluded: the packed format has no NaN code)."""
    g = load_golden(name)
    p = params(g)
    N, K = g["w"].shape
    w_dq, scale, zp, x_int = O.quantize(g["w"], p["n_bits"], p["group_size"], p["symmetric"],
                                        p["disable_zero_point"], g.get("lwc_up"), g.get("lwc_low"))
    ok = ~np.isnan(w_dq).any(axis=1)
    x_int = np.nan_to_num(x_int)
    qw, qsz, wide = O.pack_from_quant(x_int, scale, zp, p["n_bits"], N, K, p["group_size"],
                                      p["disable_zero_point"])
    sc, z = O.unpack_sz(qsz, N)
    assert bit_equal(sc.reshape(-1, 1), scale.astype(np.float16))
    dq = O.dequant_packed(qw, qsz, p["n_bits"], N, K, p["group_size"])
    assert bit_equal(dq[ok], g["w_dq"][ok])
    # real-quant packer contract: recover codes from (W_dq, scales, zeros) alone
    qw2, qsz2, _ = O.pack_from_dequant(np.where(ok[:, None], g["w_dq"], 0).astype(np.float16),
                                       scale, zp, p["n_bits"], p["group_size"],
                                       p["disable_zero_point"])
    dq2 = O.dequant_packed(qw2, qsz2, p["n_bits"], N, K, p["group_size"])
    assert bit_equal(dq2[ok], g["w_dq"][ok])


def test_wide_zero_flag():
    g = load_golden("q_w3g64_f16")
    _, scale, zp, x_int = O.quantize(g["w"], 3, 64)
    _, qsz, wide = O.pack_from_quant(np.nan_to_num(x_int), scale, zp, 3, 64, 512, 64)
    assert wide and O.unpack_sz(qsz, 64)[1].min() == -10000
    g = load_golden("q_w4g128_f16")
    _, scale, zp, x_int = O.quantize(g["w"], 4, 128)
    assert not O.pack_from_quant(np.nan_to_num(x_int), scale, zp, 4, 64, 512, 128)[2]


def test_sz_layout_roundtrip():
    rs = np.random.RandomState(0)
    sc = (rs.rand(37, 5) * 0.01).astype(np.float16)
    z = rs.randint(-3000, 3000, size=(37, 5))
    q = O.pack_sz(sc, z)
    assert q.shape == (3, 5, 16)
    s2, z2 = O.unpack_sz(q, 37)
    assert bit_equal(s2, sc) and np.array_equal(z2, z)
    assert int(q[1, 2, 3]) == (int(sc[19, 2].view(np.uint16)) | ((int(z[19, 2]) & 0xFFFF) << 16))


@pytest.mark.parametrize("tag", ["f16", "f32"])
def test_quant_linear_forward(tag):
    g = load_golden(f"lin_w4g128_{tag}")
    w_dq, *_ = O.quantize(g["w"], 4, 128)
    for xk, yk in (("x1", "y1"), ("x8", "y8")):
        y = O.linear_ref(g[xk], w_dq, g["b"])
        tol = 2e-3 if tag == "f16" else 1e-5
        np.testing.assert_allclose(y, g[yk].astype(np.float64), rtol=0, atol=tol * np.abs(y).max())
    xq, *_ = O.quantize(g["x8"], 8, None)
    y = O.linear_ref(xq, w_dq, g["b"])
    tol = 2e-3 if tag == "f16" else 1e-5
    np.testing.assert_allclose(y, g["y8_a8"].astype(np.float64), rtol=0, atol=tol * np.abs(y).max())


def test_quant_matmul_act_quant():
    g = load_golden("mm_a8_f32")
    np.testing.assert_allclose(g["x1"] @ g["x2"], g["y"], rtol=1e-5, atol=1e-5)
    a, *_ = O.quantize(g["x1"], 8, None)
    b, *_ = O.quantize(g["x2"], 8, None)
    np.testing.assert_allclose(a @ b, g["y_a8"], rtol=1e-5, atol=1e-5)


TORCH_REF_CASES = ["q_w4g128_f16", "q_w3g64_f16", "q_w2g64_f16", "q_w8pc_f16", "q_w4pc_f16_k4096",
                   "q_w4g128_sym_f16", "q_w4g128_nozp_f16", "q_w8g128_nozp_f16", "q_w4g128_f32"]


@pytest.mark.parametrize("name", TORCH_REF_CASES)
def test_torch_cpu_restatement_bit_exact(name):
    """oracle/torch_ref.py (the bench's CPU baseline: the reference's fake-quant op sequence in
    torch on the host) reproduces the reference's W_dq / scale / zp bit for bit."""
    import torch
    from oracle import torch_ref as TR
    g = load_golden(name)
    p = params(g)
    w_dq, scale, zp = TR.quantize(torch.from_numpy(g["w"]), p["n_bits"], p["group_size"],
                                  p["symmetric"], p["disable_zero_point"])
    assert bit_equal(w_dq.numpy(), g["w_dq"]), name
    assert bit_equal(scale.numpy().reshape(g["scale"].shape), g["scale"]), name
    if "zp" in g and zp is not None:
        assert bit_equal(zp.numpy().reshape(g["zp"].shape), g["zp"]), name
