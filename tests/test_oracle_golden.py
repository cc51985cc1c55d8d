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
def test_pack_roundtrip(bits):
    rs = np.random.RandomState(bits)
    u = rs.randint(0, 2 ** bits, size=(7, 256)).astype(np.uint32)
    qw = O.pack_qweight(u, bits)
    assert qw.shape == (7, 256 * bits // 32) and qw.dtype == np.uint32
    np.testing.assert_array_equal(O.unpack_qweight(qw, bits, 256), u)


def test_pack_layout_int4_known_answer():
    # element k of a chunk: word k//8, pair p=(k%8)//2, half h=k%2 -> bit 16h + 4p
    u = np.arange(32, dtype=np.uint32)[None, :] % 16
    qw = O.pack_qweight(u, 4)
    w0 = 0
    for k in range(8):
        w0 |= (k % 16) << (16 * (k % 2) + 4 * (k // 2))
    assert int(qw[0, 0]) == w0
    # the fp16 magic unpack: ((w >> 4p) & 0x000F000F) | 0x64006400 -> (1024+u[2p], 1024+u[2p+1])
    for p in range(4):
        v = ((int(qw[0, 0]) >> (4 * p)) & 0x000F000F) | 0x64006400
        lo = np.array([v & 0xFFFF], dtype=np.uint16).view(np.float16)[0]
        hi = np.array([v >> 16], dtype=np.uint16).view(np.float16)[0]
        assert (lo, hi) == (1024 + 2 * p, 1024 + 2 * p + 1)


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
    qw, sc, z = O.pack_from_quant(x_int, scale, zp, p["n_bits"], N, K, p["group_size"],
                                  p["disable_zero_point"])
    assert z.dtype in (np.int8, np.int16)
    dq = O.dequant_packed(qw, sc, z, p["n_bits"], K, p["group_size"])
    assert bit_equal(dq[ok], g["w_dq"][ok])
    # real-quant packer contract: recover codes from (W_dq, scales, zeros) alone
    qw2, sc2, z2 = O.pack_from_dequant(np.where(ok[:, None], g["w_dq"], 0).astype(np.float16),
                                       scale, zp, p["n_bits"], p["group_size"],
                                       p["disable_zero_point"])
    dq2 = O.dequant_packed(qw2, sc2, z2, p["n_bits"], K, p["group_size"])
    assert bit_equal(dq2[ok], g["w_dq"][ok])


def test_wide_zero_uses_int16():
    g = load_golden("q_w3g64_f16")
    _, scale, zp, x_int = O.quantize(g["w"], 3, 64)
    _, _, z = O.pack_from_quant(np.nan_to_num(x_int), scale, zp, 3, 64, 512, 64)
    assert z.dtype == np.int16 and z.min() == -10000


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
