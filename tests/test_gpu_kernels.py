"""GPU parity: the gfx950 kernels (through the C ABI) against the oracle and the reference's
golden vectors.  Bit-exact for quantize / pack / dequant; fp16-output tolerance for GEMV / GEMM."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from helpers import assert_close_to_ref, bit_equal, n, rand_weight, rand_x, t
from oracle import quant_oracle as O

pytestmark = pytest.mark.gpu

from quant import qlin  # noqa: E402
from quant.quantizer import UniformAffineQuantizer  # noqa: E402

WEIGHT_CASES = ["q_w4g128_f16", "q_w3g64_f16", "q_w2g64_f16", "q_w8pc_f16", "q_w4pc_f16_k4096",
                "q_w4g128_sym_f16", "q_w4g128_nozp_f16", "q_w8g128_nozp_f16",
                "q_w4g128_lwc16_f16", "q_w4g128_lwc32_f16", "q_w4g128_f32",
                "q_w3g64_symlwc_def_f16"]


def _params(g):
    gs = int(g["p_group_size"]) if "p_group_size" in g else -1
    return dict(n_bits=int(g["p_n_bits"]), group_size=None if gs < 0 else gs,
                symmetric=bool(g.get("p_symmetric", False)),
                disable_zero_point=bool(g.get("p_disable_zero_point", False)),
                lwc=bool(g.get("p_lwc", False)))


@pytest.mark.parametrize("name", WEIGHT_CASES)
def test_quantizer_kernel_matches_reference(name):
    g = load_golden(name)
    p = _params(g)
    W = t(g["w"])
    q = UniformAffineQuantizer(**p, dynamic_method="per_channel", shape=W.shape).cuda()
    if p["lwc"]:
        with torch.no_grad():
            q.upbound_factor.data = t(g["lwc_up"])
            q.lowbound_factor.data = t(g["lwc_low"])
    wdq = q(W)
    assert bit_equal(n(q.scale), g["scale"]), name
    if "zp" in g:
        assert bit_equal(n(q.round_zero_point), g["zp"]), name
    assert bit_equal(n(wdq), g["w_dq"]), f"{name}: {np.sum(n(wdq) != g['w_dq'])} mismatches"


@pytest.mark.parametrize("name", ["q_a8tok_f16", "q_a4tok_f16", "q_a8tok_f32"])
def test_act_quantizer_kernel_matches_reference(name):
    g = load_golden(name)
    q = UniformAffineQuantizer(n_bits=int(g["p_n_bits"]), dynamic_method="per_token").cuda()
    xdq = q(t(g["x"]))
    assert bit_equal(n(q.scale), g["scale"]) and bit_equal(n(q.round_zero_point), g["zp"])
    assert bit_equal(n(xdq), g["x_dq"])


def test_fake_quant_given_params_matches_reference():
    g = load_golden("q_w4g128_f16")
    q = UniformAffineQuantizer(n_bits=4, group_size=128, dynamic_method="per_channel").cuda()
    W = t(g["w"])
    out = q.fake_quant(W, t(g["scale"]), t(g["zp"]))
    assert bit_equal(n(out), g["w_dq"])


PACK_CASES = ["q_w4g128_f16", "q_w3g64_f16", "q_w2g64_f16", "q_w8pc_f16", "q_w4g128_sym_f16",
              "q_w4g128_nozp_f16", "q_w8g128_nozp_f16", "q_w4pc_f16_k4096"]


@pytest.mark.parametrize("name", PACK_CASES)
def test_pack_and_dequant_bit_exact(name):
    g = load_golden(name)
    p = _params(g)
    N, K = g["w"].shape
    grp = p["group_size"] or K
    flags = (qlin.SYMMETRIC if p["symmetric"] else 0) | (
        qlin.DISABLE_ZERO_POINT if p["disable_zero_point"] else 0)
    out = qlin.quantize(t(g["w"]), p["n_bits"], grp, flags, pack=True)
    # oracle packing of the oracle's codes
    _, scale, zp, x_int = O.quantize(g["w"], p["n_bits"], p["group_size"], p["symmetric"],
                                     p["disable_zero_point"])
    ok = ~np.isnan(g["w_dq"]).any(axis=1)
    oq, osz, owide = O.pack_from_quant(np.nan_to_num(x_int), scale, zp, p["n_bits"], N, K,
                                       p["group_size"], p["disable_zero_point"])
    gq = n(out["qweight"]).view(np.uint32)
    assert gq.shape == oq.shape
    if ok.all():
        assert np.array_equal(gq, oq)  # the kernel's packed words are the oracle's, bit for bit
    assert np.array_equal(O.unpack_qweight(gq, p["n_bits"], N, K)[ok],
                          O.unpack_qweight(oq, p["n_bits"], N, K)[ok])
    gsz = n(out["qsz"]).view(np.uint32)
    assert gsz.shape == osz.shape
    assert np.array_equal(gsz, osz)  # (scale, zero) words bit for bit
    assert (out["flags"] == qlin.WIDE_ZERO) == owide
    w = qlin.dequant(out["qweight"], out["qsz"], N, K, p["n_bits"], grp, out["flags"])
    assert bit_equal(n(w)[ok], g["w_dq"][ok])
    # the real-quant packer: codes recovered from (W_dq, scales, zeros) alone
    wdq = np.where(ok[:, None], g["w_dq"], 0).astype(np.float16)
    pz = None if p["disable_zero_point"] else t(g["zp"].reshape(-1))
    out2 = qlin.fake_quant(t(wdq), t(g["scale"].reshape(-1)), pz, p["n_bits"], grp,
                           flags & qlin.DISABLE_ZERO_POINT, want_xdq=False, pack=True)
    w2 = qlin.dequant(out2["qweight"], out2["qsz"], N, K, p["n_bits"], grp, out2["flags"])
    assert bit_equal(n(w2)[ok], g["w_dq"][ok])


def _packed(N, K, bits, group, seed, wide=False):
    """Packed operands from the HIP quantizer, and the ORACLE's W_dq of the same weight (the
    reference's UniformAffineQuantizer arithmetic restated in numpy, oracle/quant_oracle.py
    quantize): the product tests anchor on the reference's W_dq, not on the kernels' own dequant."""
    W = rand_weight(N, K, seed)
    if wide:
        W[: max(1, N // 7), :group] = 1.0 + np.random.RandomState(seed).rand(
            max(1, N // 7), group).astype(np.float16) * np.float16(1e-3)
    out = qlin.quantize(t(W), bits, group, 0, pack=True)
    wdq, *_ = O.quantize(W, bits, group)
    return out["qweight"], out["qsz"], out["flags"], wdq


GEMV_SHAPES = [(4096, 4096, 128), (1024, 4096, 128), (777, 768, 128), (300, 3072, 64),
               (130, 14336, 128), (64, 32, 32), (96, 512, 512), (50, 96, 32), (40, 4096, 4096)]


@pytest.mark.parametrize("bits", [4, 3, 2, 8])
@pytest.mark.parametrize("shape", GEMV_SHAPES)
def test_gemv_matches_oracle(bits, shape):
    N, K, group = shape
    if bits in (2, 3) and group == 128:
        group = 64 if K % 64 == 0 else group
    qw, qsz, fl, wdq = _packed(N, K, bits, group, seed=N + K + bits)
    bias = np.random.RandomState(3).randn(N).astype(np.float16) * np.float16(0.1)
    for M in (1, 2, 3, 4, 5, 8, 13, 16):
        x = rand_x(M, K, seed=M)
        for b in (None, bias):
            y = qlin.gemv(t(x), qw, qsz, None if b is None else t(b), N, K, bits, group, fl)
            ref = O.linear_ref(x, wdq, b)
            assert_close_to_ref(n(y), ref, what=f"gemv b{bits} M{M} N{N} K{K} g{group}")


@pytest.mark.parametrize("wide", [False, True])
def test_gemv_wide_zeros(wide):
    N, K, group = 512, 1024, 128
    qw, qsz, fl, wdq = _packed(N, K, 4, group, seed=5, wide=wide)
    assert (fl == qlin.WIDE_ZERO) == wide
    for M in (1, 3):
        x = rand_x(M, K, 9)
        y = qlin.gemv(t(x), qw, qsz, None, N, K, 4, group, fl)
        assert_close_to_ref(n(y), O.linear_ref(x, wdq), what="wide gemv")
    x = rand_x(40, K, 9)
    y = qlin.gemm(t(x), qw, qsz, None, N, K, 4, group, fl)
    assert_close_to_ref(n(y), O.linear_ref(x, wdq), what="wide gemm")


GEMM_SHAPES = [(5, 4096, 4096, 128), (33, 1024, 4096, 128), (128, 777, 768, 128),
               (300, 256, 3072, 64), (200, 4096, 14336, 128), (2048, 512, 1024, 128),
               (17, 100, 96, 32), (129, 136, 160, 32)]


@pytest.mark.parametrize("bits", [4, 3, 2, 8])
@pytest.mark.parametrize("shape", GEMM_SHAPES)
def test_gemm_matches_oracle(bits, shape):
    M, N, K, group = shape
    if bits in (2, 3) and group == 128:
        group = 64
    qw, qsz, fl, wdq = _packed(N, K, bits, group, seed=M + N + K + bits)
    x = rand_x(M, K, seed=M)
    bias = np.random.RandomState(4).randn(N).astype(np.float16) * np.float16(0.1)
    y = qlin.gemm(t(x), qw, qsz, t(bias), N, K, bits, group, fl)
    assert_close_to_ref(n(y), O.linear_ref(x, wdq, bias), what=f"gemm b{bits} {shape}")


def test_linear_dispatch_and_batch_shapes():
    N, K, group = 384, 1024, 128
    qw, qsz, fl, wdq = _packed(N, K, 4, group, seed=11)
    for shp in ((1, 1, K), (1, 3, K), (2, 5, K), (1, 16, K), (1, 20, K), (2, 33, K), (1, 64, K),
                (1, 65, K), (3, 50, K)):
        x = np.random.RandomState(len(shp)).randn(*shp).astype(np.float16)
        y = qlin.linear(t(x), qw, qsz, None, N, K, 4, group, fl)
        assert tuple(y.shape) == shp[:-1] + (N,)
        assert_close_to_ref(n(y).reshape(-1, N), O.linear_ref(x.reshape(-1, K), wdq))


def test_invalid_arguments_raise():
    N, K, group = 64, 256, 128
    qw, qsz, fl, _ = _packed(N, K, 4, group, seed=1)
    x = t(rand_x(1, K, 1))
    with pytest.raises(ValueError):
        qlin.gemv(x, qw, qsz, None, N, K, 5, group)            # bits
    with pytest.raises(ValueError):
        qlin.gemv(x, qw, qsz, None, N, K, 4, 100)              # group
    with pytest.raises(ValueError):
        qlin.linear(x.float(), qw, qsz, None, N, K, 4, group)  # dtype
    with pytest.raises(RuntimeError):
        qlin.linear(x.cpu(), qw, qsz, None, N, K, 4, group)    # CPU tensor: no fallback
    lib = qlin.load_library()
    y = torch.empty(1, N, dtype=torch.float16, device="cuda")
    # raw C ABI: M out of the GEMV range, null pointers
    assert lib.qlin_gemv_f16(qw.data_ptr(), qsz.data_ptr(), 0, x.data_ptr(), None, y.data_ptr(),
                             17, N, K, 4, group, None) == 1
    assert lib.qlin_gemm_f16(None, qsz.data_ptr(), 0, x.data_ptr(), None, y.data_ptr(),
                             1, N, K, 4, group, None, 0, None) == 1


@pytest.mark.parametrize("bits,group", [(4, 128), (3, 64), (2, 64), (8, 128)])
def test_gptq_checkpoint_conversion(bits, group):
    """AutoGPTQ tensors (restated format, oracle/gptq_format.py) -> tiled layout: the packed
    layer's W_dq equals AutoGPTQ's fp16 dequant bit for bit, and its forward matches x @ W^T."""
    from oracle import gptq_format as OG
    from quant import gptq
    rs = np.random.RandomState(bits + group)
    K, N = 1024, 384
    G = K // group
    q = rs.randint(0, 2 ** bits, size=(K, N))
    z = rs.randint(1, 2 ** bits, size=(G, N))
    s = (rs.rand(G, N) * 0.01 + 1e-3).astype(np.float16)
    tensors = {"lin.qweight": torch.from_numpy(OG.pack_qweight(q, bits).view(np.int32)),
               "lin.qzeros": torch.from_numpy(OG.pack_qzeros(z, bits).view(np.int32)),
               "lin.scales": torch.from_numpy(s),
               "lin.g_idx": torch.from_numpy((np.arange(K) // group).astype(np.int32)),
               "lin.bias": torch.from_numpy((rs.randn(N) * 0.1).astype(np.float16))}
    ql = gptq.packed_quant_linear(tensors, "lin", bits)
    ref_w = OG.dequant(q, z, s, np.arange(K) // group)
    assert bit_equal(n(ql.dequantized_weight()), ref_w)
    x = rand_x(3, K, seed=2)
    y = ql(t(x).unsqueeze(0))[0]
    assert_close_to_ref(n(y), O.linear_ref(x, ref_w, tensors["lin.bias"].numpy()))


def _pick_bn(M, N, cus):
    """Mirror of qlin_gemm.hip pick_bn (block width by rounds of blocks over the CUs; 128 = the
    64 x 128 block for small grids, 255 = the 64 x 256 block when that grid would exceed a round)."""
    small = -(-M // 128) * -(-N // 256)
    if small * 2 <= cus:
        return 255 if small * 4 > cus else 128
    rel = {256: 1.0, 384: 1.42, 512: 1.84}
    best = None
    for bn in (256, 384, 512):
        blocks = -(-M // 128) * -(-N // bn)
        full, f = blocks // cus, (blocks % cus) / cus
        c = rel[bn] * (full + (0.5 + 0.5 * f if f else 0.0))
        if best is None or c < best[1]:
            best = (bn, c)
    return best[0]


@pytest.mark.parametrize("M,N,bn", [(4129, 6160, 512), (4129, 4112, 384), (8225, 4240, 256),
                                    (333, 1040, 128), (65, 4112, 128), (1000, 4000, 255)])
@pytest.mark.parametrize("bits,group", [(4, 128), (4, 64), (3, 64), (2, 32)])
def test_gemm_block_widths(bits, group, M, N, bn):
    """The 128 x 256 / 384 / 512 and 64 x 128 block tiles (pick_bn: whole rounds of blocks over
    the CUs) with ragged M and N; g64 / g32 take the wider tiles' checked k-step form.  The width
    the library picks is read back through qlin_gemm_block_cols (the expected widths are those of
    a 256-CU MI355X)."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    picked = qlin.load_library().qlin_gemm_block_cols(M, N, bits)
    assert picked == _pick_bn(M, N, cus)
    if cus != 256:
        pytest.skip(f"{cus} CUs: the {bn}-column block is not what this shape picks here")
    assert picked == bn
    K = 1024
    qw, qsz, fl, wdq = _packed(N, K, bits, group, seed=bits + group)
    x = rand_x(M, K, seed=7)
    y = n(qlin.gemm(t(x), qw, qsz, None, N, K, bits, group, fl))
    rows = np.unique(np.r_[0:64, M // 2 - 64:M // 2 + 64, M - 96:M].clip(0, M - 1))  # fp64 ref sample
    assert_close_to_ref(y[rows], O.linear_ref(x[rows], wdq), what=f"gemm bn{bn} b{bits} g{group}")


@pytest.mark.parametrize("bits,group", [(4, 128), (3, 64), (2, 32)])
def test_gemm_block_widths_bit_identical(bits, group):
    """Every block width accumulates each output in the same k order: the first 128 rows of
    launches that pick the 128 x 256 / 384 / 512 blocks equal, bit for bit, a 128-row launch that
    picks the 64 x 128 block."""
    lib = qlin.load_library()
    K = 1024
    seen = set()
    for N, Ms in ((4096, (1024, 2048, 8192)), (4112, (4129,))):
        qw, qsz, fl, _ = _packed(N, K, bits, group, seed=N + bits)
        xb = t(rand_x(max(Ms), K, seed=11))
        small = qlin.gemm(xb[:128].contiguous(), qw, qsz, None, N, K, bits, group, fl,
                          split=False)
        assert lib.qlin_gemm_block_cols(128, N, bits) == 128
        for M in Ms:
            seen.add(lib.qlin_gemm_block_cols(M, N, bits))
            big = qlin.gemm(xb[:M].contiguous(), qw, qsz, None, N, K, bits, group, fl,
                            split=False)
            assert torch.equal(big[:128], small), f"M={M} N={N} b{bits} g{group}"
    assert len(seen) >= 2, seen  # 256-CU MI355X: {255 (64 x 256), 256, 384, 512}


def test_packed_operands_dequantize_to_the_oracle_wdq():
    """The operands every product test uses: the HIP dequant of the packed weight equals the
    oracle's W_dq bit for bit at LLaMA3-8B widths (4096^2, int4 g128 / int3 g64 / int2 g64)."""
    for bits, group in ((4, 128), (3, 64), (2, 64)):
        qw, qsz, fl, wdq = _packed(4096, 4096, bits, group, seed=bits)
        got = n(qlin.dequant(qw, qsz, 4096, 4096, bits, group, fl))
        assert bit_equal(got, wdq), f"b{bits} g{group}: {np.sum(got != wdq)} mismatches"


def _sample_rows(M):
    """Rows checked against the float64 product: both ends, the middle, and a spread of rows
    (every 128-row block tile of the launch contributes some)."""
    rs = np.random.RandomState(M)
    rows = np.r_[0:64, M // 2 - 32:M // 2 + 32, M - 64:M, rs.randint(0, M, 192)]
    return np.unique(rows.clip(0, M - 1))


@pytest.mark.parametrize("M", [2048, 65536])
def test_gemm_llama_shapes_configs2(M):
    """BASELINE configs[2]: QuantLinear.forward with x [32, 2048, 4096] (M = 65,536; reference
    quant/int_linear.py:48-65) and one 2048-token PPL window (M = 2048) on the int4 g128 4096^2
    packed weight, through the product dispatch (qlin.linear), against the float64 product on the
    oracle's W_dq for sampled rows; the whole output is finite and the launch deterministic."""
    N = K = 4096
    qw, qsz, fl, wdq = _packed(N, K, 4, 128, seed=M)
    g = torch.Generator(device="cuda").manual_seed(M)
    x = torch.empty(M, K, dtype=torch.float16, device="cuda").normal_(0, 1, generator=g)
    shp = (32, 2048, K) if M == 65536 else (1, 2048, K)
    y = qlin.linear(x.view(shp), qw, qsz, None, N, K, 4, 128, fl).view(M, N)
    assert torch.isfinite(y).all()
    rows = _sample_rows(M)
    assert_close_to_ref(n(y[rows]), O.linear_ref(n(x[rows]), wdq), what=f"gemm M{M}")
    y2 = qlin.linear(x.view(shp), qw, qsz, None, N, K, 4, 128, fl).view(M, N)
    assert torch.equal(y, y2)
    # the kernel reproduces F.linear(x, W_dq) (the fake-quant path's hipBLASLt GEMM) to fp16
    # output rounding
    ref = torch.nn.functional.linear(x[rows], t(wdq))
    assert (y[rows].float() - ref.float()).abs().max().item() <= \
        2e-3 * ref.float().abs().max().item()


@pytest.mark.parametrize("M,N,K", [(65, 4096, 4096), (128, 4096, 14336), (200, 1040, 4096),
                                   (256, 4096, 4096), (100, 512, 1024)])
@pytest.mark.parametrize("bits,group", [(4, 128), (3, 64), (2, 32)])
def test_gemm_split_k(M, N, K, bits, group):
    """Small grids split K (qlin_linear_workspace_bytes > 0): the fp32 partials are reduced in a
    fixed order — deterministic, within fp32 rounding of the unsplit launch, and every epilogue
    (bias, residual, SiLU·mul) goes through the reduction pass."""
    lib = qlin.load_library()
    qw, qsz, fl, wdq = _packed(N, K, bits, group, seed=M + N)
    assert lib.qlin_linear_workspace_bytes(M, N, K, bits, group, 0) > 0
    x = rand_x(M, K, seed=M)
    bias = t((np.random.RandomState(3).randn(N) * 0.1).astype(np.float16))
    y = qlin.gemm(t(x), qw, qsz, bias, N, K, bits, group, fl)
    y2 = qlin.gemm(t(x), qw, qsz, bias, N, K, bits, group, fl)
    assert torch.equal(y, y2)  # deterministic
    ref = qlin.gemm(t(x), qw, qsz, bias, N, K, bits, group, fl, split=False)
    assert (y.float() - ref.float()).abs().max().item() <= 2e-3 * ref.float().abs().max().item()
    assert_close_to_ref(n(y), O.linear_ref(x, wdq, n(bias)), what=f"splitk M{M} N{N} K{K}")
    r = t(rand_x(M, N, seed=5))
    yr = qlin.linear_ep(t(x), qw, qsz, bias, N, K, bits, group, fl, epilogue=qlin.EP_RESIDUAL,
                        residual=r)
    assert (yr.float() - (r.float() + y.float())).abs().max().item() <= \
        2e-3 * (r.float().abs().max().item() + y.float().abs().max().item())
    if N % 16 == 0:
        ys = qlin.linear_ep(t(x), qw, qsz, bias, N, K, bits, group, fl, epilogue=qlin.EP_SILU_MUL)
        assert ys.shape == (M, N // 2) and torch.isfinite(ys).all()


@pytest.mark.parametrize("N", [8192 + 16 * 3 + 5, 8192 + 16])
def test_gemv_two_row_tiles_per_block(N):
    """8-16 token rows on a wide matrix take two row tiles per block (odd tile counts clamp the
    last block's second tile)."""
    K, group = 512, 128
    qw, qsz, fl, wdq = _packed(N, K, 4, group, seed=N)
    bias = np.random.RandomState(5).randn(N).astype(np.float16) * np.float16(0.1)
    for M in (5, 8, 13, 16):
        x = rand_x(M, K, seed=M)
        y = qlin.gemv(t(x), qw, qsz, t(bias), N, K, 4, group, fl)
        assert_close_to_ref(n(y), O.linear_ref(x, wdq, bias), what=f"gemv ntb2 M{M} N{N}")
    if N % 16 == 0:  # the residual epilogue on the same path
        x = rand_x(16, K, seed=3)
        r = rand_x(16, N, seed=4)
        got = qlin.linear_ep(t(x), qw, qsz, None, N, K, 4, group, fl, epilogue=qlin.EP_RESIDUAL,
                             residual=t(r))
        ref = t(r) + qlin.gemv(t(x), qw, qsz, None, N, K, 4, group, fl)
        assert torch.equal(got, ref)


# (batch, N, K, bits, group, M): fast-path problems (one launch, grid Nt x batch) and ones the
# fast path does not take (14336-deep: > 4 tiles per wave; M > 4; K % 128) -> one launch each
BATCHED_CASES = [(3, 4096, 4096, 4, 128, 1), (4, 777, 768, 3, 64, 2), (2, 300, 3072, 2, 64, 4),
                 (3, 1040, 4096, 8, 128, 3), (2, 130, 14336, 4, 128, 1), (2, 64, 32, 4, 32, 13),
                 (5, 96, 4096, 4, 4096, 1),
                 # more tile rows than resident waves: several rows per wave, uneven split; Kt = 4
                 # (the 4-deep prefetch instance) and Kt = 8
                 (20, 4112, 512, 4, 128, 1), (20, 4096, 1024, 4, 64, 2),
                 # round-wide (scale, zero) loads: g32 (two 1-KB loads per round), g64 with 4-deep
                 # rounds (lanes wrap over 512 B); group 256 keeps per-tile loads
                 (3, 528, 1024, 4, 32, 1), (4, 1040, 512, 2, 64, 1), (3, 272, 2048, 3, 256, 2),
                 # two tile rows per wave (M = 1, narrow zeros, even tile-row count): int2 / int3
                 # g64, int4 g32 (two round loads), int8, a two-row matrix, and more row pairs
                 # than resident waves with an uneven split
                 (3, 512, 2048, 2, 64, 1), (2, 288, 1024, 3, 64, 1), (3, 544, 1024, 4, 32, 1),
                 (4, 4096, 1024, 8, 128, 1), (3, 32, 1024, 4, 128, 1), (20, 4128, 1024, 2, 64, 1)]


@pytest.mark.parametrize("case", BATCHED_CASES)
@pytest.mark.parametrize("with_bias", [False, True])
def test_gemv_batched_bit_identical_to_per_problem(case, with_bias):
    """qlin_gemv_batched_f16: every y[b] within the GEMV tolerance of the oracle's x @ W_dq^T;
    bit-identical to qlin_gemm_f16 (unsplit: one MFMA chain per output in k order) where the
    streaming kernel runs (M <= 4, K % 512 == 0), to qlin_gemv_f16 where the batch falls back
    to one launch per problem."""
    B, N, K, bits, group, M = case
    packs = [_packed(N, K, bits, group, seed=17 * b + N) for b in range(B)]
    fl = packs[0][2]
    packs = [p for p in packs if p[2] == fl]  # one layout flag per batch
    B = len(packs)
    qw = torch.stack([p[0] for p in packs])
    qsz = torch.stack([p[1] for p in packs])
    x = np.stack([rand_x(M, K, seed=100 + b) for b in range(B)])
    bias = (np.random.RandomState(5).randn(B, N) * 0.1).astype(np.float16) if with_bias else None
    y = qlin.gemv_batched(t(x), qw, qsz, None if bias is None else t(bias), N, K, bits, group, fl)
    stream = M <= 4 and K % 512 == 0
    for b in range(B):
        bb = None if bias is None else t(bias[b])
        if stream:
            yb = qlin.gemm(t(x[b]), qw[b], qsz[b], bb, N, K, bits, group, fl, split=False)
        else:
            yb = qlin.gemv(t(x[b]), qw[b], qsz[b], bb, N, K, bits, group, fl)
        assert bit_equal(n(y[b]), n(yb)), f"problem {b}"
        ref = O.linear_ref(x[b], packs[b][3], None if bias is None else bias[b])
        assert_close_to_ref(n(y[b]), ref, what=f"batched b{bits} N{N} K{K} problem {b}")


def test_gemv_batched_shared_activation():
    """x_stride 0: several matrices applied to one activation (e.g. the reference's separate
    gate_proj / up_proj modules on the same normed hidden state)."""
    N, K, bits, group = 1024, 4096, 4, 128
    packs = [_packed(N, K, bits, group, seed=40 + b) for b in range(3)]
    qw = torch.stack([p[0] for p in packs])
    qsz = torch.stack([p[1] for p in packs])
    x = rand_x(1, K, seed=9)
    y = qlin.gemv_batched(t(x), qw, qsz, None, N, K, bits, group, packs[0][2])
    for b in range(3):
        yb = qlin.gemm(t(x), qw[b], qsz[b], None, N, K, bits, group, packs[b][2], split=False)
        assert bit_equal(n(y[b]), n(yb)), f"problem {b}"


def test_gemv_batched_empty_and_shared_bias():
    N, K, bits, group = 64, 1024, 4, 128
    qw, qsz, fl, wdq = _packed(N, K, bits, group, seed=3)
    x = torch.zeros(0, 1, K, dtype=torch.float16, device="cuda")
    y = qlin.gemv_batched(x, qw[None][:0], qsz[None][:0], None, N, K, bits, group, fl)
    assert tuple(y.shape) == (0, 1, N)
    # bias_stride 0 through the C entry: one bias row shared by both problems
    lib = qlin.load_library()
    xs = t(np.stack([rand_x(1, K, seed=s_) for s_ in (1, 2)]))
    b = t((np.random.RandomState(4).randn(N) * 0.1).astype(np.float16))
    qw2, qsz2 = torch.stack([qw, qw]), torch.stack([qsz, qsz])
    y2 = torch.empty(2, 1, N, dtype=torch.float16, device="cuda")
    rc = lib.qlin_gemv_batched_f16(qw2.data_ptr(), qw.numel(), qsz2.data_ptr(), qsz.numel(), fl,
                                   xs.data_ptr(), K, b.data_ptr(), 0, y2.data_ptr(), N, 2, 1, N, K,
                                   bits, group, torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    for i in range(2):
        ref = qlin.gemm(xs[i], qw, qsz, b, N, K, bits, group, fl, split=False)
        assert bit_equal(n(y2[i]), n(ref))


def test_gemv_batched_rejects_overlapping_strides():
    lib = qlin.load_library()
    qw, qsz, fl, _ = _packed(64, 256, 4, 128, seed=1)
    x = torch.zeros(2, 1, 256, dtype=torch.float16, device="cuda")
    y = torch.zeros(2, 1, 64, dtype=torch.float16, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    ok = lib.qlin_gemv_batched_f16(qw.data_ptr(), 0, qsz.data_ptr(), 0, fl, x.data_ptr(), 256,
                                   None, 0, y.data_ptr(), 64, 2, 1, 64, 256, 4, 128, st)
    assert ok == 1  # zero weight strides would alias problems
    with pytest.raises(ValueError):
        qlin.gemv_batched(x, qw.unsqueeze(0), qsz.unsqueeze(0), None, 64, 256, 4, 128, fl)


def test_gemv_batched_geometry_per_instance():
    """Each streaming-kernel instance sizes its grid from its OWN static LDS and occupancy
    (a cache keyed on the kernel's C++ type was shared by every instance, so the first
    launch in a process decided the LDS padding and blocks per CU of all later ones).  Plan int4
    g128 first, then the two-row int2 g32 / g64 and int3 g64 instances (larger static LDS), then a
    one-row instance (odd tile-row count): every two-row instance must hold exactly 4 blocks per
    CU with its own padding, and no plan may promise more blocks per CU than its LDS allows."""
    K, B = 4096, 8
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    x = torch.zeros(B, 1, K, dtype=torch.float16, device="cuda")
    seen = {}
    for N, bits, group in ((4096, 4, 128), (4096, 2, 32), (4096, 2, 64), (4096, 3, 64),
                           (4112, 4, 128), (4096, 4, 128)):
        qw = torch.zeros(B, *qlin.packed_shape(N, K, bits), dtype=torch.int32, device="cuda")
        qsz = torch.zeros(B, *qlin.sz_shape(N, K, group), dtype=torch.int32, device="cuda")
        p = qlin.gemv_batched_plan(x, qw, qsz, N, K, bits, group)
        assert p["blocks"] > 0, (N, bits, group, p)
        lds = p["static_lds"] + p["dyn_lds"]
        assert p["blocks_per_cu"] * lds <= 160 * 1024, (N, bits, group, p)
        if p["rows_per_wave"] == 2:
            assert p["blocks_per_cu"] == 4 and lds == 40 * 1024 - 64, (N, bits, group, p)
        else:
            assert N == 4112 and p["dyn_lds"] == 0, (N, bits, group, p)
        tiles = B * (-(-N // 16)) // p["rows_per_wave"]
        assert p["blocks"] == -(-min(tiles, cus * p["blocks_per_cu"] * 4) // 4), p
        key = (N, bits, group)
        assert seen.setdefault(key, p) == p  # the same instance plans the same way every time
