"""Every one-token-row route of the packed linear against the oracle.

At M = 1 the library routes each shape to one of three kernels (``qlin_gemv_m1_route``,
csrc/qlin_gemv.hip ``m1_route``): the work-queue kernel (wide matrices: LLaMA3-8B gate/up, N =
28,672, and N = 16,384; chunks of 4 k-tiles from an LDS counter, per-chunk partial sums added per
row in k order), the fast split-K kernel (q/k/v, o, 4096^2) and the rows kernel (long K:
the down projection, 4096 x 14,336).  Here each route meets ``O.linear_ref`` (the reference's
``F.linear(x, W_dq)``, quant/int_linear.py:62, in float64) directly, at every bit width {2, 3, 4,
8} x group {32, 64, 128} and every zero-point mode of the layout: integral zeros (the
reference's RTN / GPTQ weights), zeros beyond +-1024 (QLIN_WIDE_ZERO: degenerate groups, the
reference clamps zp to +-1e4) and fp16 zeros (QLIN_FLOAT_ZERO: HQQ checkpoints, the configs[3]
decode path; reference quantizehqq.py:36-39).  Each case runs the product plain (+ bias), with
the residual epilogue, and with the RMSNorm fused in front (fp16 norm weight), plain and with
the SiLU(gate) * up epilogue — the four forms the decoder layer uses.

W_dq is formed from the integer codes and the (scale, zero) values by the reference arithmetic
RN16(RN16(u - z) * s) (quant/quantizer.py:107-110; hqq's ((W_q - zero) * scale) in fp16) in plain
torch elementwise ops, independently of the kernels, and the float64 product is the oracle's on
the host; the codes are packed by ``qlin_pack_codes`` (itself checked bit-exact against the
oracle's packer in tests/test_hqq_format.py)."""
import numpy as np
import pytest
import torch

from helpers import assert_close_to_ref, t
from oracle import quant_oracle as O

pytestmark = pytest.mark.gpu

from quant import qlin  # noqa: E402

SHAPES = {"gate_up_28672x4096": (28672, 4096, qlin.M1_WORK_QUEUE),
          "wide_16384x4096": (16384, 4096, qlin.M1_WORK_QUEUE),
          "down_4096x14336": (4096, 14336, qlin.M1_ROWS),
          "qkv_6144x4096": (6144, 4096, qlin.M1_FAST)}
BITS_GROUPS = [(b, g) for b in (2, 3, 4, 8) for g in (32, 64, 128)]
EPS = 1e-5


def _case(N, K, bits, group, zmode, seed):
    """Codes, (scale, zero) and W_dq of one packed matrix (drawn on the GPU for speed; W_dq by
    plain torch elementwise ops, then read back for the host float64 product)."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    G = K // group
    dev = "cuda"
    u = torch.randint(0, 2 ** bits, (N, K), generator=g, device=dev, dtype=torch.int32)
    # wide zeros (|u - z| up to ~1e4) get 100x smaller scales, so outputs and the SiLU * up
    # products stay inside the fp16 range
    s = ((torch.rand(N, G, generator=g, device=dev) * 4e-3 + 5e-4) *
         (1e-2 if zmode == "wide" else 1.0)).half()
    flags = 0
    if zmode == "float":
        z = (torch.rand(N, G, generator=g, device=dev) * (2 ** bits - 1)).half()
        flags = qlin.FLOAT_ZERO
        qsz = qlin.join_sz_float(s, z)
    else:
        z = torch.randint(-2, 2 ** bits + 2, (N, G), generator=g, device=dev, dtype=torch.int32)
        if zmode == "wide":
            pick = torch.rand(N, G, generator=g, device=dev) < 0.02
            vals = torch.tensor([-1500, 1800, 3001, -9999, 10000], device=dev, dtype=torch.int32)
            alt = vals[torch.randint(0, 5, (N, G), generator=g, device=dev)]
            z = torch.where(pick, alt, z)
            flags = qlin.WIDE_ZERO
        qsz = qlin.join_sz(s, z.to(torch.int16))
        assert qlin.sz_flags(qsz) == flags  # the integral layouts' flag as the packers derive it
    # W_dq = RN16(RN16(u - z) * s): u - z and the fp16 x fp16 product are exact in fp32
    d = (u.view(N, G, group).float() - z.float()[:, :, None]).half()
    wdq = (d.float() * s.float()[:, :, None]).half().view(N, K)
    qw = qlin.pack_codes(u.to(torch.uint8), bits)
    return qw, qsz, flags, wdq.cpu().numpy()


def _rmsnorm_ref(x, w16):
    """OmniLlamaRMSNorm (reference quant/omni_norm.py:52-63): fp32 statistics, RN16(w * (x * r))."""
    x32 = x.astype(np.float32)
    r = np.float32(1.0) / np.sqrt((x32 * x32).mean(-1, keepdims=True, dtype=np.float32) +
                                  np.float32(EPS), dtype=np.float32)
    return (w16.astype(np.float32) * (x32 * r)).astype(np.float16)


def _assert_residual(y, lin64, res, what):
    """RN16(res + RN16(linear)) (the reference's fp16 ``residual + o_proj(x)``) against float64:
    the GEMV tolerance on the linear part plus the two fp16 roundings (half an ulp of the linear
    output and of the sum), which dominate where res and the linear output nearly cancel."""
    y = y.astype(np.float64)
    ref = res.astype(np.float64) + lin64
    bound = (2e-3 * (np.abs(lin64) + np.abs(lin64).max() / 16.0) +
             2.0 ** -11 * (np.abs(lin64) + np.abs(ref)) + 1e-6)
    bad = np.abs(y - ref) > bound
    assert not bad.any(), f"{what}: {bad.sum()} / {bad.size} outside tolerance"


def _silu_mul64(y64):
    """Rows interleaved in 8-row halves per 16-row tile (gate rows, then up rows)."""
    v = y64.reshape(y64.shape[0], -1, 2, 8)
    g, u = v[:, :, 0].reshape(y64.shape[0], -1), v[:, :, 1].reshape(y64.shape[0], -1)
    return g / (1.0 + np.exp(-g)) * u


def _check_routes(name, bits, group, zmode):
    N, K, route = SHAPES[name]
    assert qlin.m1_route(N, K, bits, group) == route, (name, bits, group)
    seed = N + K + 10 * bits + group + {"narrow": 0, "wide": 1, "float": 2}[zmode]
    qw, qsz, fl, wdq = _case(N, K, bits, group, zmode, seed)
    rs = np.random.RandomState(seed + 1)
    x = (rs.randn(1, K) * 2).astype(np.float16)
    bias = (rs.randn(N) * 0.1).astype(np.float16)
    res = rs.randn(1, N).astype(np.float16)
    w16 = (1 + 0.1 * rs.randn(K)).astype(np.float16)
    xn = _rmsnorm_ref(x, w16)
    ref = O.linear_ref(np.concatenate([x, xn]), wdq)  # [2, N] float64
    what = f"{name} b{bits} g{group} {zmode}"
    xs = t(x).view(1, 1, K)
    y = qlin.gemv(xs, qw, qsz, t(bias), N, K, bits, group, fl)
    assert_close_to_ref(y.view(1, N).cpu().numpy(), ref[:1] + bias, what=what + " +bias")
    y = qlin.linear_ep(xs, qw, qsz, None, N, K, bits, group, fl, epilogue=qlin.EP_RESIDUAL,
                       residual=t(res).view(1, 1, N))
    _assert_residual(y.view(1, N).cpu().numpy(), ref[:1], res, what=what + " residual")
    nw = t(w16)
    y = qlin.rmsnorm_linear_ep(xs, nw, EPS, qw, qsz, None, N, K, bits, group, fl)
    assert_close_to_ref(y.view(1, N).cpu().numpy(), ref[1:], what=what + " rmsnorm")
    y = qlin.rmsnorm_linear_ep(xs, nw, EPS, qw, qsz, None, N, K, bits, group, fl,
                               epilogue=qlin.EP_SILU_MUL)
    assert_close_to_ref(y.view(1, N // 2).cpu().numpy(), _silu_mul64(ref[1:]), rtol=4e-3,
                        what=what + " rmsnorm silu*up")


LLAMA = ["gate_up_28672x4096", "down_4096x14336", "qkv_6144x4096"]


@pytest.mark.parametrize("bits,group", BITS_GROUPS)
@pytest.mark.parametrize("name", LLAMA)
def test_m1_route_integral_zeros(name, bits, group):
    _check_routes(name, bits, group, "narrow")


@pytest.mark.parametrize("bits,group", [(4, 128), (3, 64), (2, 32), (8, 64)])
def test_m1_route_work_queue_16384(bits, group):
    _check_routes("wide_16384x4096", bits, group, "narrow")


@pytest.mark.parametrize("bits,group", BITS_GROUPS)
@pytest.mark.parametrize("name", LLAMA)
def test_m1_route_hqq_float_zeros(name, bits, group):
    _check_routes(name, bits, group, "float")


@pytest.mark.parametrize("bits,group", [(4, 128), (3, 64), (2, 32), (8, 64)])
@pytest.mark.parametrize("name", LLAMA)
def test_m1_route_wide_zeros(name, bits, group):
    _check_routes(name, bits, group, "wide")
