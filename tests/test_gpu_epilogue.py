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
    assert lib.qlin_linear_ep_f16(P(qw), P(qsz), fl, P(x), None, None, P(y), 1, 32, 128, 4, 128,
                                  qlin.EP_RESIDUAL, None) == 1  # residual missing
    assert lib.qlin_linear_ep_f16(P(qw), P(qsz), fl, P(x), None, None, P(y), 1, 24, 128, 4, 128,
                                  qlin.EP_SILU_MUL, None) == 1  # N % 16
    assert lib.qlin_linear_ep_f16(P(qw), P(qsz), fl, P(x), None, None, P(y), 1, 32, 128, 4, 128,
                                  7, None) == 1  # unknown epilogue
