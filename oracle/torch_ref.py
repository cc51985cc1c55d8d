"""TEST INFRASTRUCTURE / CPU BASELINE — not product code.

A pure-PyTorch restatement of the reference's fake-quant forward on the CPU, used only as
``bench.py``'s ``cpu_baseline`` leg (the reference's own op sequence timed on the GPU box's host
cores) and pinned bit-exactly against the golden fixtures the reference wrote
(tests/test_oracle_golden.py).  Nothing under llama3-quantization_amd/ imports it.

Restated from /root/reference (read as text):
  quant/quantizer.py:15-19    round_ste
  quant/quantizer.py:132-159  per_token_dynamic_calibration (no LWC / deficiency here)
  quant/quantizer.py:94-115   fake_quant
  quant/int_linear.py:48-65   QuantLinear.forward -> F.linear(input, weight, bias)
"""
import torch
import torch.nn.functional as F

CLIPMIN = 1e-5  # quant/quantizer.py:10


def round_ste(x):
    return (x.round() - x).detach() + x


def qrange(n_bits, disable_zero_point=False):
    if disable_zero_point:
        return -(2 ** (n_bits - 1)), 2 ** (n_bits - 1) - 1
    return 0, 2 ** n_bits - 1


def calibrate(x, n_bits, group_size=None, symmetric=False, disable_zero_point=False):
    """(scale, round_zero_point) of ``x`` ([rows, K]; groups of ``group_size`` consecutive
    in-features, or the whole row) — quantizer.py:132-159, same torch ops in x's dtype."""
    if group_size:
        x = x.reshape(-1, group_size)
    xmin = x.amin([-1], keepdim=True)
    xmax = x.amax([-1], keepdim=True)
    if symmetric:
        abs_max = torch.max(xmax.abs(), xmin.abs())
        scale = (abs_max / (2 ** (n_bits - 1) - 1)).clamp(min=CLIPMIN, max=1e4)
        zero_point = (2 ** (n_bits - 1) - 1) * torch.ones_like(scale)
    else:
        scale = ((xmax - xmin) / (2 ** n_bits - 1)).clamp(min=CLIPMIN, max=1e4)
        zero_point = -xmin / scale
    rzp = None if disable_zero_point else zero_point.clamp(min=-1e4, max=1e4).round()
    return scale, rzp


def fake_quant(x, scale, rzp, n_bits, group_size=None, disable_zero_point=False):
    """quantizer.py:94-115 (no deficiency padding)."""
    qmin, qmax = qrange(n_bits, disable_zero_point)
    shape = x.shape
    if group_size:
        x = x.reshape(-1, group_size)
    x_int = round_ste(x / scale)
    if rzp is not None:
        x_int = x_int.add(rzp)
    x_int = x_int.clamp(qmin, qmax)
    x_dq = x_int
    if rzp is not None:
        x_dq = x_dq.sub(rzp)
    x_dq = x_dq.mul(scale)
    return x_dq.reshape(shape)


def quantize(w, n_bits, group_size=None, symmetric=False, disable_zero_point=False):
    """UniformAffineQuantizer.forward for a weight (quantizer.py:118-130): W_dq, scale, zp."""
    scale, rzp = calibrate(w, n_bits, group_size, symmetric, disable_zero_point)
    return fake_quant(w, scale, rzp, n_bits, group_size, disable_zero_point), scale, rzp


def quant_linear(x, w, n_bits, group_size, bias=None):
    """QuantLinear.forward with use_weight_quant=True (int_linear.py:48-65): quantize the weight on
    every call, then F.linear — the reference's calibration-time cost."""
    return F.linear(x, quantize(w, n_bits, group_size)[0], bias)
