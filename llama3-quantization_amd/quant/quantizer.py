"""UniformAffineQuantizer — MI355X build of the reference quantizer (quant/quantizer.py:23-165).

Same constructor, attributes and methods as the reference, so QuantLinear / the decoder layers /
omniquant-style drivers use it unchanged.  The arithmetic runs in ONE fused gfx950 kernel
(``qlin_quantize``: per-group amin/amax -> LWC -> scale/zero point -> fake-quant), bit-exact with
the reference's fp16 / fp32 torch ops (tests/test_gpu_quantizer.py against the reference's golden
vectors).  Gradients are not provided: LWC/LET training is calibration-time work outside the hot
path.
"""
import math

import torch
import torch.nn as nn

from . import qlin

CLIPMIN = 1e-5


def round_ste(x: torch.Tensor):
    """Straight-through round (quantizer.py:15-19); kept for API parity."""
    return (x.round() - x).detach() + x


class UniformAffineQuantizer(nn.Module):
    def __init__(
        self,
        n_bits: int = 8,
        symmetric: bool = False,
        per_channel_axes=[],
        metric="minmax",
        dynamic=False,
        dynamic_method="per_cluster",
        group_size=None,
        shape=None,
        lwc=False,
        disable_zero_point=False,
    ):
        super().__init__()
        self.symmetric = symmetric
        self.disable_zero_point = disable_zero_point
        assert 2 <= n_bits <= 16, "bitwidth not supported"
        self.n_bits = n_bits
        self._set_range()
        self.per_channel_axes = per_channel_axes
        self.metric = metric
        self.cluster_counts = None
        self.cluster_dim = None
        self.scale = None
        self.zero_point = None
        self.round_zero_point = None
        self.cached_xmin = None
        self.cached_xmax = None
        self.dynamic = dynamic
        self.dynamic_method = dynamic_method
        self.deficiency = 0
        self.lwc = lwc
        init_value = 4.0  # learnable weight clipping init (quantizer.py:68)
        if lwc:
            if group_size:
                dim1 = int(shape[0] * math.ceil(shape[1] / group_size))
                self.deficiency = shape[-1] % group_size
                if self.deficiency > 0:
                    self.deficiency = group_size - self.deficiency
                    assert self.symmetric  # mlc-llm symmetric padding (quantizer.py:75)
            else:
                dim1 = shape[0]
            self.upbound_factor = nn.Parameter(torch.ones((dim1, 1)) * init_value)
            self.lowbound_factor = nn.Parameter(torch.ones((dim1, 1)) * init_value)
        self.sigmoid = nn.Sigmoid()
        self.enable = True
        self.group_size = group_size

    def _set_range(self):
        if self.disable_zero_point:
            self.qmin = -(2 ** (self.n_bits - 1))
            self.qmax = 2 ** (self.n_bits - 1) - 1
        else:
            self.qmin = 0
            self.qmax = 2 ** self.n_bits - 1

    def change_n_bits(self, n_bits):
        self.n_bits = n_bits
        self._set_range()

    # -- helpers --------------------------------------------------------------------------------
    def _flags(self):
        f = 0
        if self.symmetric:
            f |= qlin.SYMMETRIC
        if self.disable_zero_point:
            f |= qlin.DISABLE_ZERO_POINT
        if self.lwc:
            f |= qlin.LWC
        return f

    def _view2d(self, x):
        """x as the [rows, K] operand the kernel quantizes, plus the group size it uses."""
        if self.group_size:
            assert len(x.shape) == 2, "only support linear layer now"
            if self.deficiency > 0:
                pad = torch.zeros((x.shape[0], self.deficiency), dtype=x.dtype, device=x.device)
                x = torch.cat((x, pad), dim=1)
            return x.contiguous(), self.group_size
        K = x.shape[-1]
        return x.reshape(-1, K).contiguous(), K

    def _lwc_sig(self, dtype):
        """sigmoid(factors) with the reference's own op (quantizer.py:144-145); returns the dtype
        the torch expression would promote to and the factors in it."""
        up = self.sigmoid(self.upbound_factor.detach())
        low = self.sigmoid(self.lowbound_factor.detach())
        cdt = torch.promote_types(dtype, up.dtype)
        return cdt, up.to(cdt).reshape(-1).contiguous(), low.to(cdt).reshape(-1).contiguous()

    def _run(self, x, want_xdq):
        x2, g = self._view2d(x)
        cdt, up, low = x.dtype, None, None
        if self.lwc:
            cdt, up, low = self._lwc_sig(x.dtype)
            x2 = x2.to(cdt)
        out = qlin.quantize(x2, self.n_bits, g, self._flags(), up, low, want_xdq=want_xdq)
        rows = x2.shape[0]
        if self.group_size:
            shp = (rows * (x2.shape[1] // g), 1)
        else:
            shp = tuple(x.shape[:-1]) + (1,)
        self.scale = out["scale"].reshape(shp)
        self.round_zero_point = None if self.disable_zero_point else out["zp"].reshape(shp)
        xdq = out["x_dq"]
        if want_xdq:
            if self.group_size:
                if self.deficiency > 0:
                    xdq = xdq[:, :-self.deficiency]
            else:
                xdq = xdq.reshape(x.shape)
        return xdq

    # -- reference API --------------------------------------------------------------------------
    def fake_quant(self, x, scale, round_zero_point):
        """quantizer.py:94-115 with given parameters (fused gfx950 kernel)."""
        x2, g = self._view2d(x)
        cdt = torch.promote_types(x.dtype, scale.dtype)
        x2 = x2.to(cdt)
        s = scale.to(cdt).reshape(-1).contiguous()
        z = None if round_zero_point is None else round_zero_point.to(cdt).reshape(-1).contiguous()
        if (round_zero_point is None) != bool(self.disable_zero_point):
            raise ValueError("round_zero_point must be None exactly when disable_zero_point")
        flags = qlin.DISABLE_ZERO_POINT if self.disable_zero_point else 0
        out = qlin.fake_quant(x2, s, z, self.n_bits, g, flags)["x_dq"]
        if self.group_size:
            if self.deficiency > 0:
                out = out[:, :-self.deficiency]
            return out
        return out.reshape(x.shape)

    def forward(self, x: torch.Tensor):
        if self.n_bits >= 16 or not self.enable:
            return x
        if self.metric == "fix0to1":
            return x.mul_(2 ** self.n_bits - 1).round_().div_(2 ** self.n_bits - 1)
        if self.dynamic_method == "per_token" or self.dynamic_method == "per_channel":
            return self._run(x, want_xdq=True)
        raise NotImplementedError()

    def per_token_dynamic_calibration(self, x):
        """quantizer.py:132-159: sets ``scale`` / ``round_zero_point`` (kernel, no x_dq output)."""
        self._run(x, want_xdq=False)

    def register_scales_and_zeros(self):
        self.register_buffer("scales", self.scale)
        self.register_buffer("zeros", self.round_zero_point)
        del self.scale
        del self.round_zero_point
