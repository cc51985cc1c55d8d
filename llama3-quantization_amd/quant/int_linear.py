"""QuantLinear — MI355X build of the reference drop-in nn.Linear (quant/int_linear.py:11-69).

Reference behaviour is kept verbatim at the module level:
  * constructor ``QuantLinear(org_module, weight_quant_params, act_quant_params,
    disable_input_quant)``; ``weight``/``bias`` buffers share storage with ``org_module``;
  * ``forward`` picks temp_weight / weight_quantizer(weight) / weight, optionally fake-quantizes the
    input per token, then calls ``self.fwd_func(input, weight, bias, **self.fwd_kwargs)``;
  * ``set_quant_state(weight_quant, act_quant)``.

Added (the real-quant path of quant/omniquant.py:315-335, re-done for MI355X):
  * ``pack()`` — after ``register_scales_and_zeros`` (weight == W_dq), packs the codes into the
    canonical gfx950 layout (``qlin_pack_f16``) and switches ``fwd_func`` to the fused
    unpack + dequant + GEMV/MFMA-GEMM kernels (``qlin_linear_f16``).  ``pack_from_weight()`` does the
    RTN quantize + pack of a float weight in one kernel.
  * ``packed`` / ``qweight`` / ``qsz`` / ``qflags`` / ``wbits`` / ``group`` state.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import qlin
from .quantizer import UniformAffineQuantizer


class QuantLinear(nn.Module):
    """
    Quantized Module that can perform quantized convolution or normal convolution.
    To activate quantization, please use set_quant_state function.
    """

    def __init__(
        self,
        org_module: nn.Linear,
        weight_quant_params: dict = {},
        act_quant_params: dict = {},
        disable_input_quant=False,
    ):
        super().__init__()
        self.fwd_kwargs = dict()
        self.fwd_func = F.linear
        self.register_buffer("weight", org_module.weight)
        if org_module.bias is not None:
            self.register_buffer("bias", org_module.bias)
        else:
            self.bias = None
        self.in_features = org_module.in_features
        self.out_features = org_module.out_features
        self.use_weight_quant = False
        self.use_act_quant = False
        self.weight_quantizer = UniformAffineQuantizer(**weight_quant_params,
                                                       shape=org_module.weight.shape)
        if not disable_input_quant:
            self.act_quantizer = UniformAffineQuantizer(**act_quant_params)
        else:
            self.act_quantizer = None
        self.disable_input_quant = disable_input_quant
        self.use_temporary_parameter = False
        self.packed = False
        self.wbits = None
        self.group = None
        self.qflags = 0

    def forward(self, input: torch.Tensor):
        if self.packed:
            weight = None
            bias = self.bias
        elif self.use_temporary_parameter:
            weight = self.temp_weight
            bias = self.temp_bias
        elif self.use_weight_quant:
            weight = self.weight_quantizer(self.weight)
            bias = self.bias
        else:
            weight = self.weight
            bias = self.bias

        if self.use_act_quant and not self.disable_input_quant:
            if self.packed and self._fused_act_bits(input):
                # per-token fake-quant of x inside the packed linear (bit-exact; the act
                # quantizer's scale / round_zero_point attributes are not refreshed)
                return self._packed_fwd(input, weight, bias,
                                        act_bits=self.act_quantizer.n_bits,
                                        act_flags=self.act_quantizer._flags())
            input = self.act_quantizer(input)

        out = self.fwd_func(input, weight, bias, **self.fwd_kwargs)
        return out

    def _fused_act_bits(self, x):
        """The act quantizer is the reference's per-token dynamic one (quant/int_linear.py:38-41,
        main.py act_quant_params) and can run inside the packed linear."""
        return act_spec(self) is not None and x.dtype == torch.float16 and x.shape[-1] % 8 == 0

    def set_quant_state(self, weight_quant: bool = False, act_quant: bool = False):
        self.use_weight_quant = weight_quant
        self.use_act_quant = act_quant

    # ------------------------------------------------------------------------------------------
    # packed (real-quant) mode
    # ------------------------------------------------------------------------------------------
    def _packed_fwd(self, input, weight, bias, act_bits=0, act_flags=0):
        x = input
        if x.dtype != torch.float16:
            x = x.to(torch.float16)
        b = None if bias is None else bias.to(torch.float16).contiguous()
        if act_bits:
            y = qlin.linear_ep(x.contiguous(), self.qweight, self.qsz, b, self.out_features,
                               self.in_features, self.wbits, self.group, self.qflags,
                               act_bits=act_bits, act_flags=act_flags)
        else:
            y = qlin.linear(x.contiguous(), self.qweight, self.qsz, b, self.out_features,
                            self.in_features, self.wbits, self.group, self.qflags)
        return y if input.dtype == torch.float16 else y.to(input.dtype)

    def _install(self, out, bits, group, keep_weight):
        self.register_buffer("qweight", out["qweight"])
        self.register_buffer("qsz", out["qsz"])
        self.qflags = out["flags"]
        self.wbits = bits
        self.group = group
        self.packed = True
        self.fwd_func = self._packed_fwd
        self.fwd_kwargs = {}
        if not keep_weight:
            self.weight = None

    def _check_packable(self):
        wq = self.weight_quantizer
        if not self.weight.is_cuda:
            raise RuntimeError("pack() runs the gfx950 packer: move the module to the GPU first")
        if wq.n_bits not in (2, 3, 4, 8):
            raise ValueError(f"packed mode supports 2/3/4/8-bit weights, not {wq.n_bits}")
        if wq.deficiency:
            raise ValueError("packed mode needs in_features % group_size == 0")
        return wq.group_size or self.in_features

    @torch.no_grad()
    def pack(self, keep_weight=False):
        """Pack W_dq with the registered (scales, zeros) — the reference's ``--real_quant`` step
        (quant/omniquant.py:315-335) with the gfx950 layout in place of AutoGPTQ's."""
        wq = self.weight_quantizer
        group = self._check_packable()
        if not hasattr(wq, "scales"):
            raise RuntimeError("call register_scales_and_zeros() before pack()")
        w = self.weight.to(torch.float16).contiguous()
        s = wq.scales.to(torch.float16).reshape(-1).contiguous()
        z = None if wq.zeros is None else wq.zeros.to(torch.float16).reshape(-1).contiguous()
        flags = qlin.DISABLE_ZERO_POINT if z is None else 0
        out = qlin.fake_quant(w, s, z, wq.n_bits, group, flags, want_xdq=False, pack=True)
        self._install(out, wq.n_bits, group, keep_weight)
        return self

    @torch.no_grad()
    def pack_from_weight(self, keep_weight=False):
        """RTN-quantize the float weight and pack it in one fused kernel (no LWC/LET)."""
        wq = self.weight_quantizer
        group = self._check_packable()
        if wq.lwc:
            raise ValueError("pack_from_weight() is plain RTN; use weight_quantizer + pack()")
        w = self.weight.to(torch.float16).contiguous()
        out = qlin.quantize(w, wq.n_bits, group, wq._flags(), want_xdq=keep_weight,
                            want_params=False, pack=True)
        self._install(out, wq.n_bits, group, keep_weight)
        if keep_weight:
            self.weight = out["x_dq"]
        return self

    def dequantized_weight(self):
        """W_dq [out, in] fp16 from the packed codes (bit-exact)."""
        if not self.packed:
            raise RuntimeError("module is not packed")
        return qlin.dequant(self.qweight, self.qsz, self.out_features, self.in_features,
                            self.wbits, self.group, self.qflags)

    def extra_repr(self):
        s = f"in_features={self.in_features}, out_features={self.out_features}"
        if self.packed:
            s += f", packed=int{self.wbits} g{self.group}"
        return s


def act_spec(lin):
    """(act_bits, act_flags) for the packed kernels' fused per-token activation fake-quant:
    (0, 0) when ``lin`` quantizes no activations, None when its act quantizer cannot be fused
    (not per-token dynamic, grouped, LWC, fix0to1)."""
    if not lin.use_act_quant or lin.disable_input_quant:
        return (0, 0)
    q = lin.act_quantizer
    if q is None or not q.enable or q.n_bits >= 16:
        return (0, 0)
    if (q.dynamic_method == "per_token" and not q.group_size and not q.lwc
            and q.metric != "fix0to1" and lin.in_features % 8 == 0):
        return (q.n_bits, q._flags())
    return None


def _same_act(members):
    specs = [act_spec(m) for m in members]
    return specs[0] if all(sp == specs[0] for sp in specs) else None


class FusedPackedLinear(nn.Module):
    """Several packed QuantLinear that read the same input (q/k/v, gate/up) as ONE fused
    dequant-GEMV/GEMM launch over their concatenated rows.

    The tiled layout concatenates along output rows tile by tile (each member's out_features must
    be a multiple of 16), so every output element is computed by exactly the kernel code path it
    takes unfused — results are bit-identical, with one launch instead of len(members)."""

    def __init__(self, members):
        super().__init__()
        if not members or not all(m.packed for m in members):
            raise ValueError("FusedPackedLinear needs packed QuantLinear members")
        m0 = members[0]
        for m in members:
            if (m.in_features, m.wbits, m.group) != (m0.in_features, m0.wbits, m0.group):
                raise ValueError("fused members must share in_features, bits and group")
            if m.out_features % qlin.TILE_N:
                raise ValueError("fused members need out_features % 16 == 0")
        self.splits = [m.out_features for m in members]
        self.in_features = m0.in_features
        self.out_features = sum(self.splits)
        self.wbits, self.group = m0.wbits, m0.group
        self.register_buffer("qweight", torch.cat([m.qweight for m in members], dim=0))
        self.register_buffer("qsz", torch.cat([m.qsz for m in members], dim=0))
        self.qflags = 0
        for m in members:
            self.qflags |= m.qflags
        biases = [m.bias for m in members]
        if any(b is not None for b in biases):
            dev, dt = self.qweight.device, torch.float16
            self.register_buffer("bias", torch.cat(
                [b.to(dt) if b is not None else torch.zeros(n, dtype=dt, device=dev)
                 for b, n in zip(biases, self.splits)]))
        else:
            self.bias = None

    def prenorm_ok(self, x, act=(0, 0)):
        """Whether ``forward_prenorm`` takes this input (one fp16 token row, no act quant)."""
        return (act == (0, 0) and x.dtype == torch.float16 and x.numel() == self.in_features
                and qlin.rmsnorm_linear_supported(1, self.out_features, self.in_features,
                                                  self.wbits, self.group))

    def forward_prenorm(self, x, norm):
        """``forward(rmsnorm(x))`` in one launch; ``norm`` = (fp32 weight, eps)."""
        y = qlin.rmsnorm_linear_ep(x.contiguous(), norm[0], norm[1], self.qweight, self.qsz,
                                   self.bias, self.out_features, self.in_features, self.wbits,
                                   self.group, self.qflags)
        return torch.split(y, self.splits, dim=-1)

    def forward(self, x, act=(0, 0)):
        """``act``: (act_bits, act_flags) of the members' shared per-token act quantizer."""
        xin = x if x.dtype == torch.float16 else x.to(torch.float16)
        y = qlin.linear_ep(xin.contiguous(), self.qweight, self.qsz, self.bias, self.out_features,
                           self.in_features, self.wbits, self.group, self.qflags,
                           act_bits=act[0], act_flags=act[1])
        if x.dtype != torch.float16:
            y = y.to(x.dtype)
        return torch.split(y, self.splits, dim=-1)


class SiluMulPackedLinear(nn.Module):
    """gate_proj + up_proj + ``act_fn(gate) * up`` (QuantLlamaMLP, SiLU) as ONE packed launch: the
    two matrices' rows interleaved in 8-row halves (``qlin.interleave_gate_up``) and the SiLU·mul
    applied in the kernel epilogue (``QLIN_EP_SILU_MUL``) on the fp16 gate / up values, so the
    [M, 2I] gate/up tensor is never written.  Same per-element arithmetic as the unfused modules
    (the dequant-matmul accumulators are identical; silu is fp32 x / (1 + exp(-x)) rounded to
    fp16 as torch's)."""

    def __init__(self, gate, up):
        super().__init__()
        if not (gate.packed and up.packed):
            raise ValueError("SiluMulPackedLinear needs packed QuantLinear members")
        if (gate.in_features, gate.out_features, gate.wbits, gate.group) != \
                (up.in_features, up.out_features, up.wbits, up.group):
            raise ValueError("gate and up must have the same shape, bits and group")
        if gate.out_features % qlin.TILE_N:
            raise ValueError("gate/up out_features must be a multiple of 16")
        self.in_features = gate.in_features
        self.out_features = gate.out_features  # of the product silu(gate) * up
        self.wbits, self.group = gate.wbits, gate.group
        qw, qsz = qlin.interleave_gate_up(gate.qweight, gate.qsz, up.qweight, up.qsz)
        self.register_buffer("qweight", qw)
        self.register_buffer("qsz", qsz)
        self.qflags = gate.qflags | up.qflags
        if gate.bias is not None or up.bias is not None:
            I, dev = self.out_features, qw.device
            z = torch.zeros(I, dtype=torch.float16, device=dev)
            gb = gate.bias.to(torch.float16) if gate.bias is not None else z
            ub = up.bias.to(torch.float16) if up.bias is not None else z
            self.register_buffer("bias", torch.stack([gb.view(-1, 8), ub.view(-1, 8)], 1).reshape(-1))
        else:
            self.bias = None

    def prenorm_ok(self, x, act=(0, 0)):
        """Whether ``forward_prenorm`` takes this input (one fp16 token row, no act quant)."""
        return (act == (0, 0) and x.dtype == torch.float16 and x.numel() == self.in_features
                and qlin.rmsnorm_linear_supported(1, 2 * self.out_features, self.in_features,
                                                  self.wbits, self.group))

    def forward_prenorm(self, x, norm):
        """``forward(rmsnorm(x))`` in one launch; ``norm`` = (fp32 weight, eps)."""
        return qlin.rmsnorm_linear_ep(x.contiguous(), norm[0], norm[1], self.qweight, self.qsz,
                                      self.bias, 2 * self.out_features, self.in_features,
                                      self.wbits, self.group, self.qflags,
                                      epilogue=qlin.EP_SILU_MUL)

    def forward(self, x, act=(0, 0)):
        xin = x if x.dtype == torch.float16 else x.to(torch.float16)
        y = qlin.linear_ep(xin.contiguous(), self.qweight, self.qsz, self.bias,
                           2 * self.out_features, self.in_features, self.wbits, self.group,
                           self.qflags, epilogue=qlin.EP_SILU_MUL, act_bits=act[0],
                           act_flags=act[1])
        return y if x.dtype == torch.float16 else y.to(x.dtype)


def packed_residual_linear(lin, x, residual):
    """``residual + lin(x)`` for a packed QuantLinear as one launch (``QLIN_EP_RESIDUAL``): the
    decoder layer's residual add fused into o_proj / down_proj's output."""
    xin = x if x.dtype == torch.float16 else x.to(torch.float16)
    bias = None if lin.bias is None else lin.bias.to(torch.float16).contiguous()
    act = act_spec(lin)
    if act is None:
        raise ValueError("the act quantizer of this linear cannot be fused")
    return qlin.linear_ep(xin.contiguous(), lin.qweight, lin.qsz, bias, lin.out_features,
                          lin.in_features, lin.wbits, lin.group, lin.qflags,
                          epilogue=qlin.EP_RESIDUAL, residual=residual.contiguous(),
                          act_bits=act[0], act_flags=act[1])
