"""Norm layers of the quantized decoder layers (reference quant/omni_norm.py:11-63).

RMSNorm is computed in fp32 and cast back, exactly as the reference does, with torch ops on the
device; in the fused packed decoder layer (``use_kernel``, set by
``QuantLlamaDecoderLayer.fuse_packed_projections``) decode-sized inputs (<= 64 rows) take one
gfx950 launch (``qlin_rmsnorm_f16``, same arithmetic, sum of squares in another order); with the
prefill-attention kernel (already equal to the reference to fp32 rounding, not bit for bit) every
input does (``kernel_max_rows = None``).
"""
import torch
import torch.nn as nn

from . import qlin


class OmniLayerNorm(nn.Module):
    def __init__(self, ori_layer_norm) -> None:
        super().__init__()
        self.use_act_quant = True
        self.register_buffer("weight", ori_layer_norm.weight)
        if ori_layer_norm.bias is not None:
            self.register_buffer("bias", ori_layer_norm.bias)
        else:
            self.bias = None
        self.eps = ori_layer_norm.eps
        self.norm_func = nn.functional.layer_norm
        self.normalized_shape = ori_layer_norm.normalized_shape
        self.use_temporary_parameter = False

    def forward(self, x):
        if self.use_temporary_parameter:
            weight, bias = self.temp_weight, self.temp_bias
        else:
            weight, bias = self.weight, self.bias
        return self.norm_func(x, self.normalized_shape, weight, bias, eps=self.eps)

    def set_quant_state(self, use_weight_quant, use_act_quant):
        self.use_act_quant = use_act_quant


# the kernel serves decode-sized inputs (its sum-of-squares order differs from torch's reduction,
# so it can move an fp16 ulp); prefill windows keep the reference's torch ops, where the norm is
# a negligible share of the layer and the fused layer stays bit-identical to the unfused one
KERNEL_MAX_ROWS = 64


class OmniLlamaRMSNorm(nn.Module):
    def __init__(self, ori_norm, eps=1e-6):
        super().__init__()
        self.register_buffer("weight", ori_norm.weight)
        self.bias = None
        self.variance_epsilon = eps
        self.use_temporary_parameter = False
        self.use_kernel = False
        self.kernel_max_rows = KERNEL_MAX_ROWS  # None: every input takes the kernel
        self._w32 = None

    def _kernel_weight(self):
        w = self.weight
        if self._w32 is None or self._w32[0] is not w or self._w32[1] != w._version:
            self._w32 = (w, w._version, w.detach().to(torch.float32).contiguous())
        return self._w32[2]

    def fusable(self, hidden_states):
        """(weight, eps) when the next packed linear may apply this norm itself
        (qlin.rmsnorm_linear_ep: the kernel path, one fp16 token row), else None.  An fp16 module
        weight goes as it is (the kernel reads fp16 weights: half the bytes, same result), any
        other as its fp32 copy."""
        if (self.use_kernel and not self.use_temporary_parameter and self.bias is None
                and hidden_states.is_cuda and hidden_states.dtype == torch.float16
                and hidden_states.numel() == hidden_states.shape[-1]):
            w = self.weight
            if w.dtype == torch.float16 and w.is_contiguous():
                return w.detach(), self.variance_epsilon
            return self._kernel_weight(), self.variance_epsilon
        return None

    def forward(self, hidden_states):
        if (self.use_kernel and not self.use_temporary_parameter and self.bias is None
                and hidden_states.is_cuda and hidden_states.dtype == torch.float16
                and (self.kernel_max_rows is None
                     or hidden_states.numel() <= self.kernel_max_rows * hidden_states.shape[-1])):
            return qlin.rmsnorm(hidden_states.contiguous(), self._kernel_weight(),
                                self.variance_epsilon)
        input_dtype = hidden_states.dtype
        variance = hidden_states.to(torch.float32).pow(2).mean(-1, keepdim=True)
        hidden_states = hidden_states * torch.rsqrt(variance + self.variance_epsilon)
        if self.use_temporary_parameter:
            weight, bias = self.temp_weight, self.temp_bias
        else:
            weight, bias = self.weight, self.bias
        # weight (fp16) * hidden (fp32) promotes to fp32: multiplying by the fp32 copy of the
        # weight is the same arithmetic (fp16 -> fp32 is exact) and takes PyTorch's vectorised
        # same-dtype kernel instead of the mixed-dtype one (measured 41 us vs ~3 us per call on
        # MI355X for a 4096-wide decode token)
        if weight.dtype != hidden_states.dtype:
            weight = weight.to(hidden_states.dtype)
        if bias is not None:
            return (weight * hidden_states + bias).to(input_dtype)
        return (weight * hidden_states).to(input_dtype)
