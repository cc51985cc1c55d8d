"""QuantOPTDecoderLayer — per-layer dispatch of the reference (models/int_opt_layer.py:16-452).

Biased q/k/v/out projections, ReLU FFN (fc1/fc2) and bmm attention with fp32 softmax, every linear
a QuantLinear (config 1 of BASELINE.json: OPT-125M int8).  LET smoothing is out of scope.
"""
from typing import Optional, Tuple

import torch
from torch import nn
import torch.nn.functional as F

from quant.int_linear import QuantLinear
from quant.int_matmul import QuantMatMul
from quant.omni_norm import OmniLayerNorm


class QuantOPTAttention(nn.Module):
    """Multi-headed attention from 'Attention Is All You Need' paper"""

    def __init__(self, org_module: nn.Module, embed_dim: int, num_heads: int, dropout: float = 0.0,
                 is_decoder: bool = False, bias: bool = True, args=None, disable_act_quant=False):
        super().__init__()
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.dropout = dropout
        self.head_dim = embed_dim // num_heads
        if (self.head_dim * num_heads) != self.embed_dim:
            raise ValueError(
                f"embed_dim must be divisible by num_heads (got `embed_dim`: {self.embed_dim}"
                f" and `num_heads`: {num_heads}).")
        self.scaling = self.head_dim ** -0.5
        self.is_decoder = is_decoder
        self.k_proj = QuantLinear(org_module.k_proj, args.weight_quant_params, args.act_quant_params)
        self.v_proj = QuantLinear(org_module.v_proj, args.weight_quant_params, args.act_quant_params)
        self.q_proj = QuantLinear(org_module.q_proj, args.weight_quant_params, args.act_quant_params)
        self.out_proj = QuantLinear(org_module.out_proj, args.weight_quant_params, args.act_quant_params)
        self.qkt_matmul = QuantMatMul(args.q_quant_params, args.k_quant_params, matmul_func=torch.bmm)
        self.pv_matmul = QuantMatMul(args.p_quant_params, args.v_quant_params, matmul_func=torch.bmm)
        self.use_weight_quant = False
        self.use_act_quant = False

    def _shape(self, tensor: torch.Tensor, seq_len: int, bsz: int):
        return tensor.view(bsz, seq_len, self.num_heads, self.head_dim).transpose(1, 2).contiguous()

    def forward(self, hidden_states: torch.Tensor, key_value_states: Optional[torch.Tensor] = None,
                past_key_value: Optional[Tuple[torch.Tensor]] = None,
                attention_mask: Optional[torch.Tensor] = None,
                layer_head_mask: Optional[torch.Tensor] = None, output_attentions: bool = False):
        is_cross_attention = key_value_states is not None
        bsz, tgt_len, _ = hidden_states.size()
        query_states = self.q_proj(hidden_states) * self.scaling
        query_states = self.qkt_matmul.quant_x1(query_states)
        if is_cross_attention and past_key_value is not None:
            key_states, value_states = past_key_value[0], past_key_value[1]
        elif is_cross_attention:
            key_states = self._shape(self.qkt_matmul.quant_x2(self.k_proj(key_value_states)), -1, bsz)
            value_states = self._shape(self.v_proj(key_value_states), -1, bsz)
        else:
            key_states = self._shape(self.qkt_matmul.quant_x2(self.k_proj(hidden_states)), -1, bsz)
            value_states = self._shape(self.pv_matmul.quant_x2(self.v_proj(hidden_states)), -1, bsz)
            if past_key_value is not None:
                key_states = torch.cat([past_key_value[0], key_states], dim=2)
                value_states = torch.cat([past_key_value[1], value_states], dim=2)
        if self.is_decoder:
            past_key_value = (key_states, value_states)

        proj_shape = (bsz * self.num_heads, -1, self.head_dim)
        query_states = self._shape(query_states, tgt_len, bsz).view(*proj_shape)
        key_states = key_states.reshape(*proj_shape)
        value_states = value_states.reshape(*proj_shape)
        src_len = key_states.size(1)
        attn_weights = self.qkt_matmul(query_states, key_states.transpose(1, 2))
        if attn_weights.size() != (bsz * self.num_heads, tgt_len, src_len):
            raise ValueError(
                f"Attention weights should be of size {(bsz * self.num_heads, tgt_len, src_len)}, but is"
                f" {attn_weights.size()}")
        if attention_mask is not None:
            if attention_mask.size() != (bsz, 1, tgt_len, src_len):
                raise ValueError(
                    f"Attention mask should be of size {(bsz, 1, tgt_len, src_len)}, but is {attention_mask.size()}")
            attn_weights = attn_weights.view(bsz, self.num_heads, tgt_len, src_len) + attention_mask
            attn_weights = attn_weights.clamp_min(torch.finfo(attn_weights.dtype).min)  # == torch.max(w, tensor(min))
            attn_weights = attn_weights.view(bsz * self.num_heads, tgt_len, src_len)
        if attn_weights.dtype == torch.float16:
            attn_weights = nn.functional.softmax(attn_weights, dim=-1, dtype=torch.float32).to(torch.float16)
        else:
            attn_weights = nn.functional.softmax(attn_weights, dim=-1)
        if layer_head_mask is not None:
            if layer_head_mask.size() != (self.num_heads,):
                raise ValueError(
                    f"Head mask for a single layer should be of size {(self.num_heads,)}, but is {layer_head_mask.size()}")
            attn_weights = layer_head_mask.view(1, -1, 1, 1) * attn_weights.view(bsz, self.num_heads, tgt_len, src_len)
            attn_weights = attn_weights.view(bsz * self.num_heads, tgt_len, src_len)
        attn_probs_reshaped = None
        if output_attentions:
            attn_probs_reshaped = attn_weights.view(bsz, self.num_heads, tgt_len, src_len)
        attn_weights = self.pv_matmul.quant_x1(attn_weights)
        attn_output = self.pv_matmul(attn_weights, value_states)
        if attn_output.size() != (bsz * self.num_heads, tgt_len, self.head_dim):
            raise ValueError(
                f"`attn_output` should be of size {(bsz, self.num_heads, tgt_len, self.head_dim)}, but is"
                f" {attn_output.size()}")
        attn_output = attn_output.view(bsz, self.num_heads, tgt_len, self.head_dim).transpose(1, 2)
        attn_output = attn_output.reshape(bsz, tgt_len, self.embed_dim)
        attn_output = self.out_proj(attn_output)
        return attn_output, attn_probs_reshaped, past_key_value

    def set_quant_state(self, weight_quant: bool = False, act_quant: bool = False):
        self.use_weight_quant = weight_quant
        self.use_act_quant = act_quant
        for m in self.modules():
            if isinstance(m, (QuantLinear, QuantMatMul)):
                m.set_quant_state(weight_quant, act_quant)


class QuantOPTDecoderLayer(nn.Module):
    def __init__(self, config, ori_layer, args):
        super().__init__()
        self.embed_dim = config.hidden_size
        self.self_attn = QuantOPTAttention(
            org_module=ori_layer.self_attn, embed_dim=self.embed_dim,
            num_heads=config.num_attention_heads, dropout=config.attention_dropout, is_decoder=True,
            bias=getattr(config, "enable_bias", True), args=args)
        self.do_layer_norm_before = config.do_layer_norm_before
        self.dropout = config.dropout
        self.self_attn_layer_norm = OmniLayerNorm(ori_layer.self_attn_layer_norm)
        self.fc1 = QuantLinear(ori_layer.fc1, weight_quant_params=args.weight_quant_params,
                               act_quant_params=args.act_quant_params)
        self.fc2 = QuantLinear(ori_layer.fc2, weight_quant_params=args.weight_quant_params,
                               act_quant_params=args.act_quant_params)
        self.final_layer_norm = OmniLayerNorm(ori_layer.final_layer_norm)
        self.type = ori_layer.fc1.weight.dtype
        self.let = False

    def forward(self, hidden_states: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                layer_head_mask: Optional[torch.Tensor] = None,
                output_attentions: Optional[bool] = False, use_cache: Optional[bool] = False,
                past_key_value: Optional[Tuple[torch.Tensor]] = None, **kwargs):
        residual = hidden_states
        if self.do_layer_norm_before:
            hidden_states = self.self_attn_layer_norm(hidden_states)
        hidden_states, self_attn_weights, present_key_value = self.self_attn(
            hidden_states=hidden_states, past_key_value=past_key_value,
            attention_mask=attention_mask, layer_head_mask=layer_head_mask,
            output_attentions=output_attentions)
        hidden_states = residual + hidden_states
        if not self.do_layer_norm_before:
            hidden_states = self.self_attn_layer_norm(hidden_states)
        hidden_states_shape = hidden_states.shape
        hidden_states = hidden_states.reshape(-1, hidden_states.size(-1))
        residual = hidden_states
        if self.do_layer_norm_before:
            hidden_states = self.final_layer_norm(hidden_states)
        hidden_states = self.fc1(hidden_states)
        hidden_states = F.relu(hidden_states)
        hidden_states = self.fc2(hidden_states)
        hidden_states = (residual + hidden_states).view(hidden_states_shape)
        if not self.do_layer_norm_before:
            hidden_states = self.final_layer_norm(hidden_states)
        outputs = (hidden_states,)
        if output_attentions:
            outputs += (self_attn_weights,)
        if use_cache:
            outputs += (present_key_value,)
        return outputs

    def set_quant_state(self, weight_quant: bool = False, act_quant: bool = False):
        self.use_weight_quant = weight_quant
        self.use_act_quant = act_quant
        for name, m in self.named_modules():
            if isinstance(m, (QuantLinear, QuantMatMul)):
                m.set_quant_state(weight_quant, act_quant)

    @torch.no_grad()
    def smooth_and_quant_inplace(self):
        if self.let:
            raise NotImplementedError("LET smoothing is out of scope for the MI355X hot path")
        for name, module in self.named_modules():
            if isinstance(module, QuantLinear):
                module.weight = module.weight_quantizer(module.weight)
                module.use_temporary_parameter = False

    def register_scales_and_zeros(self):
        for name, module in self.named_modules():
            if isinstance(module, QuantLinear):
                module.weight_quantizer.register_scales_and_zeros()
