"""QuantLlamaDecoderLayer — per-layer dispatch of the reference (models/int_llama_layer.py:20-368).

7 QuantLinear (q/k/v/o, gate/up/down) + 2 QuantMatMul (QK^T, PV) + 2 RMSNorm per layer, same
constructor signature ``(config, ori_layer, args)`` and forward signature as the reference.

RoPE follows the transformers-4.37.2 contract the reference was written against
(``rotary_emb(x, seq_len)`` -> cos/sin cache in x.dtype; ``apply_rotary_pos_emb(q, k, cos, sin,
position_ids)``), restated here because the installed transformers no longer has it.

Dtype policy (documented deviation): the reference casts q to fp32 (:117) but not
k/v, so its fp16 path raises in QK^T; here k and v are promoted to q's dtype for the two
attention matmuls (fp32 attention core, as the reference intends), and the attention output is
cast back to the layer's activation dtype before o_proj.  In fp32 this is exactly the reference.
"""
import math
from typing import Optional, Tuple

import torch
from torch import nn

from quant import qlin
from quant.int_linear import (FusedPackedLinear, QuantLinear, SiluMulPackedLinear, _same_act,
                              act_spec, packed_residual_linear)
from quant.int_matmul import QuantMatMul
from quant.omni_norm import KERNEL_MAX_ROWS, OmniLlamaRMSNorm


def _rope_theta(config):
    if getattr(config, "rope_theta", None) is not None:
        return float(config.rope_theta)
    rp = getattr(config, "rope_parameters", None) or {}
    return float(rp.get("rope_theta", 10000.0))


class LlamaRotaryEmbedding437(nn.Module):
    """cos/sin cache with the transformers-4.37.2 LlamaRotaryEmbedding semantics."""

    def __init__(self, dim, max_position_embeddings=2048, base=10000, device=None):
        super().__init__()
        self.dim = dim
        self.max_position_embeddings = max_position_embeddings
        self.base = base
        inv_freq = 1.0 / (self.base ** (torch.arange(0, self.dim, 2, device=device).float() / self.dim))
        self.register_buffer("inv_freq", inv_freq, persistent=False)
        self._set_cos_sin_cache(max_position_embeddings, device)

    def _set_cos_sin_cache(self, seq_len, device):
        self.max_seq_len_cached = seq_len
        t = torch.arange(seq_len, device=device, dtype=self.inv_freq.dtype)
        freqs = torch.outer(t, self.inv_freq.to(t.device))
        emb = torch.cat((freqs, freqs), dim=-1)
        self.register_buffer("cos_cached", emb.cos(), persistent=False)
        self.register_buffer("sin_cached", emb.sin(), persistent=False)

    def forward(self, x, seq_len=None):
        if seq_len > self.max_seq_len_cached:
            self._set_cos_sin_cache(seq_len, x.device)
        return (self.cos_cached[:seq_len].to(device=x.device, dtype=x.dtype),
                self.sin_cached[:seq_len].to(device=x.device, dtype=x.dtype))


def rotate_half(x):
    x1 = x[..., : x.shape[-1] // 2]
    x2 = x[..., x.shape[-1] // 2:]
    return torch.cat((-x2, x1), dim=-1)


def apply_rotary_pos_emb(q, k, cos, sin, position_ids, unsqueeze_dim=1):
    cos = cos[position_ids].unsqueeze(unsqueeze_dim)
    sin = sin[position_ids].unsqueeze(unsqueeze_dim)
    return (q * cos) + (rotate_half(q) * sin), (k * cos) + (rotate_half(k) * sin)


def repeat_kv(hidden_states: torch.Tensor, n_rep: int) -> torch.Tensor:
    b, h, s, d = hidden_states.shape
    if n_rep == 1:
        return hidden_states
    hidden_states = hidden_states[:, :, None, :, :].expand(b, h, n_rep, s, d)
    return hidden_states.reshape(b, h * n_rep, s, d)


def _act(name):
    if name == "silu":
        return nn.functional.silu
    if name == "relu":
        return nn.functional.relu
    if name in ("gelu", "gelu_new", "gelu_pytorch_tanh"):
        return (lambda x: nn.functional.gelu(x, approximate="tanh")) if name != "gelu" else nn.functional.gelu
    raise ValueError(f"unsupported hidden_act {name}")


class QuantLlamaMLP(nn.Module):
    def __init__(self, org_module: nn.Module, hidden_size: int, intermediate_size: int,
                 hidden_act: str, args=None):
        super().__init__()
        self.gate_proj = QuantLinear(org_module.gate_proj, args.weight_quant_params, args.act_quant_params)
        self.down_proj = QuantLinear(org_module.down_proj, args.weight_quant_params, args.act_quant_params)
        self.up_proj = QuantLinear(org_module.up_proj, args.weight_quant_params, args.act_quant_params)
        self.act_fn = _act(hidden_act)
        self.hidden_act = hidden_act
        self.gate_up = None  # FusedPackedLinear after fuse_packed()
        self.gate_up_act = None  # SiluMulPackedLinear after fuse_packed() (SiLU models)

    def fuse_packed(self):
        """gate_proj + up_proj as one fused packed launch (both read x); with SiLU the activation
        product is applied in that launch's epilogue."""
        if self.hidden_act == "silu" and self.gate_proj.out_features % 16 == 0:
            self.gate_up_act = SiluMulPackedLinear(self.gate_proj, self.up_proj)
        else:
            self.gate_up = FusedPackedLinear([self.gate_proj, self.up_proj])
        return self

    def fused(self):
        """Fused packed launches apply (their per-token act quantizers, if any, fuse too)."""
        return (self.gate_up is not None or self.gate_up_act is not None) and \
            _same_act([self.gate_proj, self.up_proj]) is not None and \
            act_spec(self.down_proj) is not None

    def forward(self, x, residual=None, prenorm=None):
        """``down(act(gate(x)) * up(x))``; with ``residual`` (fused packed mode only) the
        decoder layer's ``residual + mlp(x)`` is folded into down_proj's epilogue; ``prenorm``
        (fused packed mode): x is the hidden state BEFORE that RMSNorm module, applied here — for
        one token row inside the gate/up launch (qlin.rmsnorm_linear_ep)."""
        if self.fused():
            act = _same_act([self.gate_proj, self.up_proj])
            lin = self.gate_up_act if self.gate_up_act is not None else self.gate_up
            norm = prenorm.fusable(x) if prenorm is not None else None
            if norm is not None and lin.prenorm_ok(x, act):
                out = lin.forward_prenorm(x, norm)
            else:
                if prenorm is not None:
                    x = prenorm(x)
                out = lin(x, act)
            if self.gate_up_act is not None:
                h = out
            else:
                gate, up = out
                h = self.act_fn(gate) * up
            if residual is not None:
                return packed_residual_linear(self.down_proj, h, residual)
            return self.down_proj(h)
        if prenorm is not None:
            x = prenorm(x)
        out = self.down_proj(self.act_fn(self.gate_proj(x)) * self.up_proj(x))
        return out if residual is None else residual + out


class QuantLlamaAttention(nn.Module):
    """Multi-headed attention from 'Attention Is All You Need' paper"""

    def __init__(self, org_module: nn.Module, config, args=None):
        super().__init__()
        self.config = config
        self.hidden_size = config.hidden_size
        self.num_heads = config.num_attention_heads
        self.head_dim = self.hidden_size // self.num_heads
        self.num_key_value_heads = config.num_key_value_heads
        self.num_key_value_groups = self.num_heads // self.num_key_value_heads
        self.max_position_embeddings = config.max_position_embeddings
        if (self.head_dim * self.num_heads) != self.hidden_size:
            raise ValueError(
                f"hidden_size must be divisible by num_heads (got `hidden_size`: {self.hidden_size}"
                f" and `num_heads`: {self.num_heads}).")
        rot = getattr(org_module, "rotary_emb", None)
        if rot is not None and hasattr(rot, "cos_cached"):
            self.rotary_emb = rot
        else:
            self.rotary_emb = LlamaRotaryEmbedding437(
                self.head_dim, self.max_position_embeddings, _rope_theta(config),
                device=org_module.q_proj.weight.device)
        self.k_proj = QuantLinear(org_module.k_proj, args.weight_quant_params, args.act_quant_params)
        self.v_proj = QuantLinear(org_module.v_proj, args.weight_quant_params, args.act_quant_params)
        self.q_proj = QuantLinear(org_module.q_proj, args.weight_quant_params, args.act_quant_params)
        self.o_proj = QuantLinear(org_module.o_proj, args.weight_quant_params, args.act_quant_params)
        self.qkt_matmul = QuantMatMul(args.q_quant_params, args.k_quant_params, matmul_func=torch.matmul)
        self.pv_matmul = QuantMatMul(args.p_quant_params, args.v_quant_params, matmul_func=torch.matmul)
        self.use_weight_quant = False
        self.use_act_quant = False
        self.qkv = None  # FusedPackedLinear after fuse_packed()
        self.decode_kernel = False  # qlin_attn_decode for one-token steps (fuse_packed turns it on)
        self.rope_kernel = False  # qlin_rope_f16 (fuse_packed turns it on)
        self.prefill_kernel = False  # qlin_attn_prefill for multi-token windows (opt-in)
        self.kv_cache = False  # rope + KV append into a preallocated cache (opt-in)
        self._kv = None  # (k, v) cache buffers [B, Hkv, rows, D] of the kv_cache mode

    def fuse_packed(self, prefill_attention: bool = False, kv_cache: bool = False):
        """q_proj + k_proj + v_proj as one fused packed launch (all read the normed hidden), and
        the fused decode-attention kernel for one-token steps; ``prefill_attention`` also routes
        multi-token windows through the fused prefill-attention kernel (fp32, online softmax:
        equal to the reference attention to fp32 rounding instead of bit for bit).

        ``kv_cache``: with ``use_cache`` / a ``past_key_value``, RoPE writes the step's k and v
        rows straight into cache buffers owned by the module and the returned ``past_key_value``
        are row-prefix views of them, so a decode step appends two rows instead of re-copying the
        whole cache (the reference's ``torch.cat``, models/int_llama_layer.py:130-135; the values
        are identical).  A ``past_key_value`` that is not such a view (the first step, a reordered
        beam) is copied into a fresh buffer once.  Two continuations of the SAME past share its
        buffer and overwrite each other's next row, so this is opt-in."""
        self.qkv = FusedPackedLinear([self.q_proj, self.k_proj, self.v_proj])
        self.decode_kernel = True
        self.rope_kernel = hasattr(self.rotary_emb, "cos_cached")
        self.prefill_kernel = bool(prefill_attention)
        self.kv_cache = bool(kv_cache)
        return self

    def adopt_kv_cache(self, past_key_value, rows=None, batch=1, device=None):
        """kv_cache mode: copy ``past_key_value`` (fp16 [B, Hkv, L, D] each, or None) into fresh
        cache buffers with room to grow (2x the rows needed, at least 256) and return it as views
        of them, which later steps append to in place."""
        H, D = self.num_key_value_heads, self.head_dim
        L0 = past_key_value[0].shape[-2] if past_key_value is not None else 0
        if past_key_value is not None:
            batch, device = past_key_value[0].shape[0], past_key_value[0].device
        need = max(L0, rows or 0)
        cap = max(256, (2 * need + 255) // 256 * 256)
        kb = torch.empty(batch, H, cap, D, dtype=torch.float16, device=device)
        vb = torch.empty_like(kb)
        if past_key_value is not None:
            kb[:, :, :L0].copy_(past_key_value[0])
            vb[:, :, :L0].copy_(past_key_value[1])
        self._kv = (kb, vb)
        return (kb[:, :, :L0], vb[:, :, :L0])

    def _cache_for(self, past, bsz, q_len, device):
        """kv_cache mode: the cache buffers with ``past`` as their row prefix and room for
        ``q_len`` more rows (adopting ``past`` by one copy when it is not such a view)."""
        H, D = self.num_key_value_heads, self.head_dim
        L0 = past[0].shape[-2] if past is not None else 0
        buf = self._kv
        inplace = (past is not None and buf is not None and L0 + q_len <= buf[0].shape[2]
                   and past[0].data_ptr() == buf[0].data_ptr()
                   and past[1].data_ptr() == buf[1].data_ptr()
                   and tuple(past[0].shape) == (bsz, H, L0, D)
                   and tuple(past[1].shape) == (bsz, H, L0, D)
                   and past[0].stride() == buf[0].stride() and past[1].stride() == buf[1].stride())
        if not inplace:
            self.adopt_kv_cache(past, rows=L0 + q_len, batch=bsz, device=device)
        return self._kv, L0

    def _rope_append(self, q, k, v, cos_c, sin_c, position_ids, past, bsz, q_len):
        """kv_cache mode: RoPE + the cache append in one launch (qlin_rope_kv_f16); returns
        (query_states, key_states, value_states) with k / v as views of the cache buffers."""
        H, D = self.num_key_value_heads, self.head_dim
        buf, L0 = self._cache_for(past, bsz, q_len, q.device)
        need = L0 + q_len
        query_states = qlin.rope_kv(q, k, v, cos_c, sin_c, position_ids, self.num_heads, H, D,
                                    buf[0], buf[1], L0)
        return query_states, buf[0][:, :, :need], buf[1][:, :, :need]

    def _attn_bypassed(self):
        """QuantMatMul quantizers are identity (abits >= 16 or act quant off)."""
        for mm in (self.qkt_matmul, self.pv_matmul):
            if mm.use_act_quant and (mm.x1_quantizer.n_bits < 16 or mm.x2_quantizer.n_bits < 16):
                return False
        return True

    def _project(self, hidden_states, prenorm=None):
        """q, k, v of the (normed) hidden state; ``prenorm``: hidden_states is the input of that
        RMSNorm module, applied here — for one token row inside the fused q/k/v launch."""
        if self.qkv is not None:
            act = _same_act([self.q_proj, self.k_proj, self.v_proj])
            if act is not None:
                norm = prenorm.fusable(hidden_states) if prenorm is not None else None
                if norm is not None and self.qkv.prenorm_ok(hidden_states, act):
                    return self.qkv.forward_prenorm(hidden_states, norm)
                if prenorm is not None:
                    hidden_states = prenorm(hidden_states)
                return self.qkv(hidden_states, act)
        if prenorm is not None:
            hidden_states = prenorm(hidden_states)
        return self.q_proj(hidden_states), self.k_proj(hidden_states), self.v_proj(hidden_states)

    def _decode_kernel_ok(self, hidden_states, attention_mask, past_key_value, use_cache,
                          output_attentions, kv_seq_len):
        """Whether this step takes the one-launch RoPE + KV append + decode attention path."""
        q_len = hidden_states.shape[1]
        kv_mode = self.kv_cache and (use_cache or past_key_value is not None) and \
            (past_key_value is None or past_key_value[0].dtype == torch.float16)
        return (self.rope_kernel and hidden_states.dtype == torch.float16 and hidden_states.is_cuda
                and kv_mode and q_len == 1 and self.decode_kernel and not output_attentions
                and self._attn_bypassed() and self.head_dim == qlin.ATTN_D
                and kv_seq_len <= qlin.ATTN_MAX_L
                and self.num_heads // self.num_key_value_heads in (1, 2, 4, 8)
                and (attention_mask is None or (attention_mask.dtype == torch.float16
                                                and attention_mask.shape[-2] == 1)))

    def _rope_cache(self, value_states, kv_seq_len):
        """fp32 views of the rotary cos/sin cache (grown exactly as rotary_emb() grows it); a
        cache held in fp16 (after .half()) is upcast once, exactly."""
        rot = self.rotary_emb
        if kv_seq_len > rot.max_seq_len_cached:
            rot(value_states, seq_len=kv_seq_len)  # the reference's cache growth
        c, s_ = rot.cos_cached, rot.sin_cached
        key = (c.data_ptr(), c.dtype, c.shape)
        if getattr(self, "_rope32_key", None) != key:
            self._rope32 = (c.float().contiguous(), s_.float().contiguous())
            self._rope32_key = key
        return self._rope32

    # graph-replayed decode steps (models/pipeline.py generate(graphs=True)): an int32 device
    # tensor holding the step's cache length; the step then reads nothing on the host (no past /
    # mask / length checks), appends to and attends over the kv_cache buffers in self._kv;
    # _dyn_max: the longest length the captured steps reach (None: the buffers' capacity), which
    # sizes the attention grid and must stay within qlin.ATTN_MAX_L
    _dyn_len = None
    _dyn_max = None

    def _decode_step_len(self, hidden_states, position_ids, residual, prenorm):
        """One token through the fused packed attention with the cache length on the device
        (qlin_attn_decode_rope_len over self._kv's capacity): a launch sequence that stays valid
        for every step, so it can be captured once and replayed."""
        bsz = hidden_states.shape[0]
        act_dtype = hidden_states.dtype
        if not (self.kv_cache and self._kv is not None and act_dtype == torch.float16
                and position_ids is not None):
            raise ValueError("device-length decode needs kv_cache buffers, fp16 and position_ids")
        q, k, v = self._project(hidden_states, prenorm)
        buf = self._kv
        cos_c, sin_c = self._rope_cache(buf[0], buf[0].shape[2])
        attn = qlin.attn_decode_rope_len(q, k, v, cos_c, sin_c, position_ids, self.num_heads,
                                         self.num_key_value_heads, self.head_dim, buf[0], buf[1],
                                         self._dyn_len, out_dtype=torch.float16,
                                         max_len=self._dyn_max)
        attn = attn.transpose(1, 2).reshape(bsz, 1, self.hidden_size)
        return self._out(attn, residual), None, None

    def _out(self, attn_output, residual):
        if residual is None:
            return self.o_proj(attn_output)
        if self.o_proj.packed and act_spec(self.o_proj) is not None:
            return packed_residual_linear(self.o_proj, attn_output, residual)
        return residual + self.o_proj(attn_output)

    def _shape(self, tensor: torch.Tensor, seq_len: int, bsz: int):
        return tensor.view(bsz, seq_len, self.num_heads, self.head_dim).transpose(1, 2).contiguous()

    def forward(
        self,
        hidden_states: torch.Tensor,
        attention_mask: Optional[torch.Tensor] = None,
        position_ids: Optional[torch.LongTensor] = None,
        past_key_value: Optional[Tuple[torch.Tensor]] = None,
        output_attentions: bool = False,
        use_cache: bool = False,
        residual: Optional[torch.Tensor] = None,
        prenorm=None,
    ):
        """``residual`` (fused packed mode, set by the decoder layer): the output is
        ``residual + o_proj(attn)``, the add folded into o_proj's epilogue; ``prenorm``: the
        input_layernorm module, applied to hidden_states here (inside the q/k/v launch for one
        token row)."""
        bsz, q_len, _ = hidden_states.size()
        act_dtype = hidden_states.dtype
        if self._dyn_len is not None and q_len == 1:
            return self._decode_step_len(hidden_states, position_ids, residual, prenorm)
        kv_seq_len = q_len
        if past_key_value is not None:
            kv_seq_len += past_key_value[0].shape[-2]
        if position_ids is None:
            position_ids = torch.arange(kv_seq_len - q_len, kv_seq_len, device=hidden_states.device)[None]
        decode = self._decode_kernel_ok(hidden_states, attention_mask, past_key_value, use_cache,
                                        output_attentions, kv_seq_len)
        q, k, v = self._project(hidden_states, prenorm)
        value_states = v.reshape(bsz, q_len, self.num_key_value_heads, self.head_dim).transpose(1, 2)
        appended = False
        if self.rope_kernel and q.dtype == torch.float16 and q.is_cuda:
            # one launch: reshape/transpose, q -> fp32, cos/sin slice + cast, apply_rotary_pos_emb
            cos_c, sin_c = self._rope_cache(value_states, kv_seq_len)
            kv_mode = self.kv_cache and (use_cache or past_key_value is not None) and \
                (past_key_value is None or past_key_value[0].dtype == torch.float16)
            if decode:
                # one launch: RoPE, the cache append and the decode attention
                buf, L0 = self._cache_for(past_key_value, bsz, 1, q.device)
                attn_output = qlin.attn_decode_rope(
                    q, k, v, cos_c, sin_c, position_ids, self.num_heads, self.num_key_value_heads,
                    self.head_dim, buf[0], buf[1], L0, attention_mask, math.sqrt(self.head_dim),
                    out_dtype=act_dtype if act_dtype == torch.float16 else torch.float32)
                past_key_value = (buf[0][:, :, :L0 + 1], buf[1][:, :, :L0 + 1]) if use_cache else None
                attn_output = attn_output.transpose(1, 2).reshape(bsz, q_len, self.hidden_size).to(act_dtype)
                return self._out(attn_output, residual), None, past_key_value
            if kv_mode:
                # ... plus the cache append (kv_cache mode)
                query_states, key_states, value_states = self._rope_append(
                    q, k, v, cos_c, sin_c, position_ids, past_key_value, bsz, q_len)
                appended = True
            else:
                query_states, key_states = qlin.rope(q, k, cos_c, sin_c, position_ids,
                                                     self.num_heads, self.num_key_value_heads,
                                                     self.head_dim)
        else:
            query_states = q.reshape(bsz, q_len, self.num_heads, self.head_dim).transpose(1, 2).type(torch.float32)
            key_states = k.reshape(bsz, q_len, self.num_key_value_heads, self.head_dim).transpose(1, 2)
            cos, sin = self.rotary_emb(value_states, seq_len=kv_seq_len)
            query_states, key_states = apply_rotary_pos_emb(query_states, key_states, cos, sin, position_ids)

        if past_key_value is not None and not appended:
            key_states = torch.cat([past_key_value[0], key_states], dim=2)
            value_states = torch.cat([past_key_value[1], value_states], dim=2)
        past_key_value = (key_states, value_states) if use_cache else None

        if (self.decode_kernel and q_len == 1 and not output_attentions and self._attn_bypassed()
                and qlin.attn_decode_supported(query_states, key_states, attention_mask)):
            # fused decode attention: same fp32 arithmetic as the path below (repeat_kv, QK^T,
            # / sqrt(d), + mask, clamp, softmax, PV) up to summation order
            attn_output = qlin.attn_decode(query_states, key_states, value_states, attention_mask,
                                           math.sqrt(self.head_dim),
                                           out_dtype=act_dtype if act_dtype == torch.float16
                                           else torch.float32)
            attn_output = attn_output.transpose(1, 2).reshape(bsz, q_len, self.hidden_size).to(act_dtype)
            return self._out(attn_output, residual), None, past_key_value

        if (self.prefill_kernel and q_len > 1 and not output_attentions and self._attn_bypassed()
                and qlin.attn_prefill_supported(query_states, key_states, attention_mask)):
            # fused prefill attention: repeat_kv, QK^T, / sqrt(d), + mask, clamp, softmax and PV
            # in one kernel (fp32 matrix cores, online softmax), output already in the
            # transpose(1, 2) layout and, for fp16 activations, rounded once to fp16
            attn_output = qlin.attn_prefill(query_states, key_states, value_states, attention_mask,
                                            math.sqrt(self.head_dim),
                                            out_dtype=act_dtype if act_dtype == torch.float16
                                            else torch.float32)
            attn_output = attn_output.reshape(bsz, q_len, self.hidden_size).to(act_dtype)
            return self._out(attn_output, residual), None, past_key_value

        key_states = repeat_kv(key_states, self.num_key_value_groups)
        value_states = repeat_kv(value_states, self.num_key_value_groups)

        query_states = self.qkt_matmul.quant_x1(query_states)
        key_states = self.qkt_matmul.quant_x2(key_states)
        attn_weights = self.qkt_matmul(query_states, key_states.to(query_states.dtype).transpose(2, 3))

        if attn_weights.size() != (bsz, self.num_heads, q_len, kv_seq_len):
            raise ValueError(
                f"Attention weights should be of size {(bsz, self.num_heads, q_len, kv_seq_len)}, but is"
                f" {attn_weights.size()}")
        if attention_mask is not None and attention_mask.size() != (bsz, 1, q_len, kv_seq_len):
            raise ValueError(
                f"Attention mask should be of size {(bsz, 1, q_len, kv_seq_len)}, but is {attention_mask.size()}")
        fused_scores = (self.rope_kernel and attn_weights.is_cuda
                        and attn_weights.dtype == torch.float32
                        and attn_weights.is_contiguous() and kv_seq_len % 4 == 0)
        if fused_scores:
            # fused mode: / sqrt(d), + mask, clamp as one in-place pass (bit-exact)
            attn_weights = qlin.attn_scores_(attn_weights, attention_mask, math.sqrt(self.head_dim))
        else:
            attn_weights = attn_weights / math.sqrt(self.head_dim)
        if attention_mask is not None and not fused_scores:
            attn_weights = attn_weights + attention_mask
            # == torch.max(w, torch.tensor(finfo.min)) of the reference (:155-157), without the
            # host->device scalar copy (keeps the layer capturable in a HIP graph)
            attn_weights = attn_weights.clamp_min(torch.finfo(attn_weights.dtype).min)

        attn_weights = nn.functional.softmax(attn_weights, dim=-1, dtype=torch.float32).to(query_states.dtype)
        attn_weights = self.pv_matmul.quant_x1(attn_weights)
        value_states = self.pv_matmul.quant_x2(value_states)
        attn_output = self.pv_matmul(attn_weights, value_states.to(attn_weights.dtype))

        if attn_output.size() != (bsz, self.num_heads, q_len, self.head_dim):
            raise ValueError(
                f"`attn_output` should be of size {(bsz, self.num_heads, q_len, self.head_dim)}, but is"
                f" {attn_output.size()}")
        attn_output = attn_output.transpose(1, 2).reshape(bsz, q_len, self.hidden_size).to(act_dtype)
        attn_output = self._out(attn_output, residual)
        if not output_attentions:
            attn_weights = None
        return attn_output, attn_weights, past_key_value

    def set_quant_state(self, weight_quant: bool = False, act_quant: bool = False):
        self.use_weight_quant = weight_quant
        self.use_act_quant = act_quant
        for m in self.modules():
            if isinstance(m, (QuantLinear, QuantMatMul)):
                m.set_quant_state(weight_quant, act_quant)


class QuantLlamaDecoderLayer(nn.Module):
    def __init__(self, config, ori_layer, args):
        super().__init__()
        self.hidden_size = config.hidden_size
        self.self_attn = QuantLlamaAttention(org_module=ori_layer.self_attn, config=config, args=args)
        self.mlp = QuantLlamaMLP(org_module=ori_layer.mlp, hidden_size=self.hidden_size,
                                 intermediate_size=config.intermediate_size,
                                 hidden_act=config.hidden_act, args=args)
        self.input_layernorm = OmniLlamaRMSNorm(ori_layer.input_layernorm, eps=ori_layer.input_layernorm.variance_epsilon)
        self.post_attention_layernorm = OmniLlamaRMSNorm(ori_layer.post_attention_layernorm, eps=ori_layer.post_attention_layernorm.variance_epsilon)
        self.let = False
        self.fused_epilogues = False  # fuse_packed_projections() turns it on

    def forward(
        self,
        hidden_states: torch.Tensor,
        attention_mask: Optional[torch.Tensor] = None,
        position_ids: Optional[torch.LongTensor] = None,
        past_key_value: Optional[Tuple[torch.Tensor]] = None,
        output_attentions: Optional[bool] = False,
        use_cache: Optional[bool] = False,
    ):
        residual = hidden_states
        if self.fused_epilogues and self.mlp.fused():
            # fused packed mode: both residual adds run in the o_proj / down_proj epilogues
            # (same fp16 arithmetic: RN16(residual + RN16(linear))), and both RMSNorms are handed
            # to the q/k/v and gate/up launches (applied inside them for one token row)
            hidden_states, self_attn_weights, present_key_value = self.self_attn(
                hidden_states=hidden_states, attention_mask=attention_mask,
                position_ids=position_ids, past_key_value=past_key_value,
                output_attentions=output_attentions, use_cache=use_cache, residual=residual,
                prenorm=self.input_layernorm)
            residual = hidden_states
            hidden_states = self.mlp(hidden_states, residual=residual,
                                     prenorm=self.post_attention_layernorm)
        else:
            hidden_states = self.input_layernorm(hidden_states)
            hidden_states, self_attn_weights, present_key_value = self.self_attn(
                hidden_states=hidden_states, attention_mask=attention_mask,
                position_ids=position_ids, past_key_value=past_key_value,
                output_attentions=output_attentions, use_cache=use_cache)
            hidden_states = residual + hidden_states
            residual = hidden_states
            hidden_states = self.post_attention_layernorm(hidden_states)
            hidden_states = self.mlp(hidden_states)
            hidden_states = residual + hidden_states
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

    def fuse_packed_projections(self, prefill_attention: bool = False, kv_cache: bool = False):
        """After packing: q/k/v and gate/up (+ SiLU·mul) each become one fused launch, and the two
        residual adds move into the o_proj / down_proj epilogues;
        ``prefill_attention``: multi-token windows also take the fused prefill-attention kernel;
        ``kv_cache``: decode steps append to a preallocated KV cache (QuantLlamaAttention.fuse_packed)."""
        self.self_attn.fuse_packed(prefill_attention, kv_cache)
        self.mlp.fuse_packed()
        self.fused_epilogues = self.self_attn.o_proj.packed and self.mlp.down_proj.packed
        self.input_layernorm.use_kernel = True
        self.post_attention_layernorm.use_kernel = True
        # windows too take the RMSNorm kernel once the attention is no longer bit-exact anyway
        rows = None if prefill_attention else KERNEL_MAX_ROWS
        self.input_layernorm.kernel_max_rows = rows
        self.post_attention_layernorm.kernel_max_rows = rows
        return self

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
