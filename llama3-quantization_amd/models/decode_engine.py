"""DecodeEngine — one decode step (batch 1, one new token) through a stack of quantized LLaMA
decoder layers as ONE persistent gfx950 launch (``qlin_decode_llama_f16``, csrc/qlin_decode.hip).

It replaces, for q_len == 1, the chain of ``QuantLlamaDecoderLayer.forward`` calls the reference
makes per token (models/int_llama_layer.py:213-267, each QuantLinear.forward = F.linear on W_dq,
quant/int_linear.py:62), consuming exactly the operands the fused packed layer owns after
``fuse_packed_projections(kv_cache=True)``: the fused q/k/v and interleaved gate/up packed weights,
o_proj / down_proj, the RMSNorm weights (fp32) and the layer's KV-cache buffers, which it appends
to in place.  The returned ``past_key_value`` views are the same row-prefix views of those buffers
the per-layer kv_cache mode returns, so the two paths can be interleaved step by step.
"""
import math

import torch

from quant import qlin


class DecodeEngine:
    """``DecodeEngine(layers)`` over consecutive fused packed ``QuantLlamaDecoderLayer``s."""

    def __init__(self, layers):
        self.layers = list(layers)
        if not self.layers:
            raise ValueError("DecodeEngine needs at least one layer")
        at0 = self.layers[0].self_attn
        self.H = at0.hidden_size
        self.Hq = at0.num_heads
        self.Hkv = at0.num_key_value_heads
        self.D = at0.head_dim
        self.I = self.layers[0].mlp.down_proj.in_features
        self.eps = self.layers[0].input_layernorm.variance_epsilon
        self._table = None
        self._table_key = None
        self._ws = None
        self._why = self._check()

    # -- eligibility ---------------------------------------------------------------------------
    def _check(self):
        """None when every layer can run in the engine, else the reason it cannot."""
        from quant.int_linear import act_spec
        spec = None
        for layer in self.layers:
            at, mlp = layer.self_attn, layer.mlp
            if at.qkv is None or mlp.gate_up_act is None or not at.kv_cache:
                return "layer not fused with fuse_packed_projections(kv_cache=True)"
            lins = (at.q_proj, at.k_proj, at.v_proj, at.o_proj, mlp.gate_proj, mlp.up_proj,
                    mlp.down_proj)
            if not all(m.packed for m in lins):
                return "unpacked linear"
            if any(m.bias is not None for m in lins):
                return "biased linear"
            if any(act_spec(m) != (0, 0) for m in lins) or not at._attn_bypassed():
                return "activation quantization"
            s = (at.q_proj.wbits, at.q_proj.group,
                 at.qkv.qflags | at.o_proj.qflags | mlp.gate_up_act.qflags | mlp.down_proj.qflags,
                 at.hidden_size, at.num_heads, at.num_key_value_heads, at.head_dim,
                 mlp.down_proj.in_features, layer.input_layernorm.variance_epsilon,
                 layer.post_attention_layernorm.variance_epsilon)
            if any((m.wbits, m.group) != s[:2] for m in lins):
                return "mixed bits / group"
            if spec is not None and s != spec:
                return "layers differ in shape or layout"
            spec = s
            for nrm in (layer.input_layernorm, layer.post_attention_layernorm):
                if nrm.use_temporary_parameter or nrm.bias is not None:
                    return "norm with temporary parameters"
            if not hasattr(at.rotary_emb, "cos_cached"):
                return "rotary embedding without a cos/sin cache"
        self.bits, self.group, self.flags = spec[0], spec[1], spec[2]
        if spec[8] != spec[9]:
            return "input / post-attention RMSNorm epsilon differ"
        if not qlin.decode_supported(len(self.layers), self.H, self.I, self.Hq, self.Hkv, self.D,
                                     self.bits, self.group, self.flags):
            return "shape / layout not supported by qlin_decode_llama_f16"
        return None

    def supported(self, hidden_states=None, attention_mask=None, output_attentions=False):
        if self._why is not None or output_attentions:
            return False
        if hidden_states is not None:
            if (not hidden_states.is_cuda or hidden_states.dtype != torch.float16
                    or hidden_states.numel() != self.H):
                return False
        if attention_mask is not None and (attention_mask.dtype != torch.float16
                                           or attention_mask.shape[-2] != 1
                                           or attention_mask.numel() != attention_mask.shape[-1]):
            return False
        return True

    @property
    def reason(self):
        return self._why

    # -- one step ------------------------------------------------------------------------------
    def _caches(self, past, device):
        """The layers' cache buffers holding ``past`` (adopted by one copy when needed) with room
        for the new row; all layers at one length and capacity."""
        bufs, L0s = [], []
        for i, layer in enumerate(self.layers):
            pkv = None if past is None else past[i]
            buf, L0 = layer.self_attn._cache_for(pkv, 1, 1, device)
            bufs.append(buf)
            L0s.append(L0)
        if len(set(L0s)) != 1:
            raise ValueError("DecodeEngine: the layers' KV caches hold different lengths")
        L0 = L0s[0]
        if len({b[0].shape[2] for b in bufs}) != 1:
            # one capacity for all layers (the kernel takes one head stride): re-adopt each
            for i, layer in enumerate(self.layers):
                views = (bufs[i][0][:, :, :L0], bufs[i][1][:, :, :L0]) if L0 else None
                layer.self_attn.adopt_kv_cache(views, rows=L0 + 1, batch=1, device=device)
                bufs[i] = layer.self_attn._kv
        return bufs, L0

    def _pointer_table(self, bufs, device):
        ptrs = []
        for layer, (kb, vb) in zip(self.layers, bufs):
            at, mlp = layer.self_attn, layer.mlp
            ptrs += [at.qkv.qweight.data_ptr(), at.o_proj.qweight.data_ptr(),
                     mlp.gate_up_act.qweight.data_ptr(), mlp.down_proj.qweight.data_ptr(),
                     at.qkv.qsz.data_ptr(), at.o_proj.qsz.data_ptr(),
                     mlp.gate_up_act.qsz.data_ptr(), mlp.down_proj.qsz.data_ptr(),
                     layer.input_layernorm._kernel_weight().data_ptr(),
                     layer.post_attention_layernorm._kernel_weight().data_ptr(),
                     kb.data_ptr(), vb.data_ptr()]
        key = tuple(ptrs)
        if key != self._table_key:
            self._table = torch.tensor(ptrs, dtype=torch.int64).view(len(self.layers), -1).to(device)
            self._table_key = key
        return self._table

    def _workspace(self, device, L):
        n = qlin.decode_workspace_bytes(len(self.layers), self.H, self.I, self.Hq, self.Hkv,
                                        self.D, max(L, 256))
        if n < 0:
            raise ValueError("DecodeEngine: unsupported shapes")
        if self._ws is None or self._ws.numel() < n or self._ws.device != device:
            self._ws = torch.empty(max(n, 2 * (self._ws.numel() if self._ws is not None else 0)),
                                   dtype=torch.uint8, device=device)
        return self._ws

    def _rope(self, hidden_states, L):
        """The fp32 cos / sin cache the kernel reads (one for all layers: checked equal once per
        cache version, never per step — a device comparison per step would sync the host)."""
        caches = [layer.self_attn._rope_cache(hidden_states, L) for layer in self.layers]
        key = tuple((c.data_ptr(), c._version, s_.data_ptr(), s_._version) for c, s_ in caches)
        if key != getattr(self, "_rope_key", None):
            c0, s0 = caches[0]
            for c, s_ in caches[1:]:
                if (c.data_ptr() != c0.data_ptr() and not torch.equal(c, c0)) or \
                        (s_.data_ptr() != s0.data_ptr() and not torch.equal(s_, s0)):
                    raise ValueError("DecodeEngine: layers with different rotary caches")
            self._rope_key = key
        return caches[0]

    @torch.no_grad()
    def step(self, hidden_states, position_ids, past_key_values=None, attention_mask=None):
        """hidden_states fp16 [1, 1, H]; position_ids int64 (one position); past_key_values: one
        (k, v) per layer (fp16 [1, Hkv, L0, D], e.g. the views a previous step returned) or None;
        attention_mask fp16 [1, 1, 1, L0 + 1] or None.  Returns (hidden [1, 1, H], new past)."""
        if self._why is not None:
            raise ValueError(f"DecodeEngine: {self._why}")
        dev = hidden_states.device
        bufs, L0 = self._caches(past_key_values, dev)
        L = L0 + 1
        cos_c, sin_c = self._rope(hidden_states, L)
        table = self._pointer_table(bufs, dev)
        ws = self._workspace(dev, L)
        x = hidden_states.reshape(-1).contiguous()
        y = torch.empty_like(x)
        pos = position_ids.reshape(-1)[:1].to(device=dev, dtype=torch.int64).contiguous()
        mask = None
        if attention_mask is not None:
            mask = attention_mask.reshape(-1).contiguous()
            if mask.numel() != L:
                raise ValueError(f"attention mask covers {mask.numel()} keys, expected {L}")
        qlin.decode_llama(table, len(self.layers), self.H, self.I, self.Hq, self.Hkv, self.D,
                          self.bits, self.group, self.flags, self.eps, x, y, cos_c, sin_c, pos,
                          L0, bufs[0][0].shape[2], mask, math.sqrt(self.D), ws)
        past = [(kb[:, :, :L], vb[:, :, :L]) for kb, vb in bufs]
        return y.view(1, 1, self.H), past

    def status(self):
        """The workspace's error word after the last step (0 = completed; syncs the stream)."""
        if self._ws is None:
            return 0
        return int(self._ws[:4].view(torch.int32).item())
