"""Whole-model driver around QuantLlamaDecoderLayer: the slice of the reference's L0-L2 that the
hot path needs — build the quantized decoder stack from HF-style modules (a loaded
checkpoint or a random-init LLaMA3 skeleton), RTN-quantize it exactly as ``omniquant()`` does with
``epochs == 0`` (quant/omniquant.py:195-314), optionally pack every linear for the gfx950 kernels,
and evaluate logits / perplexity as ``main.py:evaluate`` does (main.py:102-154).
"""
from types import SimpleNamespace

import torch
from torch import nn

from quant.omni_norm import OmniLlamaRMSNorm
from quant.utils import pack_quant_linears, set_quant_state
from .int_llama_layer import QuantLlamaDecoderLayer


def quant_args(wbits=4, group_size=128, abits=16, symmetric=False, disable_zero_point=False,
               lwc=False):
    """The quant-param dicts of main.py:317-353."""
    a = SimpleNamespace()
    a.wbits, a.abits, a.group_size = wbits, abits, group_size
    a.let = False
    a.weight_quant_params = dict(n_bits=wbits, per_channel_axes=[0], symmetric=symmetric,
                                 dynamic_method="per_channel", group_size=group_size, lwc=lwc,
                                 disable_zero_point=disable_zero_point)
    act = dict(n_bits=abits, per_channel_axes=[], symmetric=False, dynamic_method="per_token")
    a.act_quant_params = dict(act)
    a.q_quant_params = dict(act)
    a.k_quant_params = dict(act)
    a.v_quant_params = dict(act)
    a.p_quant_params = dict(n_bits=16, metric="fix0to1")
    return a


class _Norm(nn.Module):
    def __init__(self, h, eps, device, dtype):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(h, device=device, dtype=dtype), requires_grad=False)
        self.variance_epsilon = eps


def _linear(n_in, n_out, gen, device, dtype, std):
    lin = nn.Linear(n_in, n_out, bias=False, device=device, dtype=dtype)
    with torch.no_grad():
        lin.weight.normal_(0.0, std, generator=gen)
    lin.weight.requires_grad_(False)
    return lin


def random_llama_layer(config, seed, device="cuda", dtype=torch.float16, std=0.02):
    """An HF-shaped LlamaDecoderLayer skeleton (self_attn.{q,k,v,o}_proj, mlp.{gate,up,down}_proj,
    two RMSNorms) with N(0, std^2) weights drawn on the device."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    H, I = config.hidden_size, config.intermediate_size
    hd = H // config.num_attention_heads
    kv = config.num_key_value_heads * hd
    L = nn.Module()
    L.self_attn = nn.Module()
    L.self_attn.q_proj = _linear(H, H, g, device, dtype, std)
    L.self_attn.k_proj = _linear(H, kv, g, device, dtype, std)
    L.self_attn.v_proj = _linear(H, kv, g, device, dtype, std)
    L.self_attn.o_proj = _linear(H, H, g, device, dtype, std)
    L.mlp = nn.Module()
    L.mlp.gate_proj = _linear(H, I, g, device, dtype, std)
    L.mlp.up_proj = _linear(H, I, g, device, dtype, std)
    L.mlp.down_proj = _linear(I, H, g, device, dtype, std)
    eps = getattr(config, "rms_norm_eps", 1e-5)
    L.input_layernorm = _Norm(H, eps, device, dtype)
    L.post_attention_layernorm = _Norm(H, eps, device, dtype)
    return L


def causal_mask(bsz, T, dtype, device, past=0):
    m = torch.full((T, T + past), torch.finfo(dtype).min, dtype=dtype, device=device)
    m = torch.triu(m, diagonal=1 + past)
    return m[None, None].expand(bsz, 1, T, T + past)


class QuantLlamaForEval(nn.Module):
    """embed -> QuantLlamaDecoderLayer x L -> RMSNorm -> lm_head (LlamaForCausalLM forward with the
    reference's quantized layers in place of HF's, as omniquant() leaves the model)."""

    def __init__(self, config, layers, embed, norm, lm_head):
        super().__init__()
        self.config = config
        self.embed_tokens = embed
        self.layers = nn.ModuleList(layers)
        self.norm = norm
        self.lm_head = lm_head

    def hidden(self, input_ids, layer_range=None):
        h = self.embed_tokens(input_ids)
        return self.run_layers(h, layer_range)

    def run_layers(self, h, layer_range=None):
        bsz, T = h.shape[:2]
        mask = causal_mask(bsz, T, h.dtype, h.device)
        pos = torch.arange(T, device=h.device)[None].expand(bsz, T)
        lo, hi = layer_range or (0, len(self.layers))
        for layer in self.layers[lo:hi]:
            h = layer(h, attention_mask=mask, position_ids=pos)[0]
        return h

    def head(self, h):
        return self.lm_head(self.norm(h))

    def forward(self, input_ids):
        return self.head(self.hidden(input_ids))


def build_random_quant_llama(config, args, seed=0, device="cuda", dtype=torch.float16,
                             n_layers=None, layer_ids=None):
    """Random-init LLaMA-architecture model (no checkpoints offline): weights N(0, 0.02^2),
    embeddings N(0, 1), norms 1.  ``layer_ids`` builds only those layers (pipeline stages)."""
    L = n_layers or config.num_hidden_layers
    ids = list(range(L)) if layer_ids is None else list(layer_ids)
    layers = [QuantLlamaDecoderLayer(config, random_llama_layer(config, seed * 1000 + i, device, dtype), args)
              for i in ids]
    g = torch.Generator(device=device)
    g.manual_seed(seed * 1000 + 999)
    embed = nn.Embedding(config.vocab_size, config.hidden_size, device=device, dtype=dtype)
    with torch.no_grad():
        embed.weight.normal_(0.0, 1.0, generator=g)
    eps = getattr(config, "rms_norm_eps", 1e-5)
    norm = OmniLlamaRMSNorm(_Norm(config.hidden_size, eps, device, dtype), eps=eps)
    lm_head = _linear(config.hidden_size, config.vocab_size, g, device, dtype, 0.02)
    model = QuantLlamaForEval(config, layers, embed, norm, lm_head)
    model.layer_ids = ids
    return model


@torch.no_grad()
def rtn_quantize_(model, pack=False):
    """omniquant() with epochs == 0 (quant/omniquant.py:296-314): per layer .half() ->
    smooth_and_quant_inplace -> register_scales_and_zeros; optionally the real-quant pack."""
    for layer in model.layers:
        layer.half()
        layer.smooth_and_quant_inplace()
        layer.register_scales_and_zeros()
        set_quant_state(layer, weight_quant=False, act_quant=layer_act_quant(layer))
        if pack:
            pack_quant_linears(layer)
    return model


def layer_act_quant(layer):
    for m in layer.modules():
        q = getattr(m, "act_quantizer", None)
        if q is not None and q.n_bits < 16:
            return True
    return False


def nll_from_logits(logits, tokens):
    """main.py:136-146: CE over the shifted logits (in the logits' dtype), times seqlen."""
    shift_logits = logits[:, :-1, :]
    shift_labels = tokens[:, 1:]
    loss = nn.functional.cross_entropy(shift_logits.reshape(-1, shift_logits.size(-1)),
                                       shift_labels.reshape(-1))
    return loss.float() * tokens.shape[1]


@torch.no_grad()
def window_nll(model, tokens):
    """Σ NLL of one window exactly as main.py:136-146."""
    return nll_from_logits(model(tokens), tokens)


@torch.no_grad()
def eval_ppl(model, testenc, seqlen=2048, limit=-1):
    """main.py:119-151: nsamples = numel // seqlen windows; ppl = exp(Σ nll / (nsamples*seqlen))."""
    nsamples = testenc.numel() // seqlen
    nlls = []
    for i in range(nsamples):
        batch = testenc[:, i * seqlen:(i + 1) * seqlen].to(model.lm_head.weight.device)
        nlls.append(window_nll(model, batch))
        if i == limit:
            break
    return torch.exp(torch.stack(nlls).sum() / (nsamples * seqlen)).item()
