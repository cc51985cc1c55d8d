"""Local Hugging Face LLaMA / OPT checkpoints and wikitext2 text -> the quantized evaluation model
(the reference's main.py path: LMClass loads the model (models/LMClass.py:26-45), omniquant()
wraps every decoder layer in QuantLlamaDecoderLayer and RTN-quantizes it (quant/omniquant.py:
195-314 with epochs = 0), evaluate() runs the wikitext2 perplexity loop (main.py:102-154) on
datautils.get_wikitext2's test encoding (datautils.py:35-51)).

Offline only: the model directory and the dataset must already be on local disk
(``local_files_only``); nothing is downloaded.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from torch import nn

from quant.omni_norm import OmniLlamaRMSNorm
from .int_llama_layer import QuantLlamaDecoderLayer
from .int_opt_layer import QuantOPTDecoderLayer
from .quant_llama import QuantLlamaForEval, causal_mask


def load_hf_llama(path: str, dtype=torch.float16, device="cpu"):
    """LlamaForCausalLM / OPTForCausalLM from a local directory (models/LMClass.py:39-41 loads it
    in fp16)."""
    from transformers import AutoModelForCausalLM
    model = AutoModelForCausalLM.from_pretrained(path, torch_dtype=dtype, local_files_only=True)
    return model.to(device).eval()


@torch.no_grad()
def quant_llama_from_hf(model, args):
    """Wrap an HF LlamaForCausalLM the way omniquant() does: every decoder layer becomes a
    QuantLlamaDecoderLayer (sharing the HF weights), the final norm an OmniLlamaRMSNorm."""
    cfg = model.config
    layers = [QuantLlamaDecoderLayer(cfg, layer, args) for layer in model.model.layers]
    n = model.model.norm
    norm = OmniLlamaRMSNorm(n, eps=getattr(n, "variance_epsilon", getattr(n, "eps", 1e-6)))
    q = QuantLlamaForEval(cfg, layers, model.model.embed_tokens, norm, model.lm_head)
    q.layer_ids = list(range(len(layers)))
    return q


class QuantOPTForEval(nn.Module):
    """OPTForCausalLM's decoder with the reference's QuantOPTDecoderLayer in place of HF's
    (BASELINE configs[0]: OPT-125M): token + learned position embeddings (offset 2, no padding),
    optional project_in / project_out, the causal additive mask, final LayerNorm, lm_head."""

    def __init__(self, config, hf_decoder, layers, lm_head):
        super().__init__()
        self.config = config
        self.embed_tokens = hf_decoder.embed_tokens
        self.embed_positions = hf_decoder.embed_positions
        self.project_in = getattr(hf_decoder, "project_in", None)
        self.project_out = getattr(hf_decoder, "project_out", None)
        self.final_layer_norm = getattr(hf_decoder, "final_layer_norm", None)
        self.layers = nn.ModuleList(layers)
        self.lm_head = lm_head

    def forward(self, input_ids):
        bsz, T = input_ids.shape
        h = self.embed_tokens(input_ids)
        if self.project_in is not None:
            h = self.project_in(h)
        pos = torch.arange(T, device=input_ids.device) + getattr(self.embed_positions, "offset", 2)
        h = h + self.embed_positions.weight[pos][None].to(h.dtype)
        mask = causal_mask(bsz, T, h.dtype, h.device)
        for layer in self.layers:
            h = layer(h, attention_mask=mask)[0]
        if self.final_layer_norm is not None:
            h = self.final_layer_norm(h)
        if self.project_out is not None:
            h = self.project_out(h)
        return self.lm_head(h)


@torch.no_grad()
def quant_model_from_hf(model, args):
    """LLaMA or OPT (config.model_type) -> the quantized evaluation model."""
    if model.config.model_type == "opt":
        layers = [QuantOPTDecoderLayer(model.config, layer, args)
                  for layer in model.model.decoder.layers]
        q = QuantOPTForEval(model.config, model.model.decoder, layers, model.lm_head)
        q.layer_ids = list(range(len(layers)))
        return q
    if model.config.model_type == "llama":
        return quant_llama_from_hf(model, args)
    raise NotImplementedError(f"model_type {model.config.model_type!r} (LLaMA and OPT only)")


def wikitext2_test_ids(source: str, tokenizer=None) -> torch.Tensor:
    """The wikitext2 test encoding as datautils.get_wikitext2 builds it:
    tokenizer("\\n\\n".join(test["text"]), return_tensors="pt").input_ids, [1, T].

    ``source``: a token file (.npy / .pt of int ids: used as is), a datasets.save_to_disk
    directory, a .parquet / .arrow file of the split, or a raw .txt file."""
    if source.endswith(".npy"):
        return torch.from_numpy(np.load(source, allow_pickle=False).astype(np.int64)).reshape(1, -1)
    if source.endswith(".pt"):
        return torch.load(source, weights_only=True).to(torch.int64).reshape(1, -1)
    if tokenizer is None:
        raise ValueError("a tokenizer is needed to encode text")
    if os.path.isdir(source):
        from datasets import load_from_disk
        ds = load_from_disk(source)
        text = "\n\n".join(ds["test"]["text"] if "test" in ds else ds["text"])
    elif source.endswith(".parquet"):
        import pandas as pd
        text = "\n\n".join(pd.read_parquet(source)["text"].tolist())
    elif source.endswith(".arrow"):
        from datasets import Dataset
        text = "\n\n".join(Dataset.from_file(source)["text"])
    else:
        with open(source, encoding="utf-8") as f:
            text = f.read()
    return tokenizer(text, return_tensors="pt").input_ids
