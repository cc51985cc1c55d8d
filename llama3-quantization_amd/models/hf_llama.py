"""Local Hugging Face LLaMA checkpoints and wikitext2 text -> the quantized evaluation model
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

from quant.omni_norm import OmniLlamaRMSNorm
from .int_llama_layer import QuantLlamaDecoderLayer
from .quant_llama import QuantLlamaForEval


def load_hf_llama(path: str, dtype=torch.float16, device="cpu"):
    """LlamaForCausalLM from a local directory (models/LMClass.py:39-41 loads it in fp16)."""
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
