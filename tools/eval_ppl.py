#!/usr/bin/env python3
"""Wikitext2 perplexity of a local LLaMA (or OPT) checkpoint, RTN-quantized as the reference's main.py
does (``--wbits 4 --group_size 128 --epochs 0 [--real_quant]``), on one MI355X:

  python tools/eval_ppl.py --model /path/to/Meta-Llama-3-8B --data /path/to/wikitext2_test \\
      --wbits 4 --group 128 [--abits 16] [--mode fake|packed|fused] [--limit N]

--mode fake:   the reference's eval path (weight = W_dq, dense fp16 F.linear)
--mode packed: the --real_quant path on the gfx950 kernels (pack_quant_linears)
--mode fused:  packed + fused q/k/v, gate/up(+SiLU), residual epilogues, RoPE (fuse_packed_projections)
--data: a token file (.npy/.pt) or the wikitext2 test split on local disk (save_to_disk dir,
        .parquet, .arrow, raw .txt); nothing is downloaded.
Prints one JSON line: ppl, windows, ms per window.  The PPL formula is main.py:119-151's
(nsamples = numel // seqlen windows; --limit stops early but keeps nsamples in the denominator,
as the reference does)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))

import torch  # noqa: E402

from models.hf_llama import load_hf_llama, quant_model_from_hf, wikitext2_test_ids  # noqa: E402
from models.quant_llama import nll_from_logits, quant_args, rtn_quantize_  # noqa: E402
from quant.utils import pack_quant_linears  # noqa: E402


def run(a):
    dev = torch.device(a.device)
    model = load_hf_llama(a.model, torch.float16 if a.dtype == "fp16" else torch.float32, dev)
    tok = None
    if not (a.data.endswith(".npy") or a.data.endswith(".pt")):
        from transformers import AutoTokenizer
        tok = AutoTokenizer.from_pretrained(a.model, local_files_only=True)
    ids = wikitext2_test_ids(a.data, tok)
    q = quant_model_from_hf(model, quant_args(a.wbits, a.group or None, a.abits))
    if a.wbits < 16:
        rtn_quantize_(q, pack=a.mode in ("packed", "fused"))
        if a.mode == "fused":
            for layer in q.layers:
                if hasattr(layer, "fuse_packed_projections"):  # LLaMA layers
                    layer.fuse_packed_projections()
    seqlen = a.seqlen
    nsamples = ids.numel() // seqlen
    nlls, ms = [], []
    with torch.no_grad():
        for i in range(nsamples):
            batch = ids[:, i * seqlen:(i + 1) * seqlen].to(dev)
            if dev.type == "cuda":
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            logits = q(batch)
            nlls.append(nll_from_logits(logits, batch))
            if dev.type == "cuda":
                torch.cuda.synchronize()
            ms.append((time.perf_counter() - t0) * 1e3)
            if i == a.limit:
                break
    ppl = torch.exp(torch.stack(nlls).sum() / (nsamples * seqlen)).item()
    return {"ppl": ppl, "windows": len(nlls), "nsamples": nsamples, "seqlen": seqlen,
            "mode": a.mode, "wbits": a.wbits, "group": a.group, "abits": a.abits,
            "ms_per_window": round(sum(ms[1:]) / max(1, len(ms) - 1) if len(ms) > 1 else ms[0], 2)}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", required=True)
    ap.add_argument("--data", required=True)
    ap.add_argument("--wbits", type=int, default=4)
    ap.add_argument("--group", type=int, default=128, help="0: per-channel (no groups)")
    ap.add_argument("--abits", type=int, default=16)
    ap.add_argument("--seqlen", type=int, default=2048)
    ap.add_argument("--mode", choices=("fake", "packed", "fused"), default="packed")
    ap.add_argument("--limit", type=int, default=-1)
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--dtype", choices=("fp16", "fp32"), default="fp16")
    return ap.parse_args(argv)


if __name__ == "__main__":
    print(json.dumps(run(parse())), flush=True)
