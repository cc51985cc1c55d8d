"""The main.py-style evaluation path on local HF checkpoints (models/hf_llama.py, tools/eval_ppl.py):
a tiny random LlamaForCausalLM saved to disk and reloaded offline.  CPU: the conversion to
QuantLlamaDecoderLayer reproduces the HF model's own logits (no quantization) and the PPL formula
is main.py's.  GPU: RTN int4 g128 fake-quant vs packed vs fused packed PPL."""
import math
import os
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))


def _tiny_model(path, dtype=torch.float32):
    from transformers import LlamaConfig, LlamaForCausalLM
    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_attention_heads=4,
                      num_key_value_heads=2, num_hidden_layers=2, vocab_size=512,
                      max_position_embeddings=512, rms_norm_eps=1e-5, rope_theta=500000.0,
                      tie_word_embeddings=False)
    torch.manual_seed(0)
    m = LlamaForCausalLM(cfg).to(dtype).eval()
    m.save_pretrained(path)
    return m


def _tokens(path, n=4 * 128 + 17):
    ids = np.random.RandomState(1).randint(0, 512, size=n).astype(np.int64)
    np.save(path, ids)
    return ids


def test_conversion_matches_hf_forward(tmp_path):
    from models.hf_llama import load_hf_llama, quant_llama_from_hf
    from models.quant_llama import quant_args
    _tiny_model(tmp_path / "m")
    hf = load_hf_llama(str(tmp_path / "m"), torch.float32, "cpu")
    q = quant_llama_from_hf(hf, quant_args(16, 128))
    ids = torch.from_numpy(np.random.RandomState(2).randint(0, 512, size=(1, 40)))
    with torch.no_grad():
        ref = hf(ids).logits
        got = q(ids)
    rel = ((got - ref).abs().max() / ref.abs().max()).item()
    assert rel < 1e-4, rel


def test_eval_ppl_tool_formula(tmp_path):
    import eval_ppl
    _tiny_model(tmp_path / "m")
    ids = _tokens(tmp_path / "ids.npy")
    out = eval_ppl.run(eval_ppl.parse(["--model", str(tmp_path / "m"), "--data",
                                       str(tmp_path / "ids.npy"), "--wbits", "16",
                                       "--seqlen", "128", "--device", "cpu", "--dtype", "fp32",
                                       "--mode", "fake"]))
    assert out["nsamples"] == 4 and out["windows"] == 4
    # main.py:136-151 by hand with HF's own model
    from models.hf_llama import load_hf_llama
    hf = load_hf_llama(str(tmp_path / "m"), torch.float32, "cpu")
    t = torch.from_numpy(ids[: 4 * 128]).reshape(4, 128)
    with torch.no_grad():
        nll = sum(torch.nn.functional.cross_entropy(hf(t[i:i + 1]).logits[0, :-1], t[i, 1:]).item() * 128
                  for i in range(4))
    assert abs(out["ppl"] - math.exp(nll / 512)) / out["ppl"] < 1e-4


@pytest.mark.gpu
def test_eval_ppl_tool_quantized_modes(tmp_path):
    import eval_ppl
    _tiny_model(tmp_path / "m", torch.float16)
    _tokens(tmp_path / "ids.npy", n=3 * 256)
    res = {}
    for mode in ("fake", "packed", "fused"):
        res[mode] = eval_ppl.run(eval_ppl.parse(["--model", str(tmp_path / "m"), "--data",
                                                 str(tmp_path / "ids.npy"), "--wbits", "4",
                                                 "--group", "128", "--seqlen", "256", "--mode",
                                                 mode]))["ppl"]
    assert np.isfinite(res["fake"])
    for mode in ("packed", "fused"):
        assert abs(res[mode] - res["fake"]) / res["fake"] < 1e-3, res


def _tiny_opt(path, dtype=torch.float32):
    from transformers import OPTConfig, OPTForCausalLM
    cfg = OPTConfig(hidden_size=128, ffn_dim=512, num_attention_heads=4, num_hidden_layers=2,
                    vocab_size=512, max_position_embeddings=512, word_embed_proj_dim=128)
    torch.manual_seed(0)
    m = OPTForCausalLM(cfg).to(dtype).eval()
    m.save_pretrained(path)
    return m


def test_opt_conversion_matches_hf_forward(tmp_path):
    """BASELINE configs[0]'s model family: OPTForCausalLM -> QuantOPTDecoderLayer stack."""
    from models.hf_llama import load_hf_llama, quant_model_from_hf
    from models.quant_llama import quant_args
    _tiny_opt(tmp_path / "opt")
    hf = load_hf_llama(str(tmp_path / "opt"), torch.float32, "cpu")
    q = quant_model_from_hf(hf, quant_args(16, 128))
    ids = torch.from_numpy(np.random.RandomState(3).randint(0, 512, size=(1, 33)))
    with torch.no_grad():
        ref = hf(ids).logits
        got = q(ids)
    rel = ((got - ref).abs().max() / ref.abs().max()).item()
    assert rel < 1e-4, rel


@pytest.mark.gpu
def test_opt_int8_per_channel_packed_vs_fake(tmp_path):
    """BASELINE configs[0]: OPT int8 per-channel weights (biased linears), fake-quant vs packed."""
    import eval_ppl
    _tiny_opt(tmp_path / "opt", torch.float16)
    _tokens(tmp_path / "ids.npy", n=2 * 256)
    res = {mode: eval_ppl.run(eval_ppl.parse(["--model", str(tmp_path / "opt"), "--data",
                                              str(tmp_path / "ids.npy"), "--wbits", "8",
                                              "--group", "0", "--seqlen", "256", "--mode",
                                              mode]))["ppl"] for mode in ("fake", "packed")}
    assert np.isfinite(res["fake"]) and abs(res["packed"] - res["fake"]) / res["fake"] < 1e-3, res
