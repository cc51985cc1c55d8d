"""GPU parity of the per-layer dispatch (models/int_llama_layer.py, models/int_opt_layer.py) against
the reference layers' golden outputs, and of the packed HIP path against the fake-quant path."""
import hashlib

import numpy as np
import pytest
import torch

from conftest import load_golden
from golden_common import LLAMA_CFG, OPT_CFG, layer_weights
from helpers import n, t

pytestmark = pytest.mark.gpu

from models.int_llama_layer import QuantLlamaDecoderLayer  # noqa: E402
from models.int_opt_layer import QuantOPTDecoderLayer  # noqa: E402
from models.quant_llama import quant_args  # noqa: E402
from quant.int_linear import QuantLinear  # noqa: E402
from quant.utils import pack_quant_linears, set_quant_state  # noqa: E402


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def rel_max_err(y, ref):
    y = np.asarray(y, np.float64)
    ref = np.asarray(ref, np.float64)
    return np.abs(y - ref).max() / np.abs(ref).max()


def hf_llama_layer():
    from transformers import LlamaConfig
    from transformers.models.llama.modeling_llama import LlamaDecoderLayer
    cfg = LlamaConfig(**LLAMA_CFG)
    hf = LlamaDecoderLayer(cfg, layer_idx=0)
    with torch.no_grad():
        params = dict(hf.named_parameters())
        for k, v in layer_weights("llama", LLAMA_CFG, seed=2024).items():
            params[k].copy_(torch.from_numpy(v))
    return cfg, hf.cuda()


def hf_opt_layer():
    from transformers import OPTConfig
    from transformers.models.opt.modeling_opt import OPTDecoderLayer
    cfg = OPTConfig(**OPT_CFG)
    hf = OPTDecoderLayer(cfg, layer_idx=0)
    with torch.no_grad():
        params = dict(hf.named_parameters())
        for k, v in layer_weights("opt", OPT_CFG, seed=125).items():
            params[k].copy_(torch.from_numpy(v))
    return cfg, hf.cuda()


def quantize_fp16(q):
    q.half()
    q.smooth_and_quant_inplace()
    q.register_scales_and_zeros()
    return {name.replace(".", "_"): sha(n(m.weight)) for name, m in q.named_modules()
            if isinstance(m, QuantLinear)}


def test_llama_layer_matches_reference():
    g = load_golden("llama_layer_fp32")
    cfg, hf = hf_llama_layer()
    x, mask, pos = t(g["x"]), t(g["mask"]), t(g["pos"])
    # unquantized (w16) fp32 forward: pins RoPE / GQA / softmax / RMSNorm semantics
    q16 = QuantLlamaDecoderLayer(cfg, hf, quant_args(16, None))
    with torch.no_grad():
        y16 = q16(x, attention_mask=mask, position_ids=pos)[0]
    assert rel_max_err(n(y16), g["y_w16"]) < 1e-5
    # RTN int4 g128 in fp16 through the HIP quantizer: W_dq bit-exact with the reference's
    cfg, hf = hf_llama_layer()
    q = QuantLlamaDecoderLayer(cfg, hf, quant_args(4, 128)).cuda()
    hashes = quantize_fp16(q)
    for k, v in hashes.items():
        assert v == str(g[f"sha_{k}_w4"]), k
    q.float()
    with torch.no_grad():
        y = q(x, attention_mask=mask, position_ids=pos)[0]
    assert rel_max_err(n(y), g["y_w4"]) < 1e-5
    # fp16 activations: the reference's own fake-quant path run in fp16 (dense F.linear on W_dq)
    # sets the error budget of the packed path against the reference's fp32 output — the packed
    # path may not be measurably worse than the reference arithmetic it replaces
    q.half()
    xh, mh = x.half(), mask.half()
    with torch.no_grad():
        yf = q(xh, attention_mask=mh, position_ids=pos)[0]
    err_fq = rel_max_err(n(yf), g["y_w4"])
    pack_quant_linears(q)
    with torch.no_grad():
        yp = q(xh, attention_mask=mh, position_ids=pos)[0]
    err_pk = rel_max_err(n(yp), g["y_w4"])
    assert err_fq < 1e-2 and err_pk <= 1.25 * err_fq + 1e-4, (err_pk, err_fq)


def test_llama_packed_equals_fake_quant_fp16():
    """The north-star logits criterion at layer level: packed HIP path within 1e-3 (relative to
    max) of the reference fake-quant path (dense F.linear on W_dq) on identical fp16 inputs."""
    g = load_golden("llama_layer_fp32")
    cfg, hf = hf_llama_layer()
    q = QuantLlamaDecoderLayer(cfg, hf, quant_args(4, 128)).cuda()
    quantize_fp16(q)
    x, mask, pos = t(g["x"]).half(), t(g["mask"]).half(), t(g["pos"])
    with torch.no_grad():
        y_fq = q(x, attention_mask=mask, position_ids=pos)[0]
        pack_quant_linears(q)
        y_pk = q(x, attention_mask=mask, position_ids=pos)[0]
    assert rel_max_err(n(y_pk), n(y_fq)) < 1e-3


@pytest.mark.parametrize("abits", [16, 8])
def test_opt_layer_matches_reference(abits):
    g = load_golden("opt_layer_fp32")
    cfg, hf = hf_opt_layer()
    q = QuantOPTDecoderLayer(cfg, hf, quant_args(8, None, abits)).cuda()
    hashes = quantize_fp16(q)
    tag = f"w8a{abits}"
    for k, v in hashes.items():
        assert v == str(g[f"sha_{k}_{tag}"]), k
    set_quant_state(q, weight_quant=False, act_quant=abits < 16)
    q.float()
    x, mask = t(g["x"]), t(g["mask"])
    with torch.no_grad():
        y = q(x, attention_mask=mask)[0]
    tol = 1e-5 if abits == 16 else 2e-3  # A8: a code may flip where GPU fp32 rounding differs
    assert rel_max_err(n(y), g["y_" + tag]) < tol
    q.half()
    with torch.no_grad():
        y_fq = q(x.half(), attention_mask=mask.half())[0]
        pack_quant_linears(q)
        y_pk = q(x.half(), attention_mask=mask.half())[0]
    assert rel_max_err(n(y_pk), n(y_fq)) < (1e-3 if abits == 16 else 5e-3)
    assert rel_max_err(n(y_pk), g["y_" + tag]) < 2e-2


def test_quant_matmul_a8_matches_reference():
    """QuantMatMul with per-token 8-bit activation quantizers on both operands (the reference's
    quant_x1 / quant_x2 + matmul, quant/int_matmul.py:31-42) on the GPU: the HIP quantizer's
    operands equal the oracle's bit for bit and the product equals the reference's own output
    (tests/golden/mm_a8_f32.npz, written by importing the reference) to fp32 summation order."""
    from oracle import quant_oracle as O
    from quant.int_matmul import QuantMatMul
    g = load_golden("mm_a8_f32")
    qp = dict(n_bits=8, per_channel_axes=[], symmetric=False, dynamic_method="per_token")
    mm = QuantMatMul(qp, qp, matmul_func=torch.matmul).cuda()
    x1, x2 = t(g["x1"]), t(g["x2"])
    with torch.no_grad():
        y16 = mm(x1, x2)
        mm.set_quant_state(False, True)
        a, b = mm.quant_x1(x1), mm.quant_x2(x2)
        y = mm(a, b)
    np.testing.assert_allclose(n(y16), g["y"], rtol=1e-5, atol=1e-5)
    ra, *_ = O.quantize(g["x1"], 8, None)
    rb, *_ = O.quantize(g["x2"], 8, None)
    assert np.array_equal(n(a).view(np.uint32), ra.view(np.uint32))
    assert np.array_equal(n(b).view(np.uint32), rb.view(np.uint32))
    np.testing.assert_allclose(n(y), g["y_a8"], rtol=1e-5, atol=1e-5)
