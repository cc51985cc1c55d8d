"""AutoGPTQ checkpoint tensors -> the gfx950 tiled layout.

The reference consumes GPTQ weights through AutoGPTQ (``autogptq.py`` saves them with
transformers' GPTQConfig; ``quant/omniquant.py:326-334`` packs with auto_gptq's ``QuantLinear``;
auto-gptq==0.7.1 per environment.yml:22).  Per linear a checkpoint holds

  qweight int32 [K*b/32, N]   codes packed along K (in_features); b = 3 is a 96-bit little-endian
                              bit stream per 32 codes (code i at bits 3i .. 3i+2)
  qzeros  int32 [K/g, N*b/32] (zero - 1) packed along N the same way
  scales  fp16  [K/g, N]
  g_idx   int32 [K]           group of input column k (k // g without act-order)
  bias    fp16  [N]           optional

and dequantizes W[n, k] = scales[g, n] * (q[k, n] - zeros[g, n]) in fp16 — the same identity the
qlin kernels use, so the converted layer reproduces AutoGPTQ's W bit for bit.

Conversion: unpack codes / zeros with integer tensor ops (any device), form W_dq in fp16 on the
GPU, and pack it with the library's own fake-quant packer (``qlin_fake_quant``), which recovers the
integer codes exactly (|W_dq / s - (u - z)| <= 2^-11 |u - z| < 1/2).  Act-order checkpoints
(``desc_act``: g_idx not equal to k // g) are rejected: the tiled layout needs contiguous groups.
"""
from __future__ import annotations

import torch

from . import qlin


def _unpack_rows(words: torch.Tensor, bits: int, n_codes: int) -> torch.Tensor:
    """int32 [R, C] -> int64 codes [n_codes, C], packed along dim 0 (AutoGPTQ order)."""
    w = words.to(torch.int64) & 0xFFFFFFFF
    mask = (1 << bits) - 1
    if bits in (2, 4, 8):
        per = 32 // bits
        shifts = torch.arange(per, device=w.device, dtype=torch.int64) * bits
        codes = (w[:, None, :] >> shifts[None, :, None]) & mask  # [R, per, C]
        return codes.reshape(-1, w.shape[1])[:n_codes]
    if bits != 3:
        raise ValueError(f"unsupported bits {bits}")
    # three words = one 96-bit little-endian stream of 32 codes
    R, C = w.shape
    if R % 3:
        raise ValueError("3-bit qweight rows must be a multiple of 3")
    t = w.reshape(R // 3, 3, C)
    i = torch.arange(32, device=w.device, dtype=torch.int64)
    bit = 3 * i
    word, sh = bit // 32, bit % 32
    lo = torch.gather(t, 1, word[None, :, None].expand(R // 3, 32, C)) >> sh[None, :, None]
    nxt = torch.clamp(word + 1, max=2)
    hi = torch.gather(t, 1, nxt[None, :, None].expand(R // 3, 32, C)) << (32 - sh)[None, :, None]
    spill = (sh > 29)[None, :, None]
    codes = (lo | torch.where(spill, hi, torch.zeros_like(hi))) & mask
    return codes.reshape(-1, C)[:n_codes]


def unpack_qweight(qweight: torch.Tensor, bits: int) -> torch.Tensor:
    """AutoGPTQ qweight [K*b/32, N] -> codes int64 [K, N]."""
    K = qweight.shape[0] * 32 // bits
    return _unpack_rows(qweight, bits, K)


def unpack_qzeros(qzeros: torch.Tensor, bits: int, N: int) -> torch.Tensor:
    """AutoGPTQ qzeros [G, N*b/32] -> zero points int64 [G, N] (the stored value + 1)."""
    z = _unpack_rows(qzeros.t().contiguous(), bits, N).t()
    return z + 1


def check_g_idx(g_idx, K: int, group: int):
    if g_idx is None:
        return
    expect = torch.arange(K, device=g_idx.device, dtype=torch.int64) // group
    if not torch.equal(g_idx.to(torch.int64), expect):
        raise NotImplementedError(
            "act-order (desc_act) GPTQ checkpoints are not supported: the gfx950 layout needs "
            "contiguous groups (g_idx == k // group)")


def gptq_dequant(qweight, qzeros, scales, g_idx, bits: int) -> torch.Tensor:
    """W [N, K] fp16 exactly as AutoGPTQ dequantizes it (fp16: (q - z) exact, times scale)."""
    q = unpack_qweight(qweight, bits)  # [K, N]
    K, N = q.shape
    G = scales.shape[0]
    group = K // G
    gi = (torch.arange(K, device=q.device) // group) if g_idx is None else g_idx.to(torch.int64)
    z = unpack_qzeros(qzeros, bits, N)  # [G, N]
    d = (q - z[gi]).to(torch.float16)
    return (d * scales.to(torch.float16)[gi]).t().contiguous()


@torch.no_grad()
def gptq_to_qlin(qweight, qzeros, scales, g_idx=None, bits: int = 4):
    """Convert one AutoGPTQ linear to the tiled layout.  Returns dict(qweight, qsz, flags, N, K,
    bits, group) on the device of ``qweight`` (a gfx950 device: the packer is a HIP kernel)."""
    if bits not in (2, 3, 4, 8):
        raise ValueError(f"unsupported bits {bits}")
    K = qweight.shape[0] * 32 // bits
    N = qweight.shape[1]
    G = scales.shape[0]
    if G == 0 or K % G:
        raise ValueError(f"{G} groups do not divide K = {K}")
    group = K // G
    check_g_idx(g_idx, K, group)
    w_dq = gptq_dequant(qweight, qzeros, scales, None, bits)  # [N, K] fp16
    z = unpack_qzeros(qzeros, bits, N)  # [G, N]
    s_flat = scales.to(torch.float16).t().contiguous().reshape(-1)  # [N * G], row n then group
    z_flat = z.t().contiguous().reshape(-1).to(torch.float16)
    out = qlin.fake_quant(w_dq, s_flat, z_flat, bits, group, 0, want_xdq=False, pack=True)
    return dict(qweight=out["qweight"], qsz=out["qsz"], flags=out["flags"], N=N, K=K, bits=bits,
                group=group)


def packed_quant_linear(tensors: dict, prefix: str, bits: int, device="cuda"):
    """A packed QuantLinear from the AutoGPTQ tensors ``{prefix}.qweight/.qzeros/.scales/.g_idx
    [/.bias]`` (e.g. a safetensors state dict)."""
    from .int_linear import QuantLinear
    t = {k[len(prefix) + 1:]: v for k, v in tensors.items() if k.startswith(prefix + ".")}
    dev = torch.device(device)
    conv = gptq_to_qlin(t["qweight"].to(dev), t["qzeros"].to(dev), t["scales"].to(dev),
                        t.get("g_idx").to(dev) if t.get("g_idx") is not None else None, bits)
    bias = t.get("bias")
    lin = torch.nn.Linear(conv["K"], conv["N"], bias=bias is not None, device="meta")
    ql = QuantLinear(lin, dict(n_bits=bits, group_size=conv["group"],
                               dynamic_method="per_channel", per_channel_axes=[0]), {},
                     disable_input_quant=True)
    if bias is not None:
        ql.bias = bias.to(dev, torch.float16)
    ql._install(conv, bits, conv["group"], keep_weight=False)
    return ql
