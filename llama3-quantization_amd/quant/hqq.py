"""HQQ-quantized linears -> the gfx950 tiled layout (BASELINE configs[3]).

The reference quantizes with hqq (``quantizehqq.py:40-49``: ``BaseQuantizeConfig(nbits,
group_size)`` + ``LlamaHQQ.quantize_model``) and evaluates the saved model through
``AutoHQQHFModel.from_quantized`` (``models/LMClass.py:32-34``); hqq is unpinned
(``environment.yml:42``).  An ``HQQLinear`` holds

  W_q   codes packed along dim 0 of the [N*K/g, g] group view (axis = 1): 4bit_u8 / 2bit_u8 uint8
        (2 / 4 group rows per byte row, high bits first), 3bit_32 int32 (10 group rows per word
        row, rows padded to a multiple of 10), 8bit_u8 as is;
  meta  {nbits, group_size, shape = (N, K), axis, packing, scale, zero, ...}: fp16 scale (already
        inverted) and fp16 zero of every group, [N*K/g, 1];

and dequantizes W = ((W_q - zero) * scale).reshape(N, K) in fp16.  The zero points are NOT
integral, so the packed matrix carries them as fp16 (layout flag ``QLIN_FLOAT_ZERO``): every
kernel forms RN16(RN16(u - zero) * scale), bit-identical to hqq's dequantize.

Conversion: unpack the bit-packed rows with integer tensor ops on the device, pack the codes into
the tiled layout with ``qlin_pack_codes`` and the (scale, zero) pairs into ``qsz``.  Unsupported
(raised, never approximated): axis = 0 (groups strided along the output rows — the tiled layout
needs groups of consecutive in-features), meta-quantized scale / zero (quant_scale, quant_zero),
group sizes that are not a multiple of 32.  Checker: ``oracle/hqq_format.py`` (parity unpinned:
hqq is absent here)."""
from __future__ import annotations

import torch

from . import qlin

PACKING = {8: "8bit_u8", 4: "4bit_u8", 3: "3bit_32", 2: "2bit_u8"}


def unpack(W_q: torch.Tensor, nbits: int) -> torch.Tensor:
    """hqq BitPack.unpack_<packing>: all packed rows -> uint8 codes (3-bit rows still padded)."""
    if nbits == 8:
        return W_q.to(torch.uint8)
    if nbits == 4:
        P = W_q.view(torch.uint8) if W_q.dtype != torch.uint8 else W_q
        return torch.cat([(P >> 4) & 0xF, P & 0xF], dim=0)
    if nbits == 2:
        P = W_q.view(torch.uint8) if W_q.dtype != torch.uint8 else W_q
        return torch.cat([(P >> 6) & 3, (P >> 4) & 3, (P >> 2) & 3, P & 3], dim=0)
    if nbits == 3:
        P = W_q.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        return torch.cat([(P >> (27 - 3 * i)) & 7 for i in range(10)], dim=0).to(torch.uint8)
    raise ValueError(f"unsupported nbits {nbits}")


def _meta_tensor(meta, key, rows, device):
    t = meta.get(key)
    if t is None:
        raise NotImplementedError(
            f"HQQ meta without a plain '{key}' tensor (meta-quantized scale / zero, quant_scale / "
            "quant_zero) is not supported")
    t = torch.as_tensor(t).to(device=device, dtype=torch.float16)
    if t.numel() != rows:
        raise ValueError(f"meta['{key}'] has {t.numel()} values, expected {rows} (one per group)")
    return t.reshape(-1)


@torch.no_grad()
def hqq_to_qlin(W_q: torch.Tensor, meta: dict) -> dict:
    """Convert one HQQLinear (``W_q``, ``meta``) to the tiled layout on ``W_q``'s device (a gfx950
    device: the packer is a HIP kernel).  Returns dict(qweight, qsz, flags, N, K, bits, group)."""
    nbits = int(meta["nbits"])
    if nbits not in PACKING:
        raise ValueError(f"unsupported nbits {nbits} (2, 3, 4, 8)")
    if meta.get("packing", PACKING[nbits]) != PACKING[nbits]:
        raise ValueError(f"unexpected packing {meta.get('packing')} for {nbits}-bit")
    if meta.get("group_size") is None:
        raise NotImplementedError("HQQ without group_size (one group per tensor) is not supported")
    g = int(meta["group_size"])
    N, K = (int(v) for v in meta["shape"])
    if int(meta.get("axis", 0)) != 1:
        raise NotImplementedError(
            "HQQ axis=0 groups run along the output rows; the tiled layout needs axis=1 groups")
    if g % 32 or K % g:
        raise ValueError(f"group {g} must be a multiple of 32 dividing in_features {K}")
    if meta.get("view_as_float"):
        W_q = W_q.view(torch.int32 if nbits == 3 else torch.uint8)
    rows = N * K // g
    codes = unpack(W_q, nbits)
    if codes.shape[0] < rows or codes.shape[1] != g:
        raise ValueError(f"W_q unpacks to {tuple(codes.shape)}, expected [{rows}, {g}]")
    codes = codes[:rows].reshape(N, K).contiguous()
    scale = _meta_tensor(meta, "scale", rows, W_q.device)
    zero = _meta_tensor(meta, "zero", rows, W_q.device)
    qweight = qlin.pack_codes(codes, nbits)
    qsz = qlin.join_sz_float(scale.view(N, K // g), zero.view(N, K // g))
    return dict(qweight=qweight, qsz=qsz, flags=qlin.FLOAT_ZERO, N=N, K=K, bits=nbits, group=g)


def packed_quant_linear(W_q: torch.Tensor, meta: dict, bias=None, device="cuda"):
    """A packed QuantLinear (the reference module API) from one HQQLinear's ``W_q`` / ``meta``."""
    from .int_linear import QuantLinear
    dev = torch.device(device)
    conv = hqq_to_qlin(W_q.to(dev), {k: (v.to(dev) if torch.is_tensor(v) else v)
                                     for k, v in meta.items()})
    lin = torch.nn.Linear(conv["K"], conv["N"], bias=bias is not None, device="meta")
    ql = QuantLinear(lin, dict(n_bits=conv["bits"], group_size=conv["group"],
                               dynamic_method="per_channel", per_channel_axes=[0]), {},
                     disable_input_quant=True)
    if bias is not None:
        ql.bias = bias.to(dev, torch.float16)
    ql._install(conv, conv["bits"], conv["group"], keep_weight=False)
    return ql
