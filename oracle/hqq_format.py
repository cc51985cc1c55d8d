"""HQQ (hqq, unpinned: reference environment.yml:42) weight format, restated — TEST INFRASTRUCTURE
ONLY (tests/ import it as the checker; the product never does).

hqq is not vendored under /root/reference and is not installed here, so this restates its
published ``hqq.core.quantize.Quantizer`` / ``hqq.core.bitpack.BitPack`` behaviour as the reference
calls it (``quantizehqq.py:40-49``: ``BaseQuantizeConfig(nbits, group_size)`` then
``LlamaHQQ.quantize_model``; ``models/LMClass.py:32-34``: ``AutoHQQHFModel.from_quantized``):
PARITY UNPINNED against the real library — no reference test, golden file or checkpoint pins it.
The build's converter (``quant/hqq.py``) is pinned only against this restatement.

Quantize (``Quantizer.quantize``, channel_wise, no proximal optimisation), W [N, K] float32:
  axis = 1: W.reshape(-1, g) (g consecutive in-features of one row per group);
  axis = 0: W.reshape(g, -1) (groups strided along the flat tensor — rejected by the converter);
  max_v = 2^b - 1;  scale = clamp(max_v / (max - min), max=2e4);  zero = -min * scale
  (rounded when round_zero);  W_q = clamp(round(W * scale + zero), 0, max_v);
  meta scale = 1 / scale; scale and zero are then held in the compute dtype (fp16).
Bit packing along dim 0 of W_q [rows, cols] (rows = N*K/g groups for axis = 1):
  8bit_u8: as is;  4bit_u8: step = rows/2, (W[:step] << 4) | W[step:];
  2bit_u8: step = rows/4, W[:s] << 6 | W[s:2s] << 4 | W[2s:3s] << 2 | W[3s:];
  3bit_32: rows padded to 10*ceil(rows/10), step = rows/10, int32
           W[0:s] << 27 | W[s:2s] << 24 | ... | W[9s:10s] << 0.
Dequantize (``Quantizer.dequantize``): unpack to the compute dtype (3-bit: keep the first
N*K/g rows), W_r = ((W_q - zero) * scale).reshape(N, K) — two fp16 ops, each rounded once.
"""
from __future__ import annotations

import numpy as np

PACKING = {8: "8bit_u8", 4: "4bit_u8", 3: "3bit_32", 2: "2bit_u8"}


def quantize(w, nbits, group_size, axis=1, round_zero=False):
    """RTN Quantizer.quantize (optimize=False) of w [N, K] -> (W_q uint8 [rows, cols], scale fp16
    [rows or cols], zero fp16, shape).  For axis = 1 the stats are per row of [N*K/g, g]."""
    W = np.asarray(w, dtype=np.float32)
    shape = W.shape
    W = W.reshape(-1, group_size) if axis == 1 else W.reshape(group_size, -1)
    mn = W.min(axis=axis, keepdims=True)
    mx = W.max(axis=axis, keepdims=True)
    max_v = float(2 ** nbits - 1)
    with np.errstate(divide="ignore"):
        scale = np.minimum(np.float32(max_v) / (mx - mn), np.float32(2e4)).astype(np.float32)
    zero = (-mn * scale).astype(np.float32)
    if round_zero:
        zero = np.round(zero).astype(np.float32)
    W_q = np.clip(np.round(W * scale + zero), 0, max_v).astype(np.uint8)
    inv = (np.float32(1.0) / scale).astype(np.float16)
    return W_q, inv, zero.astype(np.float16), shape


def pack(W_q, nbits):
    """BitPack.pack_<packing>(W_q) along dim 0."""
    W = np.asarray(W_q)
    if nbits == 8:
        return W.astype(np.uint8)
    if nbits == 4:
        W = W.astype(np.uint8)
        s = len(W) // 2
        return ((W[:s] << 4) | W[s:]).astype(np.uint8)
    if nbits == 2:
        W = W.astype(np.uint8)
        s = len(W) // 4
        return ((W[:s] << 6) | (W[s:2 * s] << 4) | (W[2 * s:3 * s] << 2) | W[3 * s:]).astype(np.uint8)
    if nbits == 3:
        rows = int(10 * np.ceil(W.shape[0] / 10.0))
        P = np.zeros((rows, W.shape[1]), dtype=np.int64)
        P[: len(W)] = W
        s = rows // 10
        out = np.zeros((s, W.shape[1]), dtype=np.int64)
        for i in range(10):
            out |= P[i * s:(i + 1) * s] << (27 - 3 * i)
        return out.astype(np.uint32).view(np.int32)
    raise ValueError(f"unsupported nbits {nbits}")


def unpack(packed, nbits):
    """BitPack.unpack_<packing> (uint8 codes, all packed rows)."""
    P = np.asarray(packed)
    if nbits == 8:
        return P.astype(np.uint8)
    if nbits == 4:
        return np.concatenate([(P & 0xF0) >> 4, P & 0x0F]).astype(np.uint8)
    if nbits == 2:
        return np.concatenate([(P & 0xC0) >> 6, (P & 0x30) >> 4, (P & 0x0C) >> 2,
                               P & 0x03]).astype(np.uint8)
    if nbits == 3:
        U = P.view(np.uint32).astype(np.int64)
        return np.concatenate([(U >> (27 - 3 * i)) & 7 for i in range(10)]).astype(np.uint8)
    raise ValueError(f"unsupported nbits {nbits}")


def dequantize(packed, scale, zero, nbits, group_size, shape, axis=1):
    """Quantizer.dequantize in fp16: ((W_q - zero) * scale).reshape(shape)."""
    W = unpack(packed, nbits)
    if nbits == 3:
        W = W[: group_size if axis == 0 else shape[0] * shape[1] // group_size]
    Wf = W.astype(np.float16)
    z = np.asarray(zero, dtype=np.float16).reshape(-1, 1) if axis == 1 else \
        np.asarray(zero, dtype=np.float16).reshape(1, -1)
    s = np.asarray(scale, dtype=np.float16).reshape(z.shape)
    d = (Wf.astype(np.float32) - z.astype(np.float32)).astype(np.float16)
    return (d.astype(np.float32) * s.astype(np.float32)).astype(np.float16).reshape(shape)
