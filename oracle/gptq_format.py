"""AutoGPTQ (auto-gptq==0.7.1, environment.yml:22) checkpoint tensor format, restated — TEST
INFRASTRUCTURE ONLY (tests/ import it as the checker; the product never does).

auto-gptq is not vendored under /root/reference and is not installed here, so this is a
restatement of its published packing (``qlinear_cuda`` / ``qlinear_triton`` ``QuantLinear.pack``,
the call the reference makes at quant/omniquant.py:326-334): PARITY UNPINNED against the real
library — no reference test, golden file or checkpoint pins it.

Format (per linear, in_features K, out_features N, group g, bits b):
  qweight  int32 [K * b / 32, N]: codes packed along K, 32/b per word, code k of a word at bit
           b * (k % (32/b)); b = 3 packs 32 codes into 3 words, crossing word boundaries
           (10 + 1 split + 10 + 1 split + 10 codes).
  qzeros   int32 [K / g, N * b / 32]: (zero - 1) packed along N the same way (v1 convention;
           dequant adds the 1 back).
  scales   fp16 [K / g, N];  g_idx int32 [K] (= k // g without act-order).
  W[n, k] = scales[g_idx[k], n] * (q[k, n] - zeros[g_idx[k], n])   (fp16 arithmetic)."""
from __future__ import annotations

import numpy as np


def _pack_rows(v, bits):
    """v: uint32 [R, C] codes -> uint32 [R * bits / 32, C], packing along axis 0."""
    R, C = v.shape
    v = v.astype(np.uint64)
    out = np.zeros((R * bits // 32, C), dtype=np.uint64)
    if bits in (2, 4, 8):
        per = 32 // bits
        for r in range(out.shape[0]):
            for j in range(per):
                out[r] |= v[r * per + j] << np.uint64(bits * j)
        return (out & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    assert bits == 3
    i = 0
    row = 0
    while row < out.shape[0]:
        for j in range(i, i + 10):
            out[row] |= v[j] << np.uint64(3 * (j - i))
        i += 10
        out[row] |= v[i] << np.uint64(30)
        row += 1
        out[row] |= (v[i] >> np.uint64(2)) & np.uint64(1)
        i += 1
        for j in range(i, i + 10):
            out[row] |= v[j] << np.uint64(3 * (j - i) + 1)
        i += 10
        out[row] |= v[i] << np.uint64(31)
        row += 1
        out[row] |= (v[i] >> np.uint64(1)) & np.uint64(3)
        i += 1
        for j in range(i, i + 10):
            out[row] |= v[j] << np.uint64(3 * (j - i) + 2)
        i += 10
        row += 1
    return (out & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def pack_qweight(q_kn, bits):
    """q_kn: int codes [K, N] (in, out) -> qweight uint32 [K*bits/32, N]."""
    return _pack_rows(np.asarray(q_kn, dtype=np.uint32), bits)


def pack_qzeros(z_gn, bits):
    """z_gn: integer zero points [G, N] -> qzeros uint32 [G, N*bits/32] holding (z - 1)."""
    zm1 = (np.asarray(z_gn, dtype=np.int64) - 1).astype(np.uint32) & np.uint32((1 << bits) - 1)
    return _pack_rows(zm1.T.copy(), bits).T.copy()


def dequant(q_kn, z_gn, s_gn, g_idx):
    """W [N, K] fp16 = s * (q - z) in fp16 arithmetic (q - z exact, one rounding)."""
    q = np.asarray(q_kn, dtype=np.int64)          # [K, N]
    z = np.asarray(z_gn, dtype=np.int64)[g_idx]   # [K, N]
    s = np.asarray(s_gn, dtype=np.float16)[g_idx]  # [K, N]
    d = (q - z).astype(np.float16)
    return (d.astype(np.float32) * s.astype(np.float32)).astype(np.float16).T.copy()
