"""CPU restatement of the reference quantized-linear arithmetic — TEST INFRASTRUCTURE ONLY.

This module is the parity oracle.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it, and only as the checker.  The product path
(``llama3-quantization_amd/``) never imports, calls or links anything under ``oracle/``.

Parity pinning: every function here is checked bit-for-bit against golden vectors produced by
running the reference's own ``quant/quantizer.py`` / ``quant/int_linear.py`` in the survey
container (``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``).

Reference citations are ``file:line`` under the reference repo (SilviaUvA/LLaMA3-Quantization).

Dtype semantics.  The reference computes in the weight dtype (fp16 for LLaMA3: the model is
loaded with ``torch_dtype=float16`` and ``omniquant.py:296`` calls ``.half()``).  PyTorch evaluates a
binary fp16 op as "compute in float32, round once to fp16" (verified: 0 mismatches over 1e6 random
divisions / multiplications).  ``_op`` restates exactly that: inputs are upcast to float32, the
op is evaluated in IEEE float32 and the result is rounded (nearest-even) to the compute dtype.

Canonical packed layout (the build's own format, see DESIGN.md §3 and ``pack_qweight``):
  qweight  uint32 [ceil(N/16), ceil(K/128), 64, bits]: 16-row x 128-k tiles of 64 lane pieces,
           lane l = n + 16q holding codes (s, j) of row n at k = 32s + 8q + j (s, j < 4, 8) — the
           B operand of v_mfma_f32_16x16x32_f16 k-step s; inside a piece the codes sit so that one
           v_and_or_b32 with an fp16 exponent "magic" yields the pair (off + u_j, off + u_j+1).
  qsz      uint32 [ceil(N/16), K/g, 16]: per (16-row tile, group, row) the fp16 scale (bits 0-15,
           == reference ``scales.view(N, -1)``, omniquant.py:322-325) and the int16 zero point
           (bits 16-31, == ``zeros.view(N, -1)``); one coalesced 64-B load per tile and group.
"""
from __future__ import annotations

import numpy as np

CLIPMIN = 1e-5  # quant/quantizer.py:10

F16 = np.float16
F32 = np.float32


def _op(fn, dt, *args):
    """Evaluate ``fn`` in float32 and round once to ``dt`` (torch CPU reduced-float semantics)."""
    with np.errstate(all="ignore"):
        r = fn(*[np.asarray(a, dtype=F32) for a in args])
        return np.asarray(r, dtype=F32).astype(dt)


def sigmoid(f, dt):
    """``nn.Sigmoid`` on a factor tensor of dtype ``dt`` (quantizer.py:80, :144-145)."""
    # torch evaluates sigmoid as 1 / (1 + exp(-x)) in float32 (its expf is ~1 ulp; this restates it
    # with a correctly rounded expf, which agrees on every golden factor).
    f32 = np.asarray(f, dtype=F32)
    with np.errstate(all="ignore"):
        e = np.exp(-f32.astype(np.float64)).astype(F32)
        r = (F32(1.0) / (F32(1.0) + e)).astype(F32)
    return r.astype(dt)


def qrange(n_bits: int, disable_zero_point: bool):
    """quantizer.py:46-51 / :85-92."""
    if disable_zero_point:
        return -(2 ** (n_bits - 1)), 2 ** (n_bits - 1) - 1
    return 0, 2 ** n_bits - 1


def _pad(x, deficiency):
    if deficiency > 0:
        x = np.concatenate([x, np.zeros((x.shape[0], deficiency), dtype=x.dtype)], axis=1)
    return x


def calibrate(x, n_bits, group_size=None, symmetric=False, disable_zero_point=False,
              lwc_up=None, lwc_low=None, deficiency=0):
    """``per_token_dynamic_calibration`` (quantizer.py:132-159).

    ``x`` is 2-D (or N-D for per-token with ``group_size=None``: reduction over the last dim).
    ``lwc_up`` / ``lwc_low`` are the *raw* LWC factors (dtype decides promotion, as in torch).
    Returns ``(scale, round_zero_point)`` shaped like the reference's ``[rows, 1]`` (or ``x[...,:1]``).
    """
    dt = x.dtype
    if lwc_up is not None:
        dt = np.result_type(x.dtype, np.asarray(lwc_up).dtype)
    if group_size:
        x = _pad(x, deficiency).reshape(-1, group_size)
    xmin = x.min(axis=-1, keepdims=True)
    xmax = x.max(axis=-1, keepdims=True)
    if lwc_up is not None:
        fdt = np.asarray(lwc_up).dtype
        xmax = _op(np.multiply, dt, sigmoid(lwc_up, fdt), xmax)
        xmin = _op(np.multiply, dt, sigmoid(lwc_low, fdt), xmin)
    xmin = np.asarray(xmin, dtype=dt)
    xmax = np.asarray(xmax, dtype=dt)
    if symmetric:
        abs_max = np.maximum(np.abs(xmax), np.abs(xmin))
        scale = _op(np.divide, dt, abs_max, float(2 ** (n_bits - 1) - 1))
        scale = _op(lambda s: np.clip(s, F32(CLIPMIN), F32(1e4)), dt, scale)
        zero_point = np.full_like(scale, 2 ** (n_bits - 1) - 1)
    else:
        rng = _op(np.subtract, dt, xmax, xmin)
        scale = _op(np.divide, dt, rng, float(2 ** n_bits - 1))
        scale = _op(lambda s: np.clip(s, F32(CLIPMIN), F32(1e4)), dt, scale)
        zero_point = _op(np.divide, dt, -xmin, scale)
    if disable_zero_point:
        rzp = None
    else:
        rzp = np.rint(_op(lambda z: np.clip(z, F32(-1e4), F32(1e4)), dt, zero_point)).astype(dt)
    return scale.astype(dt), rzp


def round_ste_fwd(v):
    """Forward value of ``round_ste`` (quantizer.py:15-19): ``(round(v) - v) + v`` in v's dtype.

    Equal to ``round(v)`` for finite v; NaN where v is infinite (inf - inf)."""
    dt = v.dtype
    r = np.rint(v)
    return _op(np.add, dt, _op(np.subtract, dt, r, v), v)


def fake_quant(x, scale, round_zero_point, n_bits, group_size=None, disable_zero_point=False,
               deficiency=0, return_int=False):
    """``UniformAffineQuantizer.fake_quant`` (quantizer.py:94-115)."""
    qmin, qmax = qrange(n_bits, disable_zero_point)
    dt = np.result_type(x.dtype, scale.dtype)
    x = _pad(x, deficiency)
    if group_size:
        dim1, dim2 = x.shape
        x = x.reshape(-1, group_size)
    x_int = round_ste_fwd(_op(np.divide, dt, x, scale))
    if round_zero_point is not None:
        x_int = _op(np.add, dt, x_int, round_zero_point)
    x_int = _op(lambda t: np.clip(t, F32(qmin), F32(qmax)), dt, x_int)  # NaN propagates
    x_dq = x_int
    if round_zero_point is not None:
        x_dq = _op(np.subtract, dt, x_dq, round_zero_point)
    x_dq = _op(np.multiply, dt, x_dq, scale)
    if group_size:
        x_dq = x_dq.reshape(dim1, dim2)
        x_int = x_int.reshape(dim1, dim2)
    if deficiency > 0:
        x_dq = x_dq[:, :-deficiency]
        x_int = x_int[:, :-deficiency]
    if return_int:
        return x_dq, x_int
    return x_dq


def quantize(w, n_bits, group_size=None, symmetric=False, disable_zero_point=False,
             lwc_up=None, lwc_low=None, deficiency=0):
    """``UniformAffineQuantizer.forward`` for weights (quantizer.py:118-130).

    Returns ``(w_dq, scale, round_zero_point, x_int)``."""
    if n_bits >= 16:
        return w, None, None, None
    scale, rzp = calibrate(w, n_bits, group_size, symmetric, disable_zero_point,
                           lwc_up, lwc_low, deficiency)
    w_dq, x_int = fake_quant(w, scale, rzp, n_bits, group_size, disable_zero_point,
                             deficiency, return_int=True)
    return w_dq, scale, rzp, x_int


# ----------------------------------------------------------------------------------------------
# canonical packed layout (build-defined; consumed by the HIP kernels) — "qlin tiled" layout
# ----------------------------------------------------------------------------------------------
TILE_N = 16    # rows per tile (the 16 columns of a v_mfma_f32_16x16x32_f16 B operand)
TILE_K = 128   # k per tile (4 MFMA k-steps of 32)
RHO3 = (0, 1, 8, 9)  # int3 high-bit word rotation per k-step


def tiled_shape(N, K, bits):
    return (-(-N // TILE_N), -(-K // TILE_K), 64, bits)


def _code_bit(bits, s, j):
    """(word, bit) of code (step s, j) inside a lane piece for bits in {2,4,8}."""
    p, h = j >> 1, j & 1
    if bits == 4:
        return s, 16 * h + 4 * p
    if bits == 8:
        jj = j & 3
        return 2 * s + (j >> 2), 16 * h + 8 * (jj >> 1)
    if bits == 2:
        return s >> 1, 16 * h + 8 * (s & 1) + 2 * p
    raise ValueError(bits)


def pack_qweight(u, bits):
    """Pack unsigned codes ``u`` [N, K] (0 <= u < 2**bits, K % 32 == 0) into the tiled layout.

    Tile (nt, kt) = rows 16nt..16nt+15 x k 128kt..128kt+127, stored as 64 lane pieces of ``bits``
    uint32.  Lane l = n + 16q (n = l & 15, q = l >> 4) holds the 32 codes (s, j), s = 0..3,
    j = 0..7, of row 16nt + n at k = 128kt + 32s + 8q + j — exactly the B operand lane l feeds to
    MFMA k-step s.  Rows / k beyond (N, K) are zero codes."""
    u = np.asarray(u, dtype=np.uint32)
    N, K = u.shape
    assert K % 32 == 0, "K must be a multiple of 32"
    Nt, Kt = -(-N // TILE_N), -(-K // TILE_K)
    up = np.zeros((Nt * TILE_N, Kt * TILE_K), dtype=np.uint32)
    up[:N, :K] = u
    # c[nt, kt, n, s, q, j]
    c = up.reshape(Nt, TILE_N, Kt, 4, 4, 8).transpose(0, 2, 1, 3, 4, 5)
    out = np.zeros((Nt, Kt, 4, TILE_N, bits), dtype=np.uint32)  # [nt, kt, q, n, word]
    if bits in (2, 4, 8):
        for s in range(4):
            for j in range(8):
                w, b = _code_bit(bits, s, j)
                out[:, :, :, :, w] |= (c[:, :, :, s, :, j].transpose(0, 1, 3, 2) << np.uint32(b))
    elif bits == 3:
        lo = c & np.uint32(3)
        for s in range(4):
            for j in range(8):
                w, b = _code_bit(2, s, j)
                out[:, :, :, :, w] |= (lo[:, :, :, s, :, j].transpose(0, 1, 3, 2) << np.uint32(b))
                p, h = j >> 1, j & 1
                hb = (16 * h + 2 * p + 2 + RHO3[s]) % 32
                hi = (c[:, :, :, s, :, j] >> np.uint32(2)) & np.uint32(1)
                out[:, :, :, :, 2] |= (hi.transpose(0, 1, 3, 2) << np.uint32(hb))
    else:
        raise ValueError(f"bits={bits} not supported")
    return out.reshape(Nt, Kt, 64, bits)


def unpack_qweight(qw, bits, N, K):
    """Inverse of ``pack_qweight``: codes [N, K]."""
    qw = np.asarray(qw, dtype=np.uint32)
    Nt, Kt = qw.shape[0], qw.shape[1]
    words = qw.reshape(Nt, Kt, 4, TILE_N, bits)  # [nt, kt, q, n, word]
    c = np.zeros((Nt, Kt, TILE_N, 4, 4, 8), dtype=np.uint32)  # [nt, kt, n, s, q, j]
    for s in range(4):
        for j in range(8):
            if bits in (2, 4, 8):
                w, b = _code_bit(bits, s, j)
                v = (words[..., w] >> np.uint32(b)) & np.uint32(2 ** bits - 1)
            else:
                w, b = _code_bit(2, s, j)
                p, h = j >> 1, j & 1
                hb = (16 * h + 2 * p + 2 + RHO3[s]) % 32
                v = ((words[..., w] >> np.uint32(b)) & np.uint32(3)) | \
                    (((words[..., 2] >> np.uint32(hb)) & np.uint32(1)) << np.uint32(2))
            c[:, :, :, s, :, j] = v.transpose(0, 1, 3, 2)
    full = c.transpose(0, 2, 1, 3, 4, 5).reshape(Nt * TILE_N, Kt * TILE_K)
    return full[:N, :K]


WIDE_ZERO = 1024  # |zp| above this needs the kernels' fp32 (u - zp) path (QLIN_WIDE_ZERO)


def pack_sz(scales, zeros):
    """Packed (scale, zero) words: uint32 [ceil(N/16), G, 16]; word (nt, g, n) holds the fp16 bits
    of scales[16nt + n, g] in bits 0..15 and the int16 zero point in bits 16..31 (rows >= N: 0)."""
    sc = np.asarray(scales, dtype=F16).reshape(np.asarray(scales).shape[0], -1)
    N, G = sc.shape
    z = np.asarray(zeros).reshape(N, G).astype(np.int64)
    assert z.min(initial=0) >= -32768 and z.max(initial=0) <= 32767
    Nt = -(-N // TILE_N)
    w = np.zeros((Nt * TILE_N, G), dtype=np.uint32)
    w[:N] = sc.view(np.uint16).astype(np.uint32) | ((z.astype(np.int16).view(np.uint16).astype(np.uint32)) << np.uint32(16))
    return w.reshape(Nt, TILE_N, G).transpose(0, 2, 1).copy()


def unpack_sz(qsz, N):
    """Inverse of ``pack_sz``: (scales fp16 [N, G], zeros int32 [N, G])."""
    qsz = np.asarray(qsz, dtype=np.uint32)
    Nt, G, _ = qsz.shape
    w = qsz.transpose(0, 2, 1).reshape(Nt * TILE_N, G)[:N]
    sc = (w & np.uint32(0xFFFF)).astype(np.uint16).view(F16)
    z = (w >> np.uint32(16)).astype(np.uint16).view(np.int16).astype(np.int32)
    return sc, z


def pack_from_quant(x_int, scale, rzp, n_bits, N, K, group_size, disable_zero_point=False):
    """Canonical packed tensors (qweight, qsz, wide) from the quantizer's integer codes and fp16
    (scale, zp)."""
    g = group_size or K
    if disable_zero_point:
        off = 2 ** (n_bits - 1)
        u = np.asarray(x_int, dtype=np.float32) + off
        zeros = np.full((N, K // g), off, dtype=np.int32)
    else:
        u = np.asarray(x_int, dtype=np.float32)
        zeros = np.asarray(rzp, dtype=np.float32).reshape(N, K // g).astype(np.int32)
    qweight = pack_qweight(u.astype(np.uint32), n_bits)
    scales = np.asarray(scale, dtype=F16).reshape(N, K // g)
    wide = bool(zeros.size and np.abs(zeros).max() > WIDE_ZERO)
    return qweight, pack_sz(scales, zeros), wide


def pack_from_dequant(w_dq, scales, zeros, n_bits, group_size, disable_zero_point=False):
    """Restatement of the real-quant packer input contract (omniquant.py:315-335): recover integer
    codes from ``W_dq`` and the registered fp16 (scales, zeros) with the quantizer's own fp16
    arithmetic, then pack.  Returns ``(qweight, qsz, wide)`` in the canonical layout."""
    N, K = w_dq.shape
    g = group_size or K
    qmin, qmax = qrange(n_bits, disable_zero_point)
    s = np.asarray(scales, dtype=F16).reshape(-1, 1)
    x = w_dq.reshape(-1, g)
    x_int = round_ste_fwd(_op(np.divide, F16, x, s))
    if not disable_zero_point:
        z = np.asarray(zeros, dtype=F16).reshape(-1, 1)
        x_int = _op(np.add, F16, x_int, z)
    x_int = np.clip(x_int, qmin, qmax).reshape(N, K)
    return pack_from_quant(x_int, s, None if disable_zero_point else zeros, n_bits, N, K,
                           group_size, disable_zero_point)


def dequant_packed(qweight, qsz, n_bits, N, K, group_size=None):
    """W_dq = RN16( RN16(q - zp) * s ) from the canonical layout (fp16, bit-exact with the
    reference's ``x_dequant.sub(zp).mul(scale)``, quantizer.py:107-110)."""
    g = group_size or K
    sc, zr = unpack_sz(qsz, N)
    u = unpack_qweight(qweight, n_bits, N, K).astype(np.float32).reshape(N, K // g, g)
    z = zr.astype(np.float32).reshape(N, K // g, 1)
    s = sc.reshape(N, K // g, 1)
    v = (u - z).astype(F16)  # exact integer, one fp16 rounding (matches RN16(x_int - zp))
    return _op(np.multiply, F16, v, s).reshape(N, K)


def linear_ref(x, w, bias=None):
    """``F.linear`` (int_linear.py:62) evaluated in float64 — the tolerance anchor for kernels."""
    y = np.asarray(x, dtype=np.float64) @ np.asarray(w, dtype=np.float64).T
    if bias is not None:
        y = y + np.asarray(bias, dtype=np.float64)
    return y
