"""ctypes binding of libqlin_gfx950.so (include/qlin_gfx950.h) — the only door from the Python
host mirror to the gfx950 kernels.

There is deliberately no fallback: if the library is missing, or a tensor is not on a HIP device,
every entry point raises.  PyTorch is used here only as the device allocator and for its current
HIP stream (``torch.cuda`` is PyTorch-ROCm's native HIP backend).
"""
from __future__ import annotations

import ctypes
import math
import os
import threading
import weakref

import torch

LIB_NAME = "libqlin_gfx950.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc",
                        LIB_NAME)
ABI_VERSION = 13

SYMMETRIC = 1
DISABLE_ZERO_POINT = 2
LWC = 4
WIDE_ZERO = 8
FLOAT_ZERO = 16
NORM_W16 = 32  # rmsnorm_linear_ep: fp16 norm weight
F16 = 0
F32 = 1

_DT = {torch.float16: F16, torch.float32: F32}

_lock = threading.Lock()
_lib = None

_p = ctypes.c_void_p
_i = ctypes.c_int
_l = ctypes.c_int64

SIGNATURES = {
    "qlin_abi_version": ([], _i),
    "qlin_error_string": ([_i], ctypes.c_char_p),
    "qlin_quantize": ([_p, _i, _l, _l, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p], _i),
    "qlin_fake_quant": ([_p, _i, _p, _p, _l, _l, _i, _i, _i, _p, _p, _p, _p], _i),
    "qlin_pack_f16": ([_p, _p, _p, _l, _l, _i, _i, _i, _p, _p, _p], _i),
    "qlin_pack_codes": ([_p, _l, _l, _i, _p, _p], _i),
    "qlin_dequant_f16": ([_p, _p, _i, _l, _l, _i, _i, _p, _p], _i),
    "qlin_gemv_f16": ([_p, _p, _i, _p, _p, _p, _l, _l, _l, _i, _i, _p], _i),
    "qlin_gemm_f16": ([_p, _p, _i, _p, _p, _p, _l, _l, _l, _i, _i, _p, _l, _p], _i),
    "qlin_gemv_batched_f16": ([_p, _l, _p, _l, _i, _p, _l, _p, _l, _p, _l, _l, _l, _l, _l, _i, _i,
                               _p], _i),
    "qlin_gemv_batched_plan": ([_p, _l, _p, _l, _i, _p, _l, _l, _l, _l, _l, _i, _i, _p], _i),
    "qlin_linear_f16": ([_p, _p, _i, _p, _p, _p, _l, _l, _l, _i, _i, _p], _i),
    "qlin_gemm_block_cols": ([_l, _l, _i], _i),
    "qlin_gemv_m1_route": ([_l, _l, _i, _i], _i),
    "qlin_linear_workspace_bytes": ([_l, _l, _l, _i, _i, _i], _l),
    "qlin_linear_ep_f16": ([_p, _p, _i, _p, _p, _p, _p, _l, _l, _l, _i, _i, _i, _i, _i, _p, _l, _p],
                           _i),
    "qlin_rmsnorm_f16": ([_p, _p, _p, _l, _l, ctypes.c_float, _p], _i),
    "qlin_rope_f16": ([_p, _l, _p, _l, _p, _p, _l, _p, _l, _p, _p, _l, _l, _i, _i, _i, _p], _i),
    "qlin_attn_decode_rope": ([_p, _l, _p, _l, _p, _l, _p, _p, _l, _p, _l, _p, _p, _l, _p, _p, _i,
                               _l, _i, _i, _l, _i, ctypes.c_float, _p, _p, _p], _i),
    "qlin_rmsnorm_linear_supported": ([_l, _l, _l, _i, _i], _i),
    "qlin_rmsnorm_linear_ep_f16": ([_p, _p, _i, _p, _p, ctypes.c_float, _p, _p, _p, _l, _l, _l,
                                    _i, _i, _i, _p], _i),
    "qlin_rope_kv_f16": ([_p, _l, _p, _l, _p, _l, _p, _p, _l, _p, _l, _p, _p, _p, _l, _l, _l, _l,
                          _i, _i, _i, _p], _i),
    "qlin_attn_scores_f32": ([_p, _p, _i, _l, _l, _l, _l, _l, ctypes.c_float, _p], _i),
    "qlin_attn_decode_partials_bytes": ([_l, _i, _i, _l], _l),
    "qlin_attn_prefill": ([_p, _p, _p, _p, _i, _l, _i, _p, _i, _l, _i, _i, _l, _l, _i,
                           ctypes.c_float, _p], _i),
    "qlin_attn_decode": ([_p, _p, _p, _p, _p, _i, _l, _i, _i, _l, _i, _l, ctypes.c_float, _p, _p,
                          _p],
                         _i),
    "qlin_attn_decode_splits": ([_l, _i, _l], _i),
    "qlin_attn_decode_rope_len": ([_p, _l, _p, _l, _p, _l, _p, _p, _l, _p, _l, _p, _p, _l, _p, _i,
                                   _l, _i, _i, _l, _i, ctypes.c_float, _p, _p, _p, _p], _i),
}


class QlinError(RuntimeError):
    pass


def load_library(path: str | None = None) -> ctypes.CDLL:
    """Load (once) and type the C ABI.  Raises if the library was not built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = path or os.environ.get("QLIN_LIBRARY", LIB_PATH)
        if not os.path.exists(path):
            raise QlinError(f"{LIB_NAME} not found at {path}: build it with "
                            "`python -c 'import __graft_entry__ as g; g.build()'` "
                            "(make -C llama3-quantization_amd/csrc)")
        lib = ctypes.CDLL(path)
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        v = lib.qlin_abi_version()
        if v != ABI_VERSION:
            raise QlinError(f"{path}: ABI version {v}, expected {ABI_VERSION}")
        _lib = lib
        return lib


def _check(rc: int, what: str):
    if rc != 0:
        msg = load_library().qlin_error_string(rc).decode()
        if rc == 1:
            raise ValueError(f"{what}: {msg}")
        raise QlinError(f"{what}: HIP error {rc} ({msg})")


def _dev(*ts):
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("qlin kernels run on gfx950 only: got a CPU tensor "
                               "(no CPU fallback exists)")
        if not t.is_contiguous():
            raise ValueError("qlin kernels need contiguous tensors")


def _on_gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("qlin kernels run on gfx950 only: got a CPU tensor "
                               "(no CPU fallback exists)")


def _ptr(t):
    return None if t is None else t.data_ptr()


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _dtcode(t):
    if t.dtype not in _DT:
        raise ValueError(f"unsupported dtype {t.dtype} (fp16 / fp32)")
    return _DT[t.dtype]


TILE_N = 16
TILE_K = 128


def packed_shape(N: int, K: int, bits: int):
    """qweight shape of the tiled layout: [ceil(N/16), ceil(K/128), 64 lanes, bits words]."""
    return (-(-N // TILE_N), -(-K // TILE_K), 64, bits)


def sz_shape(N: int, K: int, group: int):
    """qsz shape: [ceil(N/16), K/group, 16] words of (fp16 scale | int16 zero << 16)."""
    return (-(-N // TILE_N), K // group, TILE_N)


WIDE_LIMIT = 1024  # |zero| above this needs the fp32 (u - zero) path (QLIN_WIDE_ZERO)


def _alloc_packed(rows, K, bits, group, device):
    qw = torch.zeros(packed_shape(rows, K, bits), dtype=torch.int32, device=device)
    qsz = torch.zeros(sz_shape(rows, K, group), dtype=torch.int32, device=device)
    return qw, qsz


def split_sz(qsz: torch.Tensor, N: int):
    """qsz -> (scales fp16 [N, G], zeros int16 [N, G]) — the reference's scales / zeros views."""
    nt, G, _ = qsz.shape
    w = qsz.permute(0, 2, 1).reshape(nt * TILE_N, G)[:N]
    scales = (w & 0xFFFF).to(torch.int16).view(torch.float16)
    zeros = (w >> 16).to(torch.int16)
    return scales, zeros


def join_sz(scales: torch.Tensor, zeros: torch.Tensor) -> torch.Tensor:
    """(scales fp16 [N, G], integral zeros [N, G]) -> qsz [ceil(N/16), G, 16]."""
    N, G = scales.shape
    nt = -(-N // TILE_N)
    lo = scales.contiguous().view(torch.int16).to(torch.int32) & 0xFFFF
    hi = zeros.to(torch.int32) << 16
    w = torch.zeros(nt * TILE_N, G, dtype=torch.int32, device=scales.device)
    w[:N] = lo | hi
    return w.view(nt, TILE_N, G).permute(0, 2, 1).contiguous()


def join_sz_float(scales: torch.Tensor, zeros: torch.Tensor) -> torch.Tensor:
    """(scales fp16 [N, G], zeros fp16 [N, G]) -> qsz [ceil(N/16), G, 16] with the fp16 zero in
    the high half (layout flag QLIN_FLOAT_ZERO; HQQ's non-integral zero points)."""
    N, G = scales.shape
    nt = -(-N // TILE_N)
    lo = scales.to(torch.float16).contiguous().view(torch.int16).to(torch.int32) & 0xFFFF
    hi = zeros.to(torch.float16).contiguous().view(torch.int16).to(torch.int32) << 16
    w = torch.zeros(nt * TILE_N, G, dtype=torch.int32, device=scales.device)
    w[:N] = lo | hi
    return w.view(nt, TILE_N, G).permute(0, 2, 1).contiguous()


def pack_codes(codes: torch.Tensor, bits: int) -> torch.Tensor:
    """Integer codes uint8 [N, K] -> tiled qweight (``qlin_pack_codes``)."""
    _dev(codes)
    if codes.dtype != torch.uint8 or codes.dim() != 2:
        raise ValueError(f"codes must be uint8 [N, K], got {codes.dtype} {tuple(codes.shape)}")
    N, K = codes.shape
    qw = torch.zeros(packed_shape(N, K, bits), dtype=torch.int32, device=codes.device)
    rc = load_library().qlin_pack_codes(_ptr(codes), N, K, bits, _ptr(qw), _stream(codes))
    _check(rc, "qlin_pack_codes")
    return qw


def sz_flags(qsz: torch.Tensor) -> int:
    """QLIN_WIDE_ZERO if some zero point is outside +-1024 (degenerate groups only)."""
    if qsz.numel() == 0:
        return 0
    return WIDE_ZERO if int((qsz >> 16).abs().max()) > WIDE_LIMIT else 0


def quantize(x: torch.Tensor, bits: int, group: int, flags: int = 0, up_sig=None, low_sig=None,
             want_xdq=True, want_params=True, pack=False):
    """Fused calibrate + fake-quant (+ pack) of ``x`` viewed as [rows, K]; ``group`` divides K.

    Returns dict with ``x_dq`` [rows, K], ``scale`` / ``zp`` [rows*K/group] and, if ``pack``,
    ``qweight`` / ``qsz`` (tiled layout) and ``flags`` (layout flags for dequant / linear)."""
    _dev(x, up_sig, low_sig)
    K = x.shape[-1]
    rows = x.numel() // K if K else 0
    out = {}
    xdq = torch.empty_like(x) if want_xdq else None
    ng = rows * (K // group) if group else 0
    scale = torch.empty(ng, dtype=x.dtype, device=x.device) if want_params else None
    zp = torch.empty(ng, dtype=x.dtype, device=x.device) if (
        want_params and not flags & DISABLE_ZERO_POINT) else None
    qw = qsz = None
    if pack:
        if group <= 0 or K % group:
            raise ValueError(f"group {group} must divide K {K}")
        qw, qsz = _alloc_packed(rows, K, bits, group, x.device)
    rc = load_library().qlin_quantize(
        _ptr(x), _dtcode(x), rows, K, bits, group, flags, _ptr(up_sig), _ptr(low_sig),
        _ptr(xdq), _ptr(scale), _ptr(zp), _ptr(qw), _ptr(qsz), _stream(x))
    _check(rc, "qlin_quantize")
    out.update(x_dq=xdq, scale=scale, zp=zp)
    if pack:
        out.update(qweight=qw, qsz=qsz, flags=sz_flags(qsz))
    return out


def fake_quant(x: torch.Tensor, scale: torch.Tensor, zp, bits: int, group: int, flags: int = 0,
               want_xdq=True, pack=False):
    """``fake_quant`` with given (scale, zp) [rows*K/group]; optionally pack the codes."""
    _dev(x, scale, zp)
    K = x.shape[-1]
    rows = x.numel() // K
    xdq = torch.empty_like(x) if want_xdq else None
    qw = qsz = None
    if pack:
        if group <= 0 or K % group:
            raise ValueError(f"group {group} must divide K {K}")
        qw, qsz = _alloc_packed(rows, K, bits, group, x.device)
    if scale.dtype != x.dtype or (zp is not None and zp.dtype != x.dtype):
        raise ValueError("scale / zero point dtype must match x")
    rc = load_library().qlin_fake_quant(
        _ptr(x), _dtcode(x), _ptr(scale), _ptr(zp), rows, K, bits, group, flags, _ptr(xdq),
        _ptr(qw), _ptr(qsz), _stream(x))
    _check(rc, "qlin_fake_quant")
    return dict(x_dq=xdq, qweight=qw, qsz=qsz, flags=sz_flags(qsz) if pack else 0)


def _check_packed(qweight, qsz, N, K, bits, group):
    if group <= 0 or K % group:
        raise ValueError(f"group {group} must divide K {K}")
    if tuple(qweight.shape) != packed_shape(N, K, bits) or qweight.dtype != torch.int32:
        raise ValueError(f"qweight must be int32 {packed_shape(N, K, bits)}, got "
                         f"{qweight.dtype} {tuple(qweight.shape)}")
    if tuple(qsz.shape) != sz_shape(N, K, group) or qsz.dtype != torch.int32:
        raise ValueError(f"qsz must be int32 {sz_shape(N, K, group)}, got "
                         f"{qsz.dtype} {tuple(qsz.shape)}")


def dequant(qweight, qsz, N: int, K: int, bits: int, group: int, flags: int = 0) -> torch.Tensor:
    _dev(qweight, qsz)
    _check_packed(qweight, qsz, N, K, bits, group)
    w = torch.empty(N, K, dtype=torch.float16, device=qweight.device)
    rc = load_library().qlin_dequant_f16(_ptr(qweight), _ptr(qsz), flags, N, K, bits, group,
                                         _ptr(w), _stream(qweight))
    _check(rc, "qlin_dequant_f16")
    return w


def _linear_call(fn_name, x, qweight, qsz, bias, N, K, bits, group, flags, extra=()):
    _dev(x, qweight, qsz, bias)
    if x.dtype != torch.float16:
        raise ValueError(f"packed linear takes fp16 activations, got {x.dtype}")
    if x.shape[-1] != K:
        raise ValueError(f"input has {x.shape[-1]} features, layer expects {K}")
    if bias is not None and (bias.dtype != torch.float16 or bias.numel() != N):
        raise ValueError("bias must be fp16 [N]")
    _check_packed(qweight, qsz, N, K, bits, group)
    M = x.numel() // K if K else 0
    y = torch.empty(*x.shape[:-1], N, dtype=torch.float16, device=x.device)
    if M == 0:
        return y
    fn = getattr(load_library(), fn_name)
    rc = fn(_ptr(qweight), _ptr(qsz), flags, _ptr(x), _ptr(bias), _ptr(y), M, N, K, bits, group,
            *extra, _stream(x))
    _check(rc, fn_name)
    return y


def linear(x, qweight, qsz, bias, N, K, bits, group, flags=0):
    """Dispatching fused dequant-matmul (GEMV kernel for M <= 64 in 16-row chunks, MFMA GEMM
    above, split-K for small grids): ``qlin_linear_ep_f16`` without an epilogue, which takes the
    split-K workspace (``qlin_linear_f16``, the same dispatch without it, runs unsplit)."""
    return linear_ep(x, qweight, qsz, bias, N, K, bits, group, flags)


def gemv(x, qweight, qsz, bias, N, K, bits, group, flags=0):
    return _linear_call("qlin_gemv_f16", x, qweight, qsz, bias, N, K, bits, group, flags)


def gemv_batched(x, qweight, qsz, bias, N, K, bits, group, flags=0, out=None):
    """``qlin_gemv_batched_f16``: B independent decode products in one launch.

    x [B, M, K] fp16 (M <= 16), or [M, K] shared by every problem; qweight [B, *packed_shape],
    qsz [B, *sz_shape] (one packed matrix per problem, same N / K / bits / group / flags); bias
    [B, N] or None.  Returns y [B, M, N]: for M <= 4 and K % 512 == 0 each y[b] is bit-identical
    to ``gemm(x[b], ..., split=False)`` (one MFMA chain per output in k order), otherwise to
    ``gemv(x[b], ...)``."""
    _dev(x, qweight, qsz, bias, out)
    if x.dtype != torch.float16 or x.dim() not in (2, 3) or x.shape[-1] != K:
        raise ValueError(f"x must be fp16 [B, M, {K}] or [M, {K}], got {x.dtype} {tuple(x.shape)}")
    B = qweight.shape[0] if qweight.dim() == 5 else -1
    shared_x = x.dim() == 2
    M = x.shape[0] if shared_x else x.shape[1]
    if not shared_x and x.shape[0] != B:
        raise ValueError(f"x has {x.shape[0]} problems, qweight {B}")
    if tuple(qweight.shape) != (B, *packed_shape(N, K, bits)) or qweight.dtype != torch.int32:
        raise ValueError(f"qweight must be int32 {(B, *packed_shape(N, K, bits))}")
    if tuple(qsz.shape) != (B, *sz_shape(N, K, group)) or qsz.dtype != torch.int32:
        raise ValueError(f"qsz must be int32 {(B, *sz_shape(N, K, group))}")
    if bias is not None and (bias.dtype != torch.float16 or tuple(bias.shape) != (B, N)):
        raise ValueError("bias must be fp16 [B, N]")
    y = out if out is not None else torch.empty(B, M, N, dtype=torch.float16, device=x.device)
    if tuple(y.shape) != (B, M, N) or y.dtype != torch.float16:
        raise ValueError(f"out must be fp16 [{B}, {M}, {N}]")
    if B == 0 or M == 0:
        return y
    rc = load_library().qlin_gemv_batched_f16(
        _ptr(qweight), qweight[0].numel(), _ptr(qsz), qsz[0].numel(), flags, _ptr(x),
        0 if shared_x else M * K,
        _ptr(bias), N, _ptr(y), M * N, B, M, N, K, bits, group, _stream(x))
    _check(rc, "qlin_gemv_batched_f16")
    return y


def gemv_batched_plan(x, qweight, qsz, N, K, bits, group, flags=0):
    """The launch geometry ``gemv_batched`` would use for these operands (nothing launched;
    ``qlin_gemv_batched_plan``): dict(blocks, dyn_lds, static_lds, blocks_per_cu, rows_per_wave),
    all 0 when the arguments take the per-problem path."""
    B = qweight.shape[0]
    shared_x = x.dim() == 2
    M = x.shape[0] if shared_x else x.shape[1]
    plan = (ctypes.c_int64 * 5)()
    rc = load_library().qlin_gemv_batched_plan(
        _ptr(qweight), qweight[0].numel(), _ptr(qsz), qsz[0].numel(), flags, _ptr(x),
        0 if shared_x else M * K, B, M, N, K, bits, group, plan)
    _check(rc, "qlin_gemv_batched_plan")
    return dict(zip(("blocks", "dyn_lds", "static_lds", "blocks_per_cu", "rows_per_wave"),
                    list(plan)))


def gemm(x, qweight, qsz, bias, N, K, bits, group, flags=0, split=True):
    """``qlin_gemm_f16``; ``split``: pass the split-K workspace (small grids split K)."""
    M = x.numel() // K if K else 0
    ws = _workspace(x.device, M, N, K, bits, group) if (split and M) else None
    return _linear_call("qlin_gemm_f16", x, qweight, qsz, bias, N, K, bits, group, flags,
                        extra=(_ptr(ws), 0 if ws is None else ws.numel()))


SKINNY_MAX_M = 64  # qlin_linear_*: M <= this runs the GEMV kernel
ACT_FUSE_MAX_N = 16384  # qlin_linear_ep_f16 fuses the act fake-quant into the GEMV up to this N
EP_NONE = 0
EP_RESIDUAL = 1
EP_SILU_MUL = 2


def _workspace(device, M, N, K, bits, group, act_bits=0):
    """The launch's workspace (qlin_linear_workspace_bytes: act fake-quant x_dq, split-K
    partials) or None."""
    nb = load_library().qlin_linear_workspace_bytes(M, N, K, bits, group, act_bits)
    if nb < 0:
        raise ValueError(f"invalid linear shape M={M} N={N} K={K} b{bits} g{group}")
    return torch.empty(nb, dtype=torch.uint8, device=device) if nb else None


def linear_ep(x, qweight, qsz, bias, N, K, bits, group, flags=0, epilogue=EP_NONE,
              residual=None, act_bits=0, act_flags=0):
    """``qlin_linear_ep_f16``: the packed linear with a fused output epilogue.

    EP_RESIDUAL: ``residual + F.linear(x)`` (residual fp16, shape of the output).
    EP_SILU_MUL: rows interleaved by ``interleave_gate_up``; returns ``silu(gate) * up`` with
    N / 2 columns.
    act_bits: per-token activation fake-quant of x first (fused into the GEMV for M <= 64)."""
    _dev(x, qweight, qsz, bias, residual)
    if x.dtype != torch.float16:
        raise ValueError(f"packed linear takes fp16 activations, got {x.dtype}")
    if x.shape[-1] != K:
        raise ValueError(f"input has {x.shape[-1]} features, layer expects {K}")
    if bias is not None and (bias.dtype != torch.float16 or bias.numel() != N):
        raise ValueError("bias must be fp16 [N]")
    _check_packed(qweight, qsz, N, K, bits, group)
    ny = N // 2 if epilogue == EP_SILU_MUL else N
    y = torch.empty(*x.shape[:-1], ny, dtype=torch.float16, device=x.device)
    if epilogue == EP_RESIDUAL:
        if residual is None or residual.dtype != torch.float16 or residual.shape != y.shape:
            raise ValueError(f"residual must be fp16 {tuple(y.shape)}")
    M = x.numel() // K if K else 0
    if M == 0:
        return y
    ws = _workspace(x.device, M, N, K, bits, group, act_bits)
    rc = load_library().qlin_linear_ep_f16(_ptr(qweight), _ptr(qsz), flags, _ptr(x), _ptr(bias),
                                           _ptr(residual), _ptr(y), M, N, K, bits, group,
                                           epilogue, act_bits, act_flags, _ptr(ws),
                                           0 if ws is None else ws.numel(), _stream(x))
    _check(rc, "qlin_linear_ep_f16")
    return y


M1_GENERAL, M1_WORK_QUEUE, M1_FAST, M1_ROWS = 0, 1, 2, 3
M1_WHOLE_ROW = M1_WORK_QUEUE  # round-4 name of route 1 (its whole-row kernel became the work queue)


def m1_route(N, K, bits, group):
    """The kernel a one-token-row product of this shape runs (``qlin_gemv_m1_route``):
    M1_WORK_QUEUE (wide matrices: chunks of 4 k-tiles taken from an LDS counter, per-chunk partial
    sums added per row in k order), M1_FAST (split-K fast kernel), M1_ROWS (long K) or M1_GENERAL
    (the general GEMV kernel; no fused RMSNorm there)."""
    r = load_library().qlin_gemv_m1_route(N, K, bits, group)
    if r < 0:
        raise ValueError(f"m1_route: invalid shape N={N} K={K} b{bits} g{group}")
    return r


def rmsnorm_linear_supported(M, N, K, bits, group):
    """Whether ``rmsnorm_linear_ep`` takes this shape (one token row on the fast GEMV path)."""
    return bool(load_library().qlin_rmsnorm_linear_supported(M, N, K, bits, group))


def rmsnorm_linear_ep(x, norm_weight, eps, qweight, qsz, bias, N, K, bits, group, flags=0,
                      epilogue=EP_NONE, residual=None):
    """``qlin_rmsnorm_linear_ep_f16``: ``linear_ep(rmsnorm(x))`` for one token row in ONE launch —
    x fp16 [.., K] is the hidden state BEFORE the RMSNorm (norm_weight fp32 [K], eps), which the
    kernel applies at the reference's rounding point, RN16(w * (x * rsqrt(mean(x^2) + eps)))
    (the sum of squares in another order than ``rmsnorm``: an fp16 ulp of the normed x can
    differ from it).  An fp16 norm weight is read as fp16 (QLIN_NORM_W16: half the bytes; every
    fp16 is exact in fp32, so the result is the one of its fp32 copy)."""
    _dev(x, qweight, qsz, bias, residual, norm_weight)
    if x.dtype != torch.float16 or norm_weight.dtype not in (torch.float32, torch.float16):
        raise ValueError("rmsnorm_linear_ep takes fp16 x and an fp32 or fp16 norm weight")
    if not norm_weight.is_contiguous():
        raise ValueError("norm weight must be contiguous")
    if norm_weight.dtype == torch.float16:
        flags |= NORM_W16
    if x.shape[-1] != K or norm_weight.numel() != K:
        raise ValueError(f"input / norm weight do not have {K} features")
    if bias is not None and (bias.dtype != torch.float16 or bias.numel() != N):
        raise ValueError("bias must be fp16 [N]")
    _check_packed(qweight, qsz, N, K, bits, group)
    M = x.numel() // K
    if not rmsnorm_linear_supported(M, N, K, bits, group):
        raise ValueError(f"rmsnorm_linear_ep: unsupported shape M={M} N={N} K={K} g{group}")
    ny = N // 2 if epilogue == EP_SILU_MUL else N
    y = torch.empty(*x.shape[:-1], ny, dtype=torch.float16, device=x.device)
    if epilogue == EP_RESIDUAL:
        if residual is None or residual.dtype != torch.float16 or residual.shape != y.shape:
            raise ValueError(f"residual must be fp16 {tuple(y.shape)}")
    rc = load_library().qlin_rmsnorm_linear_ep_f16(
        _ptr(qweight), _ptr(qsz), flags, _ptr(x), _ptr(norm_weight), float(eps), _ptr(bias),
        _ptr(residual), _ptr(y), M, N, K, bits, group, epilogue, _stream(x))
    _check(rc, "qlin_rmsnorm_linear_ep_f16")
    return y


def interleave_gate_up(qw_gate, qsz_gate, qw_up, qsz_up):
    """Packed gate / up matrices (same N, a multiple of 16) -> one matrix whose 16-row tile j
    holds gate rows 8j..8j+7 then up rows 8j..8j+7 (the EP_SILU_MUL row order).  A permutation
    of whole lane pieces and (scale, zero) words: no value changes."""
    T, Kt, _, b = qw_gate.shape
    G = qsz_gate.shape[1]
    if qw_up.shape != qw_gate.shape or qsz_up.shape != qsz_gate.shape:
        raise ValueError("gate and up must have the same packed shapes")
    # qweight [T, Kt, 64 = 4 q x 16 n, b] -> [T, half, Kt, q, 8, b]
    pw = lambda w: w.view(T, Kt, 4, 2, 8, b).permute(0, 3, 1, 2, 4, 5)
    qw = torch.stack([pw(qw_gate), pw(qw_up)], dim=4).reshape(2 * T, Kt, 64, b)
    ps = lambda z: z.view(T, G, 2, 8).permute(0, 2, 1, 3)
    qsz = torch.stack([ps(qsz_gate), ps(qsz_up)], dim=3).reshape(2 * T, G, 16)
    return qw.contiguous(), qsz.contiguous()


def rmsnorm(x, weight_f32, eps):
    """``qlin_rmsnorm_f16``: OmniLlamaRMSNorm on fp16 ``x`` [..., H] with the fp32 weight."""
    _dev(x, weight_f32)
    if x.dtype != torch.float16 or weight_f32.dtype != torch.float32:
        raise ValueError("rmsnorm takes fp16 x and an fp32 weight")
    H = x.shape[-1]
    if weight_f32.numel() != H:
        raise ValueError(f"weight has {weight_f32.numel()} values, x has {H} features")
    y = torch.empty_like(x)
    rc = load_library().qlin_rmsnorm_f16(_ptr(x), _ptr(weight_f32), _ptr(y), x.numel() // H, H,
                                         float(eps), _stream(x))
    _check(rc, "qlin_rmsnorm_f16")
    return y


def _rows(t):
    """(row stride) of a [B, S, C] tensor whose rows are uniformly strided with unit inner
    stride, else None."""
    if t.dim() == 3 and t.stride(2) == 1 and (t.shape[0] == 1 or t.stride(0) == t.shape[1] * t.stride(1)):
        return t.stride(1)
    return None


def rope(q, k, cos_cache, sin_cache, position_ids, n_heads, n_kv_heads, head_dim):
    """``qlin_rope_f16``: q [B, S, Hq*D], k [B, S, Hkv*D] fp16 (row-strided views allowed) ->
    (q_rot fp32 [B, Hq, S, D], k_rot fp16 [B, Hkv, S, D]) exactly as the reference's
    ``apply_rotary_pos_emb(q.transpose(1, 2).float(), k.transpose(1, 2), cos, sin, pos)``."""
    if _rows(q) is None:
        q = q.contiguous()
    if _rows(k) is None:
        k = k.contiguous()
    for t_ in (q, k, cos_cache, sin_cache, position_ids):
        if not t_.is_cuda:
            raise RuntimeError("qlin kernels run on gfx950 only: got a CPU tensor")
    if q.dtype != torch.float16 or k.dtype != torch.float16:
        raise ValueError("rope takes fp16 q / k")
    if cos_cache.dtype != torch.float32 or sin_cache.dtype != torch.float32 or \
            not cos_cache.is_contiguous() or not sin_cache.is_contiguous():
        raise ValueError("rope takes contiguous fp32 cos / sin caches")
    B, S = q.shape[0], q.shape[1]
    pos = position_ids
    if pos.dtype != torch.int64:
        pos = pos.to(torch.int64)
    if pos.dim() == 1:
        pos = pos[None]
    if pos.stride(-1) != 1:
        pos = pos.contiguous()
    pbs = pos.stride(0) if pos.shape[0] > 1 else 0
    if pos.shape[-1] != S or pos.shape[0] not in (1, B):
        raise ValueError(f"position_ids {tuple(pos.shape)} do not match [B={B}, S={S}]")
    q_out = torch.empty(B, n_heads, S, head_dim, dtype=torch.float32, device=q.device)
    k_out = torch.empty(B, n_kv_heads, S, head_dim, dtype=torch.float16, device=q.device)
    if cos_cache.shape != sin_cache.shape or cos_cache.shape[-1] != head_dim:
        raise ValueError("cos / sin caches must be [rows, head_dim]")
    rc = load_library().qlin_rope_f16(_ptr(q), _rows(q), _ptr(k), _rows(k), _ptr(cos_cache),
                                      _ptr(sin_cache), cos_cache.shape[0], _ptr(pos), pbs, _ptr(q_out), _ptr(k_out),
                                      B, S, n_heads, n_kv_heads, head_dim, _stream(q))
    _check(rc, "qlin_rope_f16")
    return q_out, k_out


def _pos_ids(position_ids, B, S):
    pos = position_ids
    if pos.dtype != torch.int64:
        pos = pos.to(torch.int64)
    if pos.dim() == 1:
        pos = pos[None]
    if pos.stride(-1) != 1:
        pos = pos.contiguous()
    if pos.shape[-1] != S or pos.shape[0] not in (1, B):
        raise ValueError(f"position_ids {tuple(pos.shape)} do not match [B={B}, S={S}]")
    return pos, (pos.stride(0) if pos.shape[0] > 1 else 0)


def rope_kv(q, k, v, cos_cache, sin_cache, position_ids, n_heads, n_kv_heads, head_dim,
            k_cache, v_cache, kv0):
    """``qlin_rope_kv_f16``: ``rope`` plus the KV-cache append of the step. q [B, S, Hq*D],
    k / v [B, S, Hkv*D] fp16 row-strided views; k_cache / v_cache fp16 [B, Hkv, rows, D]
    contiguous buffers, rows kv0 .. kv0 + S - 1 written in place (the rotated k, and v).
    Returns q_rot fp32 [B, Hq, S, D] (the reference's apply_rotary_pos_emb output for q)."""
    for t_ in (q, k, v):
        if _rows(t_) is None:
            raise ValueError("rope_kv takes row-strided [B, S, H*D] q / k / v")
    for t_ in (q, k, v, cos_cache, sin_cache, position_ids, k_cache, v_cache):
        if not t_.is_cuda:
            raise RuntimeError("qlin kernels run on gfx950 only: got a CPU tensor")
    if q.dtype != torch.float16 or k.dtype != torch.float16 or v.dtype != torch.float16 or \
            k_cache.dtype != torch.float16 or v_cache.dtype != torch.float16:
        raise ValueError("rope_kv takes fp16 q / k / v and caches")
    if not (k_cache.is_contiguous() and v_cache.is_contiguous()) or k_cache.shape != v_cache.shape:
        raise ValueError("rope_kv takes contiguous [B, Hkv, rows, D] caches of one shape")
    B, S = q.shape[0], q.shape[1]
    if tuple(k_cache.shape[:2]) != (B, n_kv_heads) or k_cache.shape[3] != head_dim:
        raise ValueError(f"cache {tuple(k_cache.shape)} does not match [B={B}, Hkv={n_kv_heads}, ., D]")
    if kv0 < 0 or kv0 + S > k_cache.shape[2]:
        raise ValueError(f"cache rows {k_cache.shape[2]} cannot take rows {kv0} .. {kv0 + S - 1}")
    pos, pbs = _pos_ids(position_ids, B, S)
    q_out = torch.empty(B, n_heads, S, head_dim, dtype=torch.float32, device=q.device)
    rc = load_library().qlin_rope_kv_f16(
        _ptr(q), _rows(q), _ptr(k), _rows(k), _ptr(v), _rows(v), _ptr(cos_cache),
        _ptr(sin_cache), cos_cache.shape[0], _ptr(pos), pbs, _ptr(q_out), _ptr(k_cache),
        _ptr(v_cache), k_cache.shape[2], kv0, B, S, n_heads, n_kv_heads, head_dim, _stream(q))
    _check(rc, "qlin_rope_kv_f16")
    return q_out


def attn_scores_(w, mask, scale_div):
    """In place: w = max(w / scale_div + mask, finfo(fp32).min) (``qlin_attn_scores_f32``); w fp32
    [B, H, T, L] contiguous, mask [B or 1, 1, T, L] fp16/fp32 or None.  Returns w."""
    _dev(w)
    if w.dtype != torch.float32 or w.dim() != 4 or w.shape[-1] % 4:
        raise ValueError("scores must be contiguous fp32 [B, H, T, L] with L % 4 == 0")
    B, H, T, L = w.shape
    m, mbs, mdt = None, 0, F16
    if mask is not None:
        if mask.dtype not in (torch.float16, torch.float32) or mask.shape[-2:] != (T, L) or \
                mask.shape[1] != 1 or mask.shape[0] not in (1, B):
            raise ValueError(f"mask {tuple(mask.shape)} does not match scores {tuple(w.shape)}")
        if mask.stride(-1) != 1 or mask.stride(-2) != L:
            mask = mask.contiguous()
        m = mask
        mbs = mask.stride(0) if mask.shape[0] > 1 else 0
        mdt = _DT[mask.dtype]
        if not m.is_cuda:
            raise RuntimeError("qlin kernels run on gfx950 only: got a CPU tensor")
    rc = load_library().qlin_attn_scores_f32(_ptr(w), _ptr(m), mdt, B, H, T, L, mbs,
                                             float(scale_div), _stream(w))
    _check(rc, "qlin_attn_scores_f32")
    return w


ATTN_MAX_L = 4096
ATTN_D = 128


def attn_decode_supported(q, k, mask=None):
    """Whether qlin_attn_decode takes this call (see attn_decode)."""
    return (q.is_cuda and q.dim() == 4 and q.shape[2] == 1 and q.shape[-1] == ATTN_D
            and q.dtype == torch.float32 and k.dtype == torch.float16
            and k.shape[2] <= ATTN_MAX_L and q.shape[1] % k.shape[1] == 0
            and q.shape[1] // k.shape[1] in (1, 2, 4, 8)
            and (mask is None or (mask.dtype == torch.float16 and mask.shape[-2] == 1)))


_ATTN_COUNTERS = {}


def _attn_counters(device, heads):
    """Zero-filled split-L merge counters, one buffer per (device, stream), grown on demand (the
    kernel leaves them zero).  Grow outside graph capture: an eager call before capture sizes it."""
    key = (device.index, torch.cuda.current_stream(device).cuda_stream)
    c = _ATTN_COUNTERS.get(key)
    if c is None or c.numel() < heads:
        c = torch.zeros(max(heads, 4096), dtype=torch.int32, device=device)
        _ATTN_COUNTERS[key] = c
    return c


def _cache_head_stride(k, v):
    """Head stride (elements) when k / v [B, Hkv, L, D] are row-prefix views of contiguous
    [B, Hkv, rows, D] cache buffers (rope_kv), else None (the caller makes them contiguous)."""
    if k.stride() != v.stride() or k.stride(3) != 1 or k.stride(2) != k.shape[3]:
        return None
    hs = k.stride(1)
    if hs < k.shape[2] * k.shape[3] or hs % 8 or (k.shape[0] > 1 and k.stride(0) != k.shape[1] * hs):
        return None
    return hs


def attn_decode(q, k, v, mask, scale_div, out_dtype=torch.float32):
    """softmax(q k^T / scale_div + mask) v for one query token: q fp32 [B, Hq, 1, D], k/v fp16
    [B, Hkv, L, D], mask fp16 [B, 1, 1, L] or None -> [B, Hq, 1, D] in out_dtype (fp32, or the
    fp32 result rounded to fp16 in the kernel); k / v may be row-prefix views of KV cache
    buffers (rope_kv), read in place."""
    _on_gpu(q, k, v)
    if not attn_decode_supported(q, k, mask):
        raise ValueError("attn_decode: unsupported shapes / dtypes")
    B, Hq, _, D = q.shape
    Hkv, L = k.shape[1], k.shape[2]
    hs = _cache_head_stride(k, v)
    if hs is None:
        k = k.contiguous()
        v = v.contiguous()
        hs = 0
    m = None
    if mask is not None:
        m = mask.reshape(B, L).contiguous() if mask.shape[0] == B else \
            mask.expand(B, 1, 1, L).reshape(B, L).contiguous()
    out = torch.empty(B, Hq, 1, D, dtype=out_dtype, device=q.device)
    lib = load_library()
    part, cnt = _attn_partials(lib, q.device, B, Hq, Hkv, L)
    rc = lib.qlin_attn_decode(_ptr(q.contiguous()), _ptr(k), _ptr(v), _ptr(m), _ptr(out),
                              _dtcode(out),
                              B, Hq, Hkv, L, D, hs, float(scale_div), _ptr(part), _ptr(cnt),
                              _stream(q))
    _check(rc, "qlin_attn_decode")
    return out


def _attn_partials(lib, device, B, Hq, Hkv, L):
    """(partials scratch, merge counters) of a decode attention launch."""
    nbytes = lib.qlin_attn_decode_partials_bytes(B, Hq, Hkv, L)
    if nbytes < 0:
        raise ValueError("attn_decode: unsupported shapes")
    if not nbytes:
        return None, None
    part = torch.empty(nbytes // 4, dtype=torch.float32, device=device)
    return part, _attn_counters(device, B * Hkv)


def attn_decode_rope(q, k, v, cos_cache, sin_cache, position_ids, n_heads, n_kv_heads, head_dim,
                     k_cache, v_cache, kv0, mask, scale_div, out_dtype=torch.float32):
    """``qlin_attn_decode_rope``: ``rope_kv`` + ``attn_decode`` in one launch for one new token:
    q [B, 1, Hq*D], k / v [B, 1, Hkv*D] fp16 row-strided views (before RoPE); k_cache / v_cache
    fp16 [B, Hkv, rows, D] contiguous buffers holding rows 0 .. kv0 - 1, row kv0 written here;
    mask fp16 [B, 1, 1, kv0 + 1] or None -> [B, Hq, 1, D] (out_dtype), bit-identical to the two
    launches."""
    for t_ in (q, k, v):
        if _rows(t_) is None:
            raise ValueError("attn_decode_rope takes row-strided [B, 1, H*D] q / k / v")
    _on_gpu(q, k, v, cos_cache, sin_cache, position_ids, k_cache, v_cache, mask)
    B = q.shape[0]
    if q.shape[1] != 1 or head_dim != ATTN_D or n_heads % n_kv_heads or \
            n_heads // n_kv_heads not in (1, 2, 4, 8):
        raise ValueError("attn_decode_rope: one token, head_dim 128, GQA group 1/2/4/8")
    if q.dtype != torch.float16 or k.dtype != torch.float16 or v.dtype != torch.float16 or \
            k_cache.dtype != torch.float16 or v_cache.dtype != torch.float16:
        raise ValueError("attn_decode_rope takes fp16 q / k / v and caches")
    if not (k_cache.is_contiguous() and v_cache.is_contiguous()) or k_cache.shape != v_cache.shape \
            or tuple(k_cache.shape[:2]) != (B, n_kv_heads) or k_cache.shape[3] != head_dim:
        raise ValueError("attn_decode_rope takes contiguous [B, Hkv, rows, D] caches of one shape")
    L = kv0 + 1
    if kv0 < 0 or L > k_cache.shape[2] or L > ATTN_MAX_L:
        raise ValueError(f"cache rows {k_cache.shape[2]} cannot take row {kv0}")
    if cos_cache.dtype != torch.float32 or not cos_cache.is_contiguous() or \
            sin_cache.dtype != torch.float32 or not sin_cache.is_contiguous():
        raise ValueError("rope takes contiguous fp32 cos / sin caches")
    if position_ids is None:
        # cos_cache / sin_cache are the step's own rows (rmsnorm_linear_ep(..., rope=...))
        if B != 1:
            raise ValueError("attn_decode_rope: position_ids None needs batch 1")
        pos, pbs = None, 0
    else:
        pos, pbs = _pos_ids(position_ids, B, 1)
    m = None
    if mask is not None:
        if mask.dtype != torch.float16 or mask.shape[-1] != L or mask.shape[-2] != 1:
            raise ValueError("attn_decode_rope: mask fp16 [B, 1, 1, L]")
        m = mask.reshape(B, L).contiguous() if mask.shape[0] == B else \
            mask.expand(B, 1, 1, L).reshape(B, L).contiguous()
    out = torch.empty(B, n_heads, 1, head_dim, dtype=out_dtype, device=q.device)
    lib = load_library()
    part, cnt = _attn_partials(lib, q.device, B, n_heads, n_kv_heads, L)
    rows = k_cache.shape[2]
    args = (_ptr(q), _rows(q), _ptr(k), _rows(k), _ptr(v), _rows(v), _ptr(cos_cache),
            _ptr(sin_cache), cos_cache.shape[0], _ptr(pos), pbs, _ptr(k_cache), _ptr(v_cache),
            rows * head_dim, _ptr(m), _ptr(out), _dtcode(out), B, n_heads, n_kv_heads, L, head_dim,
            float(scale_div), _ptr(part), _ptr(cnt), _stream(q))
    rc = lib.qlin_attn_decode_rope(*args)
    _check(rc, "qlin_attn_decode_rope")
    return out


def attn_decode_rope_len(q, k, v, cos_cache, sin_cache, position_ids, n_heads, n_kv_heads,
                         head_dim, k_cache, v_cache, length, out_dtype=torch.float32,
                         max_len=None):
    """``qlin_attn_decode_rope_len``: attn_decode_rope for graph-replayed decode steps — the cache
    length (this step's new row + 1) is read from the int32 device tensor ``length`` [1]; no mask.

    ``max_len``: the largest length ``length`` will hold over the captured steps (default: the
    caches' capacity, k_cache.shape[2] rows); the grid and the partials are sized for it.  It
    must fit the caches and the kernel's ATTN_MAX_L rows — a longer sequence has to take the
    per-step path (the kernel clamps the device length to max_len, so a length beyond it would
    attend over a prefix and rewrite row max_len - 1: rejected here, not clamped)."""
    for t_ in (q, k, v):
        if _rows(t_) is None:
            raise ValueError("attn_decode_rope_len takes row-strided [B, 1, H*D] q / k / v")
    _on_gpu(q, k, v, cos_cache, sin_cache, position_ids, k_cache, v_cache, length)
    B = q.shape[0]
    if q.shape[1] != 1 or head_dim != ATTN_D or n_heads % n_kv_heads or \
            n_heads // n_kv_heads not in (1, 2, 4, 8):
        raise ValueError("attn_decode_rope_len: one token, head_dim 128, GQA group 1/2/4/8")
    if length.dtype != torch.int32 or length.numel() < 1 or position_ids is None:
        raise ValueError("attn_decode_rope_len: int32 length tensor and position_ids required")
    if not (k_cache.is_contiguous() and v_cache.is_contiguous()) or k_cache.shape != v_cache.shape \
            or tuple(k_cache.shape[:2]) != (B, n_kv_heads) or k_cache.shape[3] != head_dim:
        raise ValueError("attn_decode_rope_len takes contiguous [B, Hkv, rows, D] caches")
    cap = k_cache.shape[2] if max_len is None else int(max_len)
    if cap < 1 or cap > k_cache.shape[2] or cap > ATTN_MAX_L:
        raise ValueError(f"attn_decode_rope_len: max length {cap} must fit the cache "
                         f"({k_cache.shape[2]} rows) and ATTN_MAX_L ({ATTN_MAX_L})")
    pos, pbs = _pos_ids(position_ids, B, 1)
    out = torch.empty(B, n_heads, 1, head_dim, dtype=out_dtype, device=q.device)
    lib = load_library()
    part, cnt = _attn_partials(lib, q.device, B, n_heads, n_kv_heads, cap)
    rc = lib.qlin_attn_decode_rope_len(
        _ptr(q), _rows(q), _ptr(k), _rows(k), _ptr(v), _rows(v), _ptr(cos_cache), _ptr(sin_cache),
        cos_cache.shape[0], _ptr(pos), pbs, _ptr(k_cache), _ptr(v_cache),
        k_cache.shape[2] * head_dim, _ptr(out), _dtcode(out), B, n_heads, n_kv_heads, cap,
        head_dim, ctypes.c_float(scale_div_default(head_dim)), _ptr(part), _ptr(cnt),
        _ptr(length), _stream(q))
    _check(rc, "qlin_attn_decode_rope_len")
    return out


def scale_div_default(head_dim):
    return math.sqrt(head_dim)


def attn_prefill_supported(q, k, mask=None):
    """Whether qlin_attn_prefill takes this call (see attn_prefill)."""
    return (q.is_cuda and q.dim() == 4 and k.dim() == 4 and q.shape[-1] == ATTN_D
            and q.dtype == torch.float32 and k.dtype == torch.float16
            and q.shape[0] == k.shape[0] and q.shape[2] <= k.shape[2]
            and q.shape[1] % k.shape[1] == 0 and q.shape[1] // k.shape[1] in (1, 2, 4, 8)
            and (mask is None or (mask.dim() == 4 and mask.shape[1] == 1
                                  and mask.shape[-2:] == (q.shape[2], k.shape[2])
                                  and mask.shape[0] in (1, q.shape[0])
                                  and mask.dtype in (torch.float16, torch.float32))))


_CAUSAL = []  # [(weakref to the mask tensor, its _version, S, L, result)], most recent last
_CAUSAL_KEEP = 4


def mask_is_causal(mask, S, L) -> int:
    """1 if the additive mask [B', 1, S, L] leaves every key past a query's diagonal
    (key > L - S + i) at <= -1e4 (so its exp() underflows to 0) and keeps some key of every row
    open, 2 if moreover every key on and below the diagonal is exactly 0 (the pure causal
    pattern), else 0.  Cached per tensor OBJECT and version (one check per forward: the decoder
    layers share the mask): the cache holds a weak reference to the mask and matches it with
    ``is``, so a new mask that the allocator places at a freed mask's address is never taken for
    it, and a cached mask's memory is freed with its last user."""
    for ent in _CAUSAL:
        if ent[0]() is mask and ent[1] == mask._version and ent[2] == S and ent[3] == L:
            return ent[4]
    i = torch.arange(S, device=mask.device)[:, None]
    j = torch.arange(L, device=mask.device)[None, :]
    above = j > (L - S) + i
    m = mask[:, 0].float()
    open_max = torch.where(above, torch.full_like(m, -float("inf")), m).amax(dim=-1)  # per row
    ok = int(bool((m[:, above] <= -1e4).all()) and bool((open_max > -1e4).all()))
    if ok and bool((m[:, ~above] == 0).all()):
        ok = 2
    _CAUSAL.append((weakref.ref(mask), mask._version, S, L, ok))
    del _CAUSAL[:-_CAUSAL_KEEP]
    return ok


def attn_prefill(q, k, v, mask, scale_div, out_dtype=torch.float32):
    """softmax(q k^T / scale_div + mask) v for a window of S query tokens: q fp32 [B, Hq, S, D]
    (after RoPE), k/v fp16 [B, Hkv, L, D] (L >= S: a cached prefix precedes the window), mask
    [B', 1, S, L] fp16/fp32 or None -> [B, S, Hq, D] (the layer's transposed layout) in out_dtype
    (fp32, or the fp32 result rounded once to fp16)."""
    if not attn_prefill_supported(q, k, mask):
        raise ValueError("attn_prefill: unsupported shapes / dtypes")
    if not (q.is_cuda and k.is_cuda and v.is_cuda):
        raise RuntimeError("qlin kernels run on gfx950 only: got a CPU tensor")
    B, Hq, S, D = q.shape
    Hkv, L = k.shape[1], k.shape[2]
    q = q.contiguous()
    k = k.contiguous()
    v = v.contiguous()
    m, mdt, mbs, causal = None, F16, 0, 0
    if mask is not None:
        # batch-broadcast masks (expand()ed views, batch stride 0) are passed as they lie
        m = mask
        if m.stride(-1) != 1 or m.stride(-2) != L or (m.shape[0] > 1 and m.stride(0) not in (0, S * L)):
            m = m.contiguous()
        mdt = _dtcode(m)
        mbs = m.stride(0) if m.shape[0] > 1 else 0
        causal = int(mask_is_causal(m, S, L))
    out = torch.empty(B, S, Hq, D, dtype=out_dtype, device=q.device)
    rc = load_library().qlin_attn_prefill(_ptr(q), _ptr(k), _ptr(v), _ptr(m), mdt, mbs, causal,
                                          _ptr(out), _dtcode(out), B, Hq, Hkv, S, L, D,
                                          float(scale_div), _stream(q))
    _check(rc, "qlin_attn_prefill")
    return out
