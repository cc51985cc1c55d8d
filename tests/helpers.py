"""Shared test helpers (test infrastructure)."""
import numpy as np
import torch


def t(a, dev="cuda", dtype=None):
    x = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        x = x.to(dtype)
    return x.to(dev)


def n(x):
    return x.detach().cpu().numpy()


def bit_equal(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    return np.array_equal(a.view(np.uint8), b.view(np.uint8)) or np.array_equal(a, b, equal_nan=True)


def assert_close_to_ref(y, ref, rtol=2e-3, what=""):
    """fp16-output GEMM tolerance: |y - ref| <= rtol * (|ref| + max|ref|/16), ref in float64.

    The kernels accumulate in fp32 and round the result once to fp16 (rel. 2^-11 = 4.9e-4), so
    2e-3 leaves 4x headroom for the accumulation-order difference."""
    y = np.asarray(y, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert y.shape == ref.shape, (y.shape, ref.shape)
    scale = np.abs(ref).max() if ref.size else 0.0
    err = np.abs(y - ref)
    bound = rtol * (np.abs(ref) + scale / 16.0) + 1e-6
    bad = err > bound
    assert not bad.any(), (f"{what}: {bad.sum()} / {bad.size} outside tolerance; "
                           f"max err {err.max():.3e} (max|ref| {scale:.3e})")


def rand_weight(N, K, seed, std=0.02):
    rs = np.random.RandomState(seed)
    return (rs.randn(N, K) * std).astype(np.float16)


def rand_x(M, K, seed):
    rs = np.random.RandomState(seed)
    return rs.randn(M, K).astype(np.float16)
