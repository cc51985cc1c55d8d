"""CPU-side checks: the C-ABI library loads and exports every declared symbol, argument
validation fails cleanly without a GPU, and the host mirror keeps the reference module API."""
import ctypes
import os
import re

import pytest
import torch

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "qlin_gfx950.h")
HEADERS = sorted(os.path.join(ROOT, "include", f) for f in os.listdir(os.path.join(ROOT, "include"))
                 if f.endswith(".h"))


def declared_symbols():
    syms = set()
    for h in HEADERS:  # every include/*.h
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        syms.update(re.findall(r"\b(qlin_\w+)\s*\(", src))
    return sorted(syms)


def test_header_declares_the_abi():
    syms = declared_symbols()
    for s in ("qlin_quantize", "qlin_fake_quant", "qlin_pack_f16", "qlin_dequant_f16",
              "qlin_gemv_f16", "qlin_gemm_f16", "qlin_linear_f16", "qlin_abi_version",
              "qlin_error_string", "qlin_pack_codes"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from quant import qlin
    lib = qlin.load_library()
    for s in declared_symbols():
        assert hasattr(lib, s), s
        assert s in qlin.SIGNATURES, f"binding lacks {s}"
    assert lib.qlin_abi_version() == qlin.ABI_VERSION


def test_invalid_arguments_return_einval_without_a_gpu():
    from quant import qlin
    lib = qlin.load_library()
    # every entry point validates before touching the device
    assert lib.qlin_dequant_f16(None, None, 0, 16, 64, 4, 64, None, None) == 1
    assert lib.qlin_gemv_f16(None, None, 0, None, None, None, 1, 16, 64, 4, 64, None) == 1
    assert lib.qlin_gemm_f16(None, None, 0, None, None, None, 8, 16, 64, 4, 64, None, 0, None) == 1
    assert lib.qlin_quantize(None, 0, 4, 64, 4, 64, 0, None, None, None, None, None, None, None,
                             None) == 1
    assert lib.qlin_fake_quant(None, 0, None, None, 4, 64, 4, 64, 0, None, None, None, None) == 1
    assert lib.qlin_pack_f16(None, None, None, 4, 64, 4, 64, 0, None, None, None) == 1
    p = ctypes.c_void_p(16)  # never dereferenced: the shape check fails first
    assert lib.qlin_gemv_f16(p, p, 0, p, None, p, 1, 16, 65, 4, 64, None) == 1   # K % 32
    assert lib.qlin_gemv_f16(p, p, 0, p, None, p, 17, 16, 64, 4, 64, None) == 1  # M > 16
    assert lib.qlin_gemv_f16(p, p, 0, p, None, p, 1, 16, 64, 5, 64, None) == 1   # bits
    assert lib.qlin_gemv_f16(p, p, 0, p, None, p, 1, 16, 128, 4, 96, None) == 1  # group | K
    assert lib.qlin_gemm_f16(p, p, 0, p, None, p, 8, 16, 64, 4, 48, None, 0, None) == 1  # group % 32
    assert lib.qlin_gemm_f16(p, p, 0, p, None, p, 8, 16, 64, 4, 64, None, -1, None) == 1  # ws bytes
    assert lib.qlin_linear_f16(p, p, 0, p, None, p, 8, -1, 64, 4, 64, None) == 1  # N < 0
    assert lib.qlin_dequant_f16(p, p, 0, 16, 64, 3, 128, p, None) == 1  # group > K
    ep = lib.qlin_linear_ep_f16
    assert ep(p, p, 0, p, None, None, p, 1, 16, 64, 4, 64, 1, 0, 0, None, 0, None) == 1  # residual
    assert ep(p, p, 0, p, None, None, p, 1, 24, 64, 4, 64, 2, 0, 0, None, 0, None) == 1  # N % 16
    assert ep(p, p, 0, p, None, None, p, 1, 16, 64, 4, 64, 0, 9, 0, None, 0, None) == 1  # act bits
    assert ep(p, p, 0, p, None, None, p, 100, 16, 64, 4, 64, 0, 8, 0, None, 0, None) == 1  # no ws
    assert ep(p, p, 0, p, None, None, p, 100, 16, 64, 4, 64, 0, 8, 0, p, 64, None) == 1  # short ws
    # ABI 10: the fused RMSNorm + linear takes one token row on whole k-tiles
    assert lib.qlin_rmsnorm_linear_supported(1, 16, 256, 4, 128) == 1
    assert lib.qlin_rmsnorm_linear_supported(2, 16, 256, 4, 128) == 0
    assert lib.qlin_rmsnorm_linear_supported(1, 16, 1000, 4, 40) == 0
    assert lib.qlin_rmsnorm_linear_ep_f16(p, p, 0, p, p, 1e-5, None, None, p, 1, 16, 256, 4, 128,
                                          1, None) == 1  # residual epilogue without residual
    # ABI 12: which M = 1 kernel a shape takes (without a device: the 256-CU MI355X geometry)
    assert lib.qlin_gemv_m1_route(28672, 4096, 4, 128) == 1   # gate/up: work-queue kernel
    assert lib.qlin_gemv_m1_route(6144, 4096, 3, 64) == 2     # q/k/v: fast kernel
    assert lib.qlin_gemv_m1_route(4096, 14336, 2, 32) == 3    # down: rows kernel
    assert lib.qlin_gemv_m1_route(4096, 1000, 4, 40) == -1    # invalid layout
    assert lib.qlin_pack_codes(None, 16, 64, 4, None, None) == 1
    assert lib.qlin_pack_codes(p, 16, 48, 4, p, None) == 1  # K % 32
    assert lib.qlin_pack_codes(p, 16, 64, 5, p, None) == 1  # bits
    gb = lib.qlin_gemv_batched_f16
    assert gb(None, 0, None, 0, 0, None, 0, None, 0, None, 0, 2, 1, 16, 128, 4, 128, None) == 1
    assert gb(p, 255, p, 16, 0, p, 128, None, 0, p, 16, 2, 1, 16, 128, 4, 128, None) == 1  # qw
    assert gb(p, 256, p, 16, 0, p, 127, None, 0, p, 16, 2, 1, 16, 128, 4, 128, None) == 1  # x
    assert gb(p, 256, p, 16, 0, p, 128, p, 8, p, 16, 2, 1, 16, 128, 4, 128, None) == 1  # bias
    assert gb(p, 256, p, 16, 0, p, 128, None, 0, p, 16, 70000, 1, 16, 128, 4, 128, None) == 1
    assert lib.qlin_attn_decode_splits(1, 8, 40) == 1 and lib.qlin_attn_decode_splits(1, 8, 0) == -1
    assert lib.qlin_attn_decode_splits(1, 8, 513) >= 2
    assert lib.qlin_gemm_block_cols(0, 16, 4) == -1 and lib.qlin_gemm_block_cols(16, 16, 5) == -1
    assert lib.qlin_error_string(1) == b"invalid argument"


def test_reference_module_api_is_kept():
    from quant.int_linear import QuantLinear
    from quant.int_matmul import QuantMatMul
    from quant.quantizer import UniformAffineQuantizer
    lin = torch.nn.Linear(256, 64, bias=True)
    q = QuantLinear(lin, dict(n_bits=4, group_size=128, dynamic_method="per_channel",
                              per_channel_axes=[0], lwc=True),
                    dict(n_bits=8, dynamic_method="per_token"))
    # buffers alias the original module (quant/int_linear.py:26-30)
    assert q.weight.data_ptr() == lin.weight.data_ptr()
    assert q.bias.data_ptr() == lin.bias.data_ptr()
    for a in ("in_features", "out_features", "weight_quantizer", "act_quantizer",
              "use_weight_quant", "use_act_quant", "use_temporary_parameter", "fwd_func",
              "fwd_kwargs", "disable_input_quant"):
        assert hasattr(q, a), a
    q.set_quant_state(weight_quant=True, act_quant=True)
    assert q.use_weight_quant and q.use_act_quant
    wq = q.weight_quantizer
    assert isinstance(wq, UniformAffineQuantizer)
    assert (wq.qmin, wq.qmax) == (0, 15)
    assert wq.upbound_factor.shape == (64 * 2, 1) and float(wq.upbound_factor[0]) == 4.0
    wq.change_n_bits(3)
    assert wq.qmax == 7
    sym = UniformAffineQuantizer(n_bits=4, disable_zero_point=True)
    assert (sym.qmin, sym.qmax) == (-8, 7)
    with pytest.raises(AssertionError):
        UniformAffineQuantizer(n_bits=17)
    # dense (unquantized) forward is the reference's F.linear
    x = torch.randn(2, 256)
    q.set_quant_state(False, False)
    torch.testing.assert_close(q(x), torch.nn.functional.linear(x, lin.weight, lin.bias))
    mm = QuantMatMul(matmul_func=torch.matmul)
    a, b = torch.randn(2, 3, 4), torch.randn(2, 4, 5)
    torch.testing.assert_close(mm(mm.quant_x1(a), mm.quant_x2(b)), a @ b)


def test_quantizer_bypass_and_errors_match_reference():
    from quant.quantizer import UniformAffineQuantizer
    x = torch.randn(4, 64)
    assert UniformAffineQuantizer(n_bits=16)(x) is x            # quantizer.py:119-120
    q = UniformAffineQuantizer(n_bits=4)
    q.enable = False
    assert q(x) is x
    with pytest.raises(NotImplementedError):                    # quantizer.py:124-127
        UniformAffineQuantizer(n_bits=4, dynamic_method="per_cluster")(x)


def test_no_cpu_fallback():
    """The product path refuses CPU tensors instead of silently computing on the host."""
    from quant.quantizer import UniformAffineQuantizer
    q = UniformAffineQuantizer(n_bits=4, group_size=32, dynamic_method="per_channel")
    with pytest.raises(RuntimeError, match="gfx950"):
        q(torch.randn(4, 64).half())
    from quant import qlin
    qw = torch.zeros(2, *qlin.packed_shape(16, 128, 4), dtype=torch.int32)
    qsz = torch.zeros(2, *qlin.sz_shape(16, 128, 128), dtype=torch.int32)
    with pytest.raises(RuntimeError, match="gfx950"):
        qlin.gemv_batched(torch.zeros(2, 1, 128).half(), qw, qsz, None, 16, 128, 4, 128)


def test_mask_is_causal_cache_keys_on_the_tensor_object():
    """A padded mask built after a causal mask of the same shape was freed (the allocator often
    hands it the same address, and both start at _version 0) must be classified afresh."""
    from quant import qlin
    S = L = 8
    minv = torch.finfo(torch.float16).min

    def causal():
        return torch.triu(torch.full((S, L), minv), 1).half()[None, None]

    m = causal()
    assert qlin.mask_is_causal(m, S, L) == 2
    assert qlin.mask_is_causal(m, S, L) == 2  # cached
    storage = m.untyped_storage()
    del m
    padded = causal()
    padded[..., 1:, 0] = minv  # left padding: key 0 masked for query rows 1.. (row 0 keeps it)
    assert qlin.mask_is_causal(padded, S, L) == 1
    # the same object again after an in-place edit (version bump) is re-checked too
    padded[..., 3, 5] = 0  # opens a key past the diagonal
    assert qlin.mask_is_causal(padded, S, L) == 0
    # a fresh tensor written into the freed storage (same address, _version 0)
    reused = torch.empty(0, dtype=torch.float16).set_(storage).view(1, 1, S, L)
    reused.fill_(0)
    assert qlin.mask_is_causal(reused, S, L) == 0


def test_product_path_never_imports_the_oracle():
    pkg = os.path.join(ROOT, "llama3-quantization_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in src.replace("oracle/", ""), f


def test_integration_stub_matches_the_header_abi():
    """The reference-side binding in INTEGRATION.md asserts the ABI version the header declares."""
    hdr = open(HEADER).read()
    abi = int(re.search(r"#define QLIN_ABI_VERSION (\d+)", hdr).group(1))
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    stubs = re.findall(r"qlin_abi_version\(\) == (\d+)", doc)
    assert stubs and all(int(v) == abi for v in stubs), (stubs, abi)


def test_mask_cache_does_not_keep_masks_alive():
    import gc
    import weakref
    from quant import qlin
    m = torch.triu(torch.full((4, 4), -6e4), 1).half()[None, None]
    qlin.mask_is_causal(m, 4, 4)
    r = weakref.ref(m)
    del m
    gc.collect()
    assert r() is None


def test_bench_graph_steps_divide_the_timed_steps():
    """bench.py captures G steps per graph and replays steps / G graphs: G must divide the step
    count (the timed region is exactly --steps steps) and stay <= 10."""
    import importlib
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    bench = importlib.import_module("bench")
    for n, g in ((50, 10), (5, 5), (7, 7), (13, 1), (12, 6), (1, 1), (100, 10)):
        assert bench.graph_steps(n) == g
        assert n % bench.graph_steps(n) == 0
