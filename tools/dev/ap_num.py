"""Dev: prefill-attention numerics variants (libap<EXP2>_<LAZY>.so) vs float64 on the S = 2048 causal
case of tests/test_gpu_attn.py, plus timing."""
import ctypes, math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
from test_gpu_attn import _ref, _causal_mask
P, L64, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
for B, Hq, Hkv, S, L in [(1, 32, 8, 2048, 2048), (1, 32, 8, 257, 257)]:
    g = torch.Generator(device="cuda").manual_seed(B * 7919 + S * 31 + L)
    q = torch.randn(B, Hq, S, 128, device="cuda", generator=g) * 0.5
    k = torch.randn(B, Hkv, L, 128, device="cuda", generator=g).half()
    v = torch.randn(B, Hkv, L, 128, device="cuda", generator=g).half()
    ref = _ref(q, k, v, _causal_mask(B, S, L)).transpose(1, 2)
    for name in sys.argv[1:]:
        lib = ctypes.CDLL(os.path.join(ROOT, "tools/dev", name))
        out = torch.empty(B, S, Hq, 128, device="cuda")
        def f():
            rc = lib.qlin_attn_prefill(P(q.data_ptr()), P(k.data_ptr()), P(v.data_ptr()), None, 1, L64(0), 2,
                                       P(out.data_ptr()), 1, L64(B), Hq, Hkv, L64(S), L64(L), 128,
                                       ctypes.c_float(math.sqrt(128)), P(torch.cuda.current_stream().cuda_stream))
            assert rc == 0
        f(); torch.cuda.synchronize()
        err = (out.double() - ref).abs()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(10): f()
        e1.record(); torch.cuda.synchronize()
        i = int(err.argmax())
        print(f"S={S} {name}: max err {err.max().item():.3g} (tol {1e-5*max(1,ref.abs().max().item()):.3g}) "
              f"at flat {i}, mean err {err.mean().item():.3g}, {e0.elapsed_time(e1)/10:.3f} ms", flush=True)
