"""Dev: qlin_attn_prefill timing (LLaMA3-8B window: B=1, Hq=32, Hkv=8, S=L=2048, causal) against
the reference's materialised fp32 attention (repeat_kv, matmul, scores pass, softmax, matmul)."""
import math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
sys.path.insert(0, ROOT)
import torch
from quant import qlin
from models.quant_llama import causal_mask

dev = torch.device("cuda:0")
B, Hq, Hkv, S = 1, 32, 8, int(os.environ.get("S", "2048"))
g = torch.Generator(device=dev).manual_seed(0)
q = torch.randn(B, Hq, S, 128, device=dev, generator=g)
k = torch.randn(B, Hkv, S, 128, device=dev, generator=g).half()
v = torch.randn(B, Hkv, S, 128, device=dev, generator=g).half()
mask = causal_mask(B, S, torch.float16, dev)


def ref():
    kk = k.repeat_interleave(Hq // Hkv, dim=1).float()
    vv = v.repeat_interleave(Hq // Hkv, dim=1).float()
    w = q @ kk.transpose(2, 3)
    w = qlin.attn_scores_(w, mask, math.sqrt(128))
    w = torch.softmax(w, dim=-1, dtype=torch.float32)
    return (w @ vv).transpose(1, 2).half()


def timeit(fn, reps=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


flops = 4 * B * Hq * S * S * 128 / 2  # causal half of QK^T + PV
t_k = timeit(lambda: qlin.attn_prefill(q, k, v, mask, math.sqrt(128), out_dtype=torch.float16))
t_r = timeit(ref)
o = qlin.attn_prefill(q, k, v, mask, math.sqrt(128))
r = ref().float()
err = ((o - r).abs().max() / r.abs().max()).item()
print(f"S={S}: kernel {t_k:.3f} ms ({flops / t_k / 1e9:.1f} TFLOP/s causal), reference path "
      f"{t_r:.3f} ms, max rel diff vs the fp16 reference output {err:.2e}", flush=True)
