"""Dev (round 6): where the fused q/k/v + attention launch spends its time.  LLaMA3-8B shapes, int4
g128, KV 513, a ring of R distinct weight sets and caches, graph-replayed, us per step:
  two      rmsnorm_linear_ep (q/k/v) + attn_decode_rope (the two launches)
  qkv      rmsnorm_linear_ep alone;  attn   attn_decode_rope alone
  fused    qkv_attn_decode
  fused/dbg=N  QLIN_QKV_ATTN_DBG ablations (wrong results): 1 consumers exit (producers alone),
           2 consumers skip the wait, 6 producers exit + no wait (consumers alone)"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch  # noqa: E402

from quant import qlin  # noqa: E402

dev = torch.device("cuda:0")
H, HQ, HKV, D, KV = 4096, 32, 8, 128, 512
N = (HQ + 2 * HKV) * D
R = int(os.environ.get("RING", "8"))


def timed(fn, reps=20):
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(5):
        gr.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(reps):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


from models.int_llama_layer import LlamaRotaryEmbedding437  # noqa: E402
rot = LlamaRotaryEmbedding437(D, 8192, 500000.0, device="cuda").half()
cos, sin = rot.cos_cached.float().contiguous(), rot.sin_cached.float().contiguous()
g = torch.Generator(device=dev).manual_seed(0)
sets = []
for i in range(R):
    w = (torch.randn(N, H, device=dev, generator=g) * 0.02).half()
    o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
    kc = torch.randn(1, HKV, 1024, D, device=dev, generator=g).half()
    vc = torch.randn(1, HKV, 1024, D, device=dev, generator=g).half()
    sets.append((o["qweight"], o["qsz"], o["flags"], kc, vc))
x = (torch.randn(1, 1, H, device=dev, generator=g)).half()
nw = torch.ones(H, device=dev, dtype=torch.float16)
pos = torch.tensor([[KV]], device=dev)


def two(i, parts=("qkv", "attn")):
    qw, qsz, fl, kc, vc = sets[i]
    y = qlin.rmsnorm_linear_ep(x, nw, 1e-5, qw, qsz, None, N, H, 4, 128, fl) if "qkv" in parts \
        else qkv_static[i]
    if "attn" in parts:
        q, k, v = torch.split(y, [HQ * D, HKV * D, HKV * D], dim=-1)
        qlin.attn_decode_rope(q, k, v, cos, sin, pos, HQ, HKV, D, kc, vc, KV, None, math.sqrt(D),
                              out_dtype=torch.float16)


def fused(i):
    qw, qsz, fl, kc, vc = sets[i]
    qlin.qkv_attn_decode(x, nw, 1e-5, qw, qsz, fl, 4, 128, cos, sin, pos, HQ, HKV, D, kc, vc,
                         kv0=KV)


qkv_static = [qlin.rmsnorm_linear_ep(x, nw, 1e-5, s_[0], s_[1], None, N, H, 4, 128, s_[2])
              for s_ in sets]
res = {}
res["two"] = timed(lambda: [two(i) for i in range(R)]) / R
res["qkv"] = timed(lambda: [two(i, ("qkv",)) for i in range(R)]) / R
res["attn"] = timed(lambda: [two(i, ("attn",)) for i in range(R)]) / R
for dbg in ("0", "1", "2", "6"):
    os.environ["QLIN_QKV_ATTN_DBG"] = dbg
    res[f"fused/dbg={dbg}"] = timed(lambda: [fused(i) for i in range(R)]) / R
os.environ.pop("QLIN_QKV_ATTN_DBG")
for sl in ("1", "4", "16"):
    for rmw in ("0", "1"):
        os.environ["QLIN_QKV_POLL_SLEEPS"], os.environ["QLIN_QKV_POLL_RMW"] = sl, rmw
        res[f"fused/sleeps={sl},rmw={rmw}"] = timed(lambda: [fused(i) for i in range(R)]) / R
print({k: round(v, 2) for k, v in res.items()}, flush=True)
