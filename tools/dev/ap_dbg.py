"""Dev: where does a prefill-attention variant differ from float64 (row / head / d pattern)."""
import ctypes, math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
from test_gpu_attn import _ref, _causal_mask
P, L64 = ctypes.c_void_p, ctypes.c_int64
B, Hq, Hkv, S, L = 1, 32, 8, int(os.environ.get("S", "2048")), int(os.environ.get("S", "2048"))
g = torch.Generator(device="cuda").manual_seed(B * 7919 + S * 31 + L)
q = torch.randn(B, Hq, S, 128, device="cuda", generator=g) * 0.5
k = torch.randn(B, Hkv, L, 128, device="cuda", generator=g).half()
v = torch.randn(B, Hkv, L, 128, device="cuda", generator=g).half()
ref = _ref(q, k, v, _causal_mask(B, S, L)).transpose(1, 2)[0]  # [S, Hq, D]
outs = {}
for name in sys.argv[1:]:
    lib = ctypes.CDLL(os.path.join(ROOT, "tools/dev", name))
    out = torch.empty(B, S, Hq, 128, device="cuda")
    rc = lib.qlin_attn_prefill(P(q.data_ptr()), P(k.data_ptr()), P(v.data_ptr()), None, 1, L64(0), 2,
                               P(out.data_ptr()), 1, L64(B), Hq, Hkv, L64(S), L64(L), 128,
                               ctypes.c_float(math.sqrt(128)), P(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    err = (out[0].double() - ref).abs()
    per_row = err.amax(dim=(1, 2))
    top = torch.topk(err.flatten(), 8)
    print(name, "rows with err > 1e-6:", (per_row > 1e-6).nonzero().flatten()[:20].tolist())
    for val, idx in zip(top.values.tolist(), top.indices.tolist()):
        r, rem = divmod(idx, Hq * 128)
        h, d = divmod(rem, 128)
        print(f"   err {val:.3g} row {r} head {h} d {d} ref {ref[r, h, d].item():.6g} got {out[0, r, h, d].item():.6g}"
              f"  row-head max err {err[r, h].max().item():.3g} n>1e-6 in row-head {(err[r, h] > 1e-6).sum().item()}")

# which key explains row 38 / head 31's error (single-key weight perturbation fit)
r, h = int(os.environ.get("ROW", "38")), int(os.environ.get("HEAD", "31"))
hk = h // (Hq // Hkv)
qd = q[0, h, r].double()
kd = k[0, hk, :r + 1].double()
vd = v[0, hk, :r + 1].double()
s = kd @ qd / math.sqrt(128)
p = torch.softmax(s, 0)
o_ref = p @ vd
e = out[0, r, h].double() - o_ref
best = []
for j in range(r + 1):
    dvec = (vd[j] - o_ref) * p[j]  # d o / d (log p_j) direction
    t = (e @ dvec) / (dvec @ dvec)
    resid = (e - t * dvec).norm().item()
    best.append((resid, j, t.item()))
best.sort()
print("err norm", e.norm().item(), "best single-key fits (resid, key, dlogp):", best[:4])
print("scores (nat) of those keys:", [round(s[j].item(), 5) for _, j, _ in best[:4]], "max", s.max().item())
# also the masked key r+1 (if it leaked in)
if r + 1 < L:
    kx = k[0, hk, r + 1].double(); vx = v[0, hk, r + 1].double()
    sx = (kx @ qd) / math.sqrt(128)
    print("next (masked) key score", sx.item())
