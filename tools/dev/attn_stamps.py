"""Dev: stamped timeline of the decode attention launch (libattn_st.so, ATTN_STAMP build):
attn_decode_rope, LLaMA3-8B shapes, batch 1, cold caches (after a 512 MiB write).
Per stage: median over blocks of (stamp - earliest block start) in us, over the last of R runs.
Usage: QLIN_LIBRARY=tools/dev/libattn_st.so python tools/dev/attn_stamps.py [L ...]"""
import ctypes
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch  # noqa: E402
from quant import qlin  # noqa: E402
from models.int_llama_layer import LlamaRotaryEmbedding437  # noqa: E402

lib = qlin.load_library()
lib.qlin_dev_attn_stamps.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda:0")
Hq, Hkv, D = 32, 8, 128
NAMES = ["start", "q", "scores", "pv", "counted", "merge_in", "out", "softmax"]
ONAMES = []


def summarize(st, nblk, na, names_a, names_o):
    t = st[:nblk].double()
    t0 = t[:, 0][t[:, 0] > 0].min()
    rel = (t - t0) / 100.0  # 100 MHz -> us
    rows = {}
    for i, nm in enumerate(names_a):
        v = rel[:na, i][t[:na, i] > 0]
        if v.numel():
            rows["a." + nm] = (round(v.median().item(), 2), round(v.max().item(), 2), v.numel())
    for i, nm in enumerate(names_o):
        v = rel[na:nblk, i][t[na:nblk, i] > 0]
        if v.numel():
            rows["o." + nm] = (round(v.median().item(), 2), round(v.max().item(), 2), v.numel())
    return rows


for L in [int(a) for a in sys.argv[1:]] or [513, 4096]:
    kv0 = L - 1
    g = torch.Generator(device=dev).manual_seed(L)
    qkv = (torch.randn(1, 1, (Hq + 2 * Hkv) * D, device=dev, generator=g)).half()
    q, k, v = torch.split(qkv, [Hq * D, Hkv * D, Hkv * D], dim=-1)
    rot = LlamaRotaryEmbedding437(D, 8192, 500000.0, device=dev).half()
    cos, sin = rot.cos_cached.float().contiguous(), rot.sin_cached.float().contiguous()
    pos = torch.full((1, 1), kv0, device=dev, dtype=torch.int64)
    kc = torch.randn(1, Hkv, L + 64, D, device=dev, generator=g).half()
    vc = torch.randn(1, Hkv, L + 64, D, device=dev, generator=g).half()
    st = torch.zeros(4096, 8, dtype=torch.int64, device=dev)
    lib.qlin_dev_attn_stamps(ctypes.c_void_p(st.data_ptr()))
    S = lib.qlin_attn_decode_splits(1, Hkv, L)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    for name in ("rope",):
        for _ in range(5):
            flush.zero_()  # K/V and weights out of the MALL
            st.zero_()
            qlin.attn_decode_rope(q, k, v, cos, sin, pos, Hq, Hkv, D, kc, vc, kv0, None,
                                  math.sqrt(D), out_dtype=torch.float16)
            torch.cuda.synchronize()
        na = Hkv * S
        nblk = na
        rows = summarize(st.cpu(), nblk, na, NAMES, ONAMES)
        print(f"L={L} S={S} {name}: stage (median us, max us, blocks) {rows}", flush=True)
    lib.qlin_dev_attn_stamps(None)
