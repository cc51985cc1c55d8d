"""Dev: the 32x32x16 GEMM lab kernel (tools/dev/gemm32_lab.hip) vs the product GEMM: agreement
with float64 on ragged shapes / every bit width, then timings at the LLaMA shapes."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin
dev = torch.device("cuda:0")
lab = ctypes.CDLL(os.path.join(ROOT, "tools/dev/libgemm32.so"))
P = ctypes.c_void_p


def timeit(fn, reps):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def pack(N, K, bits, group, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    w = torch.randn(N, K, device=dev, dtype=torch.float16, generator=g) * 0.02
    o = qlin.quantize(w, bits, group, 0, want_xdq=False, want_params=False, pack=True)
    return o


def run32(o, x, y, M, N, K, bits, group, bn):
    st = P(torch.cuda.current_stream().cuda_stream)
    return lab.lab_gemm32(P(o["qweight"].data_ptr()), P(o["qsz"].data_ptr()), P(x.data_ptr()),
                          P(y.data_ptr()), ctypes.c_int64(M), N, K, bits, group, bn, st)


if os.environ.get("CHECK", "1") == "1":
    for (M, N, K, bits, group) in [(300, 1000, 4096, 4, 128), (2048, 4096, 4096, 4, 128),
                                   (129, 520, 4160, 4, 64), (256, 512, 2048, 4, 32),
                                   (200, 4096, 4096, 3, 64), (200, 4096, 4096, 2, 64),
                                   (512, 6144, 4096, 4, 256)]:
        o = pack(N, K, bits, group)
        wdq = qlin.dequant(o["qweight"], o["qsz"], N, K, bits, group, o["flags"])
        x = torch.randn(M, K, device=dev, dtype=torch.float16)
        ref = (x.double() @ wdq.double().t())
        prod = qlin.gemm(x, o["qweight"], o["qsz"], None, N, K, bits, group, o["flags"])
        for bn in (256, 512):
            y = torch.full((M, N), float("nan"), device=dev, dtype=torch.float16)
            assert run32(o, x, y, M, N, K, bits, group, bn) == 0
            torch.cuda.synchronize()
            err = (y.double() - ref).abs()
            tol = 2e-3 * (ref.abs() + ref.abs().max() / 16)
            ok = bool((err <= tol).all())
            dp = (y.float() - prod.float()).abs().max().item()
            ne = (y != prod).float().mean().item()
            print(f"M={M} N={N} K={K} b{bits} g{group} bn={bn}: ok={ok} max err {err.max().item():.3g} "
                  f"| vs product max {dp:.3g}, {ne*100:.2f}% elements differ", flush=True)
            assert ok

SHAPES = [tuple(map(int, t.split("x"))) for t in os.environ.get(
    "SHAPES", "4096x4096,6144x4096,28672x4096,4096x14336").split(",")]
MS = [int(m) for m in os.environ.get("MS", "2048,8192,65536").split(",")]
VARIANTS = [tuple(map(int, t.split("/"))) for t in os.environ.get(
    "VARIANTS", "0/256,0/512,1/512,2/512").split(",")]
for (N, K) in SHAPES:
    o = pack(N, K, 4, 128)
    for M in MS:
        x = torch.randn(M, K, device=dev, dtype=torch.float16)
        y = torch.empty(M, N, device=dev, dtype=torch.float16)
        f = 2 * M * N * K
        reps = max(3, int(2e9 / f * 20))
        arms = [("product", lambda: qlin.gemm(x, o["qweight"], o["qsz"], None, N, K, 4, 128, o["flags"]))]
        for v, bn in VARIANTS:
            def fn(v=v, bn=bn):
                lab.lab_gemm32_variant(v)
                run32(o, x, y, M, N, K, 4, 128, bn)
            arms.append((f"v{v}/{bn}", fn))
        best = [1e9] * len(arms)
        for _ in range(int(os.environ.get("ROUNDS", "3"))):
            for i, (_, fn) in enumerate(arms):
                best[i] = min(best[i], timeit(fn, reps))
        print(f"N={N} K={K} M={M}: " + " | ".join(f"{nm} {f/t/1e12:5.0f} ({t*1e6:7.1f} us)"
                                                   for (nm, _), t in zip(arms, best)), flush=True)
