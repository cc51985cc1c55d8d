"""Dev reference point: dense fp16 torch.matmul (hipBLASLt) vs qlin GEMM at the bench shapes."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))
import torch
from quant import qlin
dev = torch.device("cuda:0")
SHAPES = [tuple(map(int, t.split("x"))) for t in os.environ.get("SHAPES", "4096x4096").split(",")]
MS = [int(m) for m in os.environ.get("MS", "256,512,1024,2048,8192,65536").split(",")]


def timeit(fn, reps):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


for (N, K) in SHAPES:
  w = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.02
  o = qlin.quantize(w, 4, 128, 0, want_xdq=False, want_params=False, pack=True)
  wdq = qlin.dequant(o["qweight"], o["qsz"], N, K, 4, 128, o["flags"])
  for M in MS:
      x = torch.randn(M, K, device=dev, dtype=torch.float16)
      reps = max(3, int(2e9 / (2 * M * N * K) * 20))
      t_blas = timeit(lambda: torch.matmul(x, wdq.t()), reps)
      t_q = timeit(lambda: qlin.gemm(x, o["qweight"], o["qsz"], None, N, K, 4, 128, o["flags"]), reps)
      t_dq = timeit(lambda: qlin.dequant(o["qweight"], o["qsz"], N, K, 4, 128, o["flags"]), 20)
      f = 2 * M * N * K
      print(f"N={N} K={K} M={M:6d}: hipBLASLt fp16 {f/t_blas/1e12:7.1f} TF/s ({t_blas*1e6:8.1f} us)  "
            f"qlin_gemm {f/t_q/1e12:7.1f} TF/s ({t_q*1e6:8.1f} us)  dequant {t_dq*1e6:6.1f} us", flush=True)
