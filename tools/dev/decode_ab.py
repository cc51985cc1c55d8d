"""Dev: the bench's decode-layer line (bench.py decode_layer_bench: 8 distinct LLaMA3-8B layers,
packed + fused, KV 513, graph-replayed) with the library named by QLIN_LIBRARY (a dev build may
lack newer introspection symbols: those are dropped from the binding).  Prints us per layer.
Run it once per library in separate processes, interleaved, for an A/B on one box."""
import os
import sys
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "llama3-quantization_amd")]
import ctypes  # noqa: E402
import torch  # noqa: E402
from quant import qlin  # noqa: E402

lib = ctypes.CDLL(os.environ["QLIN_LIBRARY"])
for name in list(qlin.SIGNATURES):
    if not hasattr(lib, name):
        del qlin.SIGNATURES[name]
import bench  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
args = SimpleNamespace(decode_layers=8, decode_kv=512, steps=int(os.environ.get("STEPS", 60)),
                       warmup=10, ramp_s=0.3)


def timed(run, steps, warmup):
    import time
    t = time.perf_counter()
    while time.perf_counter() - t < args.ramp_s:
        run()
        torch.cuda.synchronize()
    for _ in range(warmup):
        run()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(steps):
            run()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 1e3)
    return best, 0.0


out = bench.decode_layer_bench(args, dev, timed)
print(f"{os.path.basename(os.environ['QLIN_LIBRARY'])}: decode layer {out['us_per_layer']} us", flush=True)
