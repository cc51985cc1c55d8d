#!/usr/bin/env python3
"""Benchmark of the quantized-linear hot path on MI355X (BASELINE.json metric).

Default workload (BASELINE.json configs[1]): LLaMA3-8B-shaped int4 group_size=128 dequant-GEMV at
batch 1 — y[1, 4096] = x[1, 4096] @ W_dq[4096, 4096]^T through the fused gfx950 kernels, over a
ring of R distinct synthetic matrices (W ~ N(0, 0.02^2), RTN int4 g128 by the build's own HIP
quantizer; R >= 64 so 563 MB of codes cannot be served by the 256 MB Infinity Cache), each with
its own activation row.  One step = one pass over the ring: R products.

Two ways to run that step, both timed in every GEMV run (the headline `--mode`, the other under
`other_mode`):
  batched  (default) the whole ring as ONE strided-batch launch (qlin_gemv_batched_f16: the
           streaming kernel, every output one MFMA chain in k order) — the kernel's HBM
           throughput when the kernel boundary is paid once per ring;
  launches one dependent qlin_gemv_f16 launch per matrix (graph-replayed) — the per-launch cost a
           decode chain of dependent GEMVs pays (boundary + wave ramp of an 8.8 MB launch).

Prints ONE JSON line (rank 0).  value = whole-job dequant-matmul TFLOP/s (sum over ranks: every
rank streams its own ring, no collective in the data path -> weak scaling).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME] [--ring R]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "llama3-quantization_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)
MFMA_F16_PEAK_TFS = 2500.0  # dense fp16/bf16 MFMA spec (no sparsity)

WORKLOADS = {
    # name: (M, N, K, bits, group, ring, kernel, note)
    "gemv_int4_g128": (1, 4096, 4096, 4, 128, 64, "gemv",
                       "LLaMA3-8B int4 g128 dequant-GEMV batch=1 (configs[1]), 4096x4096"),
    "gemv_int3_g64": (1, 4096, 4096, 3, 64, 64, "gemv", "int3 g64 sub-byte GEMV (configs[3])"),
    "gemv_int2_g64": (1, 4096, 4096, 2, 64, 96, "gemv", "int2 g64 sub-byte GEMV (configs[3])"),
    "gemv_int3_g64_hqq": (1, 4096, 4096, 3, 64, 64, "gemv",
                          "int3 g64 GEMV, HQQ fp16 zero points (QLIN_FLOAT_ZERO, configs[3])"),
    "gemv_int2_g64_hqq": (1, 4096, 4096, 2, 64, 96, "gemv",
                          "int2 g64 GEMV, HQQ fp16 zero points (QLIN_FLOAT_ZERO, configs[3])"),
    "gemm_int4_g64_hqq_m2048": (2048, 4096, 4096, 4, 64, 4, "gemm",
                                "int4 g64 HQQ fp16 zero points, one 2048-token window"),
    "gemm_int4_g128_m32": (32, 4096, 4096, 4, 128, 64, "linear",
                           "int4 g128, 32 tokens (qlin_linear_f16 dispatch: GEMV kernel x2)"),
    "gemm_int4_g128_m2048": (2048, 4096, 4096, 4, 128, 4, "gemm",
                             "int4 g128, one 2048-token PPL window"),
    "gemm_int4_g128_m65536": (65536, 4096, 4096, 4, 128, 1, "gemm",
                              "int4 g128 batch 32 x seq 2048 (configs[2], MFMA path)"),
    # QuantLinear with act_quantizer on (quant/int_linear.py:59-60), per-token
    # 8-bit fake-quant of x (W4A8) through qlin_linear_ep_f16 act_bits = 8
    "gemv_int4_g128_a8": (1, 4096, 4096, 4, 128, 64, "linear_aq",
                          "W4A8: per-token act fake-quant fused into the GEMV blocks (row f3)"),
    "gemm_int4_g128_a8_m2048": (2048, 4096, 4096, 4, 128, 4, "linear_aq",
                                "W4A8, one 2048-token window: act quantizer kernel + MFMA GEMM (row f3)"),
}


PIPE_WORKLOAD = "pipeline_llama3_8b_int4_g128"


def algo_bytes(M, N, K, bits, group, zero_bytes=1):
    """Algorithmic bytes of one launch, SURVEY.md §8(d) / BASELINE.md §2:
    2MK + N*K*bits/8 + N*(K/g)*(2 + zb) + 2MN with zb = 1 (fp16 scale + int8 zero per group).
    The qsz layout actually stores an int16 zero (4 B per group, zero_bytes=2): reported as
    bytes_read_per_launch beside it."""
    return 2 * M * K + N * K * bits // 8 + N * (K // group) * (2 + zero_bytes) + 2 * M * N


def _pmc_traffic(workload):
    """HBM bytes per launch from the newest committed PMC pass for this workload
    (profiles/*_<workload>_pmc.json, written by tools/pmc_traffic.py from rocprofv3 --pmc
    FETCH_SIZE with the gfx950 x2 correction), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{workload}_pmc.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    d["file"] = os.path.relpath(files[-1], ROOT)
    return d


def _attach_traffic(roof, pmc, algo, launch_products=None):
    """roofline.traffic from a committed PMC pass, or null: a pass that reports fewer HBM bytes
    than the launch's algorithmic bytes (every algorithmic byte is read at least once) missed
    dispatches and is not published; traffic_ratio = traffic / algorithmic.
    A pass records the products one profiled launch computed (`products_per_launch`, the bench
    ring); a line whose launches hold another number of products gets the pass's bytes per product
    times its own (a strided batch streams each product's bytes once), and says so."""
    if pmc is None:
        return
    t = pmc["fetch_bytes_per_launch"]
    roof["traffic_source"] = pmc["file"]
    if launch_products is not None:
        p = pmc.get("products_per_launch")
        if p is None:
            roof["traffic"] = None
            roof["traffic_rejected"] = f"{pmc['file']}: launch size of the pass not recorded"
            return
        if p != launch_products:
            t = t / p * launch_products
            roof["traffic_scaled"] = (f"per product from a pass at {p} products per launch, x "
                                      f"{launch_products}")
    if t < algo:
        roof["traffic"] = None
        roof["traffic_rejected"] = (f"{pmc['file']}: {round(t)} B < {algo} algorithmic B per "
                                    "launch (incomplete PMC pass)")
        return
    roof["traffic"] = round(t)
    roof["traffic_ratio"] = round(t / algo, 4)


def parse():
    ap = argparse.ArgumentParser()
    # default: the launcher's WORLD_SIZE (torchrun without --gpus), else 1
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="gemv_int4_g128",
                    choices=sorted(WORKLOADS) + [PIPE_WORKLOAD])
    ap.add_argument("--ring", type=int, default=None)
    ap.add_argument("--split", action="store_true",
                    help="strong scaling: every rank streams rows [r*N/P, (r+1)*N/P) of the SAME "
                         "ring (output-feature sharding, SURVEY.md §8(e)); default: weak scaling, "
                         "an independent ring per rank")
    ap.add_argument("--mode", choices=("batched", "launches"), default="batched",
                    help="GEMV workloads: 'batched' = the whole ring as one strided-batch launch "
                         "(qlin_gemv_batched_f16); 'launches' = one dependent launch per matrix "
                         "(the decode chain's per-launch cost); the other mode is timed too and "
                         "reported beside it")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--ramp-s", type=float, default=0.3,
                    help="untimed seconds of runs before the warmup steps (GPU clock ramp)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-other-mode", action="store_true",
                    help="skip timing the other GEMV mode (batched / launches)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-decode-layer", action="store_true",
                    help="skip the decode-layer line (configs[1] inside the model, DESIGN.md §5)")
    ap.add_argument("--decode-layers", type=int, default=8)
    ap.add_argument("--decode-kv", type=int, default=512)
    ap.add_argument("--pipeline", choices=("auto", "on", "off"), default="auto",
                    help="the configs[4] pipeline leg (32 LLaMA3-8B layers as N stages, RCCL "
                         "send / recv): auto = with N > 1 ranks or --workload "
                         f"{PIPE_WORKLOAD}")
    ap.add_argument("--pipe-layers", type=int, default=32)
    ap.add_argument("--pipe-tokens", type=int, default=2048, help="tokens per PPL window")
    ap.add_argument("--pipe-windows", type=int, default=0,
                    help="windows in flight per timed pass (default: max(4, 2 x ranks))")
    ap.add_argument("--pipe-decode", type=int, default=16,
                    help="greedy decode steps per sequence (one sequence per stage), graphs=True")
    ap.add_argument("--pipe-no-check", action="store_true",
                    help="skip the one-process reference run (NLL / token bit-identity)")
    return ap.parse_args()


def _host_cpus():
    """(CPUs this process may run on, physical cores among them, CPU model) from the affinity
    mask and /proc/cpuinfo (SMT siblings share a (physical id, core id) pair)."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        cpus = list(range(os.cpu_count() or 1))
    model, cores, cur = None, set(), {}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f.read().split("\n") + [""]:
                if not line.strip():
                    if cur.get("processor") in cpus:
                        cores.add((cur.get("physical id", 0), cur.get("core id", cur["processor"])))
                    cur = {}
                    continue
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k in ("processor", "physical id", "core id"):
                    cur[k] = int(v)
                elif k == "model name" and model is None:
                    model = v
    except OSError:
        pass
    return cpus, (len(cores) or len(cpus)), model


def cpu_baseline(M, N, K, bits, group, seconds):
    """The reference's fake-quant path on the host cores, restated in torch
    (oracle/torch_ref.py, pinned bit-exactly to the reference's golden W_dq), swept over torch
    thread counts {1, 8, 16, 32, 64, 128, all} and dtypes {fp16, fp32}:
      mode (ii) — what the reference runs at eval (weight == W_dq; quant/int_linear.py:62):
               F.linear(x, W_dq) over a bounded sample of distinct pre-dequantized matrices;
               TFLOP/s of the best of 3 timed runs per (threads, dtype);
      mode (i)  — quantize every call (use_weight_quant=True, quant/quantizer.py:118-159 then
               F.linear, fp16): median ms per call, per thread count.
    value = the reference's op as it runs (fp16 F.linear) at its best thread count."""
    import statistics
    import torch
    import torch.nn.functional as F
    from oracle import torch_ref as TR
    cpus, phys, model = _host_cpus()
    avail = len(cpus)
    counts = sorted({t for t in (1, 8, 16, 32, 64, 128) if t <= avail} | {avail})
    prev = torch.get_num_threads()
    sweep, qsweep = {}, {}
    nmat = 4
    g = torch.Generator().manual_seed(0)
    w16 = [(torch.randn(N, K, generator=g) * 0.02).half() for _ in range(nmat)]
    wdq16 = [TR.quantize(w, bits, group)[0].contiguous() for w in w16]
    wdq32 = [w.float() for w in wdq16]
    x16 = torch.randn(M, K, generator=g).half()
    x32 = x16.float()
    per_run = max(0.05, 0.5 * seconds / (len(counts) * 2 * 3))
    try:
        for t in counts:
            torch.set_num_threads(t)
            for dt, x, ws in (("fp16", x16, wdq16), ("fp32", x32, wdq32)):
                F.linear(x, ws[0])  # warm-up
                best = 0.0
                for _ in range(3):
                    n = 0
                    t0 = time.perf_counter()
                    while time.perf_counter() - t0 < per_run:
                        for w in ws:
                            F.linear(x, w)
                            n += 1
                    best = max(best, 2.0 * M * N * K * n / (time.perf_counter() - t0) / 1e12)
                sweep[f"{dt}@{t}"] = round(best, 6)
        for t in sorted({1, min(8, avail), avail}):
            torch.set_num_threads(t)
            calls = []
            t1 = time.perf_counter()
            while len(calls) < 3 or (time.perf_counter() - t1 < 0.4 * seconds / 3 and len(calls) < 20):
                t0 = time.perf_counter()
                TR.quant_linear(x16, w16[len(calls) % nmat], bits, group)
                calls.append(time.perf_counter() - t0)
                if time.perf_counter() - t1 > 0.4 * seconds:
                    break
            qsweep[f"fp16@{t}"] = round(statistics.median(calls) * 1e3, 2)
    finally:
        torch.set_num_threads(prev)
    best_key = max((k for k in sweep if k.startswith("fp16@")), key=lambda k: sweep[k])
    best_t = int(best_key.split("@")[1])
    return {"value": sweep[best_key], "unit": "TFLOP/s", "cores": best_t,
            "kind": "port", "cpu_model": model, "physical_cores": phys,
            "cpus_available": avail, "nproc": os.cpu_count(),
            "sweep_tflops": sweep, "quantize_every_call_ms": qsweep,
            "sample": (f"torch F.linear(x, W_dq) on the host (the reference's eval op, "
                       f"quant/int_linear.py:62; W_dq from oracle/torch_ref.py), M={M} N={N} "
                       f"K={K}, {nmat} distinct pre-dequantized int{bits} g{group} matrices, "
                       f"best of 3 runs of {per_run:.2f}s per (dtype, threads); value = fp16 at "
                       f"its best thread count ({best_t} of {avail} CPUs available, {phys} "
                       f"physical cores); quantize_every_call_ms: use_weight_quant=True, fp16")}


def decode_layer_bytes(cfg, L, bits=4, group=128):
    """Algorithmic HBM bytes of one batch-1 decode step of one LLaMA decoder layer: every packed
    linear by SURVEY.md §8(d)'s formula (M = 1, fp16 scale + int8 zero per group) plus the K / V
    cache rows the attention reads (L rows per KV head, fp16)."""
    H, I = cfg.hidden_size, cfg.intermediate_size
    D = H // cfg.num_attention_heads
    kv = cfg.num_key_value_heads * D
    lin = [(H, H), (kv, H), (kv, H), (H, H), (I, H), (I, H), (H, I)]  # (N, K): q k v o gate up down
    w = sum(algo_bytes(1, N, K, bits, group) for N, K in lin)
    return w + 2 * cfg.num_key_value_heads * L * D * 2, sum(2 * N * K for N, K in lin)


def graph_steps(n, cap=10):
    """Steps per captured graph: the largest divisor of n up to cap (n steps = n / G replays)."""
    return max(g for g in range(1, min(n, cap) + 1) if n % g == 0)


def decode_layer_bench(args, dev, timed):
    """The product's decode path (BASELINE configs[1] inside the model): one batch-1 decode step
    through R distinct LLaMA3-8B-shaped QuantLlamaDecoderLayers (hidden 4096, intermediate 14336,
    32 / 8 heads; random N(0, 0.02^2) weights, RTN int4 g128, packed and fused with the KV cache
    appended in place: five launches per layer), KV cache of --decode-kv rows, graph-replayed;
    R * 114 MB of weights stream from HBM (beyond the 256 MB MALL).  The reference path it replaces
    is QuantLlamaDecoderLayer.forward at q_len 1 (models/int_llama_layer.py:213-267, every
    QuantLinear.forward = F.linear on W_dq, quant/int_linear.py:62)."""
    import torch
    from transformers import LlamaConfig
    from models.int_llama_layer import QuantLlamaDecoderLayer
    from models.quant_llama import quant_args, random_llama_layer, rtn_quantize_
    R, kv = args.decode_layers, args.decode_kv
    cfg = LlamaConfig(hidden_size=4096, intermediate_size=14336, num_attention_heads=32,
                      num_key_value_heads=8, num_hidden_layers=R, vocab_size=128256,
                      max_position_embeddings=8192, rms_norm_eps=1e-5, rope_theta=500000.0)
    qa = quant_args(4, 128)

    class Stack(torch.nn.Module):
        def __init__(self, ls):
            super().__init__()
            self.layers = torch.nn.ModuleList(ls)
    layers = []
    for i in range(R):
        st1 = Stack([QuantLlamaDecoderLayer(cfg, random_llama_layer(cfg, 100 + i, dev,
                                                                    torch.float16), qa)])
        rtn_quantize_(st1, pack=True)  # fp16 weights dropped per layer: only packed bytes stay
        st1.layers[0].fuse_packed_projections(kv_cache=True)
        layers.append(st1.layers[0])
    g = torch.Generator(device=dev).manual_seed(0)
    D = cfg.hidden_size // cfg.num_attention_heads
    past = []
    for layer in layers:
        pk = (torch.randn(1, cfg.num_key_value_heads, kv, D, device=dev, dtype=torch.float16,
                          generator=g),
              torch.randn(1, cfg.num_key_value_heads, kv, D, device=dev, dtype=torch.float16,
                          generator=g))
        past.append(layer.self_attn.adopt_kv_cache(pk))
    x = torch.randn(1, 1, cfg.hidden_size, device=dev, dtype=torch.float16, generator=g)
    mask = torch.zeros(1, 1, 1, kv + 1, device=dev, dtype=torch.float16)
    pos = torch.tensor([[kv]], device=dev)

    def step():
        h = x
        for layer, pkv in zip(layers, past):
            h = layer(h, attention_mask=mask, position_ids=pos, past_key_value=pkv,
                      use_cache=True)[0]
        return h

    # one graph = one 32-layer token's worth of layers (the R distinct layers repeated), as the
    # decode loop captures a token step: its graph-launch overhead is paid once per token
    reps = max(1, 32 // R)

    def time_graph():
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s), torch.no_grad():
            step()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s), torch.no_grad():  # capture on the warm-up stream
            for _ in range(reps):
                step()
        torch.cuda.current_stream(dev).wait_stream(s)
        steps = max(5, args.steps // 4)
        el, _ = timed(graph.replay, steps, max(2, args.warmup // 4))
        del graph
        return el / (steps * reps * R) * 1e6

    us = time_graph()
    nbytes, flops = decode_layer_bytes(cfg, kv + 1)
    out = {"workload": "decode_layer_int4_g128",
           "what": ("LLaMA3-8B decoder layer, batch-1 decode step, int4 g128 packed + fused "
                    "(q/k/v+RMSNorm, attention+RoPE+KV append, o+residual, gate/up+RMSNorm+SiLU*up, "
                    "down+residual: 5 launches), graph-replayed over distinct layers"),
           "layers": R, "layers_per_graph": reps * R, "kv_len": kv + 1,
           "launches_per_layer": 5,
           "us_per_layer": round(us, 2),
           "est_32_layer_token_ms": round(us * 32 / 1e3, 3),
           "tflops": round(flops / us / 1e6, 3),
           "roofline": {"bound": "hbm", "achieved": round(nbytes / us / 1e3, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(nbytes / us / 1e3 / HBM_PEAK_GBS, 4), "traffic": None,
                        "bytes_per_layer": nbytes,
                        "bytes": "7 packed linears by SURVEY §8(d) + the K / V rows read",
                        "timing": ("HIP events over graph replays / layers (one graph = "
                                   f"{reps} x the {R} distinct layers)")}}
    _attach_traffic(out["roofline"], _pmc_traffic("decode_layer_int4_g128"), nbytes)
    del layers
    torch.cuda.empty_cache()
    return out


def pipeline_bench(args, dev, world, rank, backend):
    """BASELINE configs[4]: 32 LLaMA3-8B-width decoder layers, RTN int4 g128, packed + fused
    (prefill-attention kernel for the windows, in-place KV cache for decode), partitioned over the
    N ranks as contiguous pipeline stages with point-to-point hand-offs of the hidden states (RCCL
    over xGMI with the nccl backend; models/pipeline.py) — the counterpart of the reference's
    multi-GPU placement (parallel_utils.py:89-163, main.py:64-80) and PPL loop (main.py:125-151).

      windows: W 2048-token windows in flight through the stages (GPipe fill), Σ NLL per window
               broadcast from the last stage; ms per window = the max-over-ranks wall time of
               the whole pass / W.
      decode:  greedy generation of N sequences (one per stage in flight), every decode step a
               replayed HIP graph per stage (graphs=True); ms per step = the difference of two
               runs of different lengths (prefill and captures cancel) / the extra steps.
      check:   rank 0 builds all layers in one process and runs the same windows and the same
               generation: NLL and tokens must be bit-identical (each layer sees the same input
               tensor, only on another device).
    Random-init weights and synthetic tokens (no checkpoints or datasets offline)."""
    import torch
    import torch.distributed as dist
    from transformers import LlamaConfig
    from models.pipeline import PipelineRunner, greedy_generate, single_stage_nlls, stage_info
    from models.quant_llama import build_random_quant_llama, quant_args, rtn_quantize_
    nl, T = args.pipe_layers, args.pipe_tokens
    W = args.pipe_windows or max(4, 2 * world)
    cfg = LlamaConfig(hidden_size=4096, intermediate_size=14336, num_attention_heads=32,
                      num_key_value_heads=8, num_hidden_layers=nl, vocab_size=128256,
                      max_position_embeddings=max(8192, T + 256), rms_norm_eps=1e-5,
                      rope_theta=500000.0)

    def build(layer_ids):
        m = build_random_quant_llama(cfg, quant_args(4, 128), seed=1, device=dev,
                                     dtype=torch.float16, layer_ids=layer_ids)
        rtn_quantize_(m, pack=True)
        for layer in m.layers:
            layer.fuse_packed_projections(prefill_attention=True, kv_cache=True)
        return m

    def progress(*a):  # a long leg shows it is alive (stderr; stdout keeps the one JSON line)
        if rank == 0:
            print("[pipeline]", *a, file=sys.stderr, flush=True)

    info = stage_info(nl, rank, world)
    t_b = time.perf_counter()
    model = build(range(info.lo, info.hi))
    build_s = time.perf_counter() - t_b
    progress(f"stage {info.lo}..{info.hi} built in {build_s:.1f}s")
    g = torch.Generator(device=dev).manual_seed(123)
    wins = [torch.randint(0, cfg.vocab_size, (1, T), device=dev, generator=g) for _ in range(W)]
    prompts = [torch.randint(0, cfg.vocab_size, (1, 128), device=dev, generator=g)
               for _ in range(world)]
    multi = world > 1

    def wall(fn):
        torch.cuda.synchronize(dev)
        if multi:
            dist.barrier()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize(dev)
        if multi:
            dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                         device=dev if backend == "nccl" else "cpu")
        if multi:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item()), r

    runner = PipelineRunner(model, info, (1, T, cfg.hidden_size), torch.float16, dev)
    first = info.first
    runner.window_nlls(wins if first else None)  # warm: workspaces, code objects, clocks
    t_win, nll = wall(lambda: runner.window_nlls(wins if first else None))
    progress(f"{W} windows: {t_win * 1e3:.1f} ms")
    dr = PipelineRunner(model, info, (1, 1, cfg.hidden_size), torch.float16, dev)
    n_long = max(4, args.pipe_decode)
    n_short = max(2, n_long // 4)
    wall(lambda: dr.generate(prompts if first else None, 2, graphs=True))  # warm
    t_s, _ = wall(lambda: dr.generate(prompts if first else None, n_short, graphs=True))
    t_l, toks = wall(lambda: dr.generate(prompts if first else None, n_long, graphs=True))
    step_s = (t_l - t_s) / (n_long - n_short)
    progress(f"decode: {step_s * 1e3:.3f} ms per step")
    out = {"workload": PIPE_WORKLOAD,
           "what": (f"{nl} LLaMA3-8B decoder layers (4096 / 14336 / 32q 8kv / vocab 128,256), "
                    "RTN int4 g128 packed + fused, as contiguous pipeline stages, hidden states "
                    f"handed stage to stage by {'RCCL (xGMI) ' if backend == 'nccl' else ''}"
                    f"{backend} send / recv" if multi else
                    f"{nl} LLaMA3-8B decoder layers (4096 / 14336 / 32q 8kv / vocab 128,256), "
                    "RTN int4 g128 packed + fused, one stage (the one-rank pipeline)"),
           "backend": backend if multi else None,
           "stages": [[stage_info(nl, r, world).lo, stage_info(nl, r, world).hi]
                      for r in range(world)],
           "build_s_rank0": round(build_s, 2),
           "windows": {"windows_in_flight": W, "tokens_per_window": T,
                       "ms_per_window": round(t_win / W * 1e3, 3),
                       "tokens_per_s": round(W * T / t_win, 1),
                       "ppl": float(torch.exp(nll.double().sum() / (W * T))),
                       "timing": "wall, barrier + synchronize around one pass, max over ranks"},
           "decode": {"sequences": world, "prompt": 128, "graphs": True,
                      "ms_per_step": round(step_s * 1e3, 3),
                      "ms_per_token_per_sequence": round(step_s * 1e3, 3),
                      "tokens_per_s": round(world / step_s, 1),
                      "timing": (f"({n_long} - {n_short}) step difference of two generations, "
                                 "max over ranks")}}
    if not args.pipe_no_check:
        # the one-process reference on rank 0 (every other rank waits at the barrier)
        ok = torch.zeros(2, dtype=torch.int64, device=dev if backend == "nccl" else "cpu")
        if rank == 0:
            if multi:
                del runner, dr
                full = build(range(nl))
            else:
                full = model
            ref_nll = single_stage_nlls(full, wins)
            progress("one-process reference built")
            ref_tok = greedy_generate(full, prompts, n_long, graphs=True)
            ok[0] = int(torch.equal(ref_nll.float(), nll.float().to(ref_nll.device)))
            ok[1] = int(torch.equal(ref_tok, toks))
            del full
            torch.cuda.empty_cache()
        if multi:
            dist.broadcast(ok, src=0)
        out["check"] = {"nll_bit_identical_to_one_process": bool(ok[0]),
                        "tokens_identical_to_one_process": bool(ok[1]),
                        "nll": [round(float(v), 6) for v in nll]}
    return out


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """``--gpus N`` (N > 1) without a launcher: start N rank processes of this script through
    torch.distributed.run (one per GPU, rendezvous on 127.0.0.1) as a CHILD process and return
    its exit code.  Runs before anything in this process touches the GPU (no torch import here),
    so no process that initialised HIP is replaced or forked."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    import torch
    import torch.distributed as dist
    from quant import qlin

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BENCH_DIST_BACKEND=gloo + BENCH_SHARE_GPU=1: rehearse the N > 1 path with several ranks on
    # one GPU (the driver's multi-GPU runs use RCCL, one rank per GPU)
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    gpu = local % torch.cuda.device_count() if os.environ.get("BENCH_SHARE_GPU") else local
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    if args.workload == PIPE_WORKLOAD:
        pipe = pipeline_bench(args, dev, world, rank, backend)
        w = pipe["windows"]
        out = {"metric": "dequant-matmul TFLOP/s + HBM GB/s, int4 g128 4096x4096; LLaMA3-8B PPL delta",
               "value": w["tokens_per_s"], "unit": "tokens/s (2048-token PPL windows)",
               "n_gpus": world, "steps": 1, "warmup": 1,
               "ms_per_step": w["ms_per_window"] * w["windows_in_flight"],
               "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
               "dtype": "f16", "data": "synthetic (random-init weights, random tokens)",
               "config": {"workload": PIPE_WORKLOAD, "model": "LLaMA3-8B architecture",
                          "layers": args.pipe_layers, "bits": 4, "group_size": 128,
                          "parallelism": f"pipeline x{world} (contiguous stages, P2P)"},
               "pipeline": pipe}
        if rank == 0:
            print(json.dumps(out), flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    M, N_full, K, bits, group, ring, kernel, note = WORKLOADS[args.workload]
    N = N_full
    row0 = 0
    if args.split and world > 1:
        # output-feature shard, whole 16-row tiles: the packed layout of a row range is contiguous
        tiles = -(-N_full // 16)
        t0, t1 = tiles * rank // world, tiles * (rank + 1) // world
        row0, N = 16 * t0, min(N_full, 16 * t1) - 16 * t0
    R = args.ring or ring
    gen = torch.Generator(device=dev)
    zb = 2
    hqq = args.workload.endswith("_hqq") or "_hqq_" in args.workload
    # the ring lives in two stacked tensors (problem i = qw[i], qsz[i]): the strided batch reads
    # it in one launch, the per-launch mode through views of the same bytes
    qw_all = torch.zeros((R, *qlin.packed_shape(N, K, bits)), dtype=torch.int32, device=dev)
    sz_all = torch.zeros((R, *qlin.sz_shape(N, K, group)), dtype=torch.int32, device=dev)
    flags = set()
    for i in range(R):
        gen.manual_seed((0 if args.split else 1_000_003 * rank) + i)
        w = torch.empty(N_full, K, device=dev, dtype=torch.float16).normal_(0.0, 0.02, generator=gen)
        w = w[row0:row0 + N].contiguous()
        o = qlin.quantize(w, bits, group, 0, want_xdq=False, want_params=False, pack=True)
        if hqq:
            # HQQ-style non-integral zero points: same codes and bytes, fp16 zero in the qsz word
            sc, zi = qlin.split_sz(o["qsz"], N)
            o["qsz"] = qlin.join_sz_float(sc, zi.to(torch.float16) + 0.375)
            o["flags"] = qlin.FLOAT_ZERO
        qw_all[i].copy_(o["qweight"])
        sz_all[i].copy_(o["qsz"])
        flags.add(o["flags"])
        del w, o
    fl = qlin.FLOAT_ZERO if hqq else (qlin.WIDE_ZERO if qlin.WIDE_ZERO in flags else 0)
    mats = [(qw_all[i], sz_all[i], fl) for i in range(R)]
    gen.manual_seed(1234)
    batched = kernel == "gemv" and args.mode == "batched"
    # one activation row block per problem (the batch reads x[i]; the launches mode reads x[0])
    xs = torch.empty(R, M, K, device=dev, dtype=torch.float16).normal_(0.0, 1.0, generator=gen)
    x = xs[0]
    ys = [torch.empty(M, N, device=dev, dtype=torch.float16) for _ in range(min(R, 4))]
    yb = torch.empty(R, M, N, device=dev, dtype=torch.float16)
    lib = qlin.load_library()
    fn = {"gemv": lib.qlin_gemv_f16, "linear": lib.qlin_linear_f16,
          "gemm": lib.qlin_gemm_f16, "linear_aq": lib.qlin_linear_ep_f16}[kernel]
    ws, ws_bytes = None, 0
    if kernel == "linear_aq":
        ws_bytes = lib.qlin_linear_workspace_bytes(M, N, K, bits, group, 8)
        ws = torch.empty(max(ws_bytes, 2) // 2, dtype=torch.float16, device=dev)

    def step_launches():
        st = torch.cuda.current_stream(dev).cuda_stream
        for i, (qw, qsz, fl_) in enumerate(mats):
            y = ys[i % len(ys)]
            if kernel in ("gemv", "linear"):
                rc = fn(qw.data_ptr(), qsz.data_ptr(), fl_, x.data_ptr(), None,
                        y.data_ptr(), M, N, K, bits, group, st)
            elif kernel == "linear_aq":
                rc = fn(qw.data_ptr(), qsz.data_ptr(), fl_, x.data_ptr(), None, None, y.data_ptr(),
                        M, N, K, bits, group, qlin.EP_NONE, 8, 0, ws.data_ptr(), ws_bytes, st)
            else:
                rc = fn(qw.data_ptr(), qsz.data_ptr(), fl_, x.data_ptr(), None, y.data_ptr(),
                        M, N, K, bits, group, None, 0, st)
            if rc != 0:
                raise RuntimeError(f"kernel failed: {rc}")

    def step_batched():
        st = torch.cuda.current_stream(dev).cuda_stream
        rc = lib.qlin_gemv_batched_f16(qw_all.data_ptr(), qw_all[0].numel(), sz_all.data_ptr(),
                                       sz_all[0].numel(), fl, xs.data_ptr(), M * K, None, 0,
                                       yb.data_ptr(), M * N, R, M, N, K, bits, group, st)
        if rc != 0:
            raise RuntimeError(f"kernel failed: {rc}")

    use_graph = not args.no_graph and (kernel in ("gemv", "linear") or
                                       (kernel == "linear_aq" and M <= 64))

    def make_runner(step, per_graph=1):
        """One HIP graph holding `per_graph` consecutive steps (a replay = that many steps): the
        host's graph-launch overhead (~5 us between the kernels of two replays, against ~0 inside
        one graph; tools/dev/ring_sweep.py) is paid once per graph, as a serving loop that
        captures its steps pays it, not once per step."""
        if not use_graph:
            return step
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            step()  # warm the code objects outside capture
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            for _ in range(per_graph):
                step()
        torch.cuda.current_stream(dev).wait_stream(s)
        return graph.replay

    def timed(run, steps, warmup):
        """HIP events on the launch stream around `steps` runs; barrier + synchronize on both
        sides; MAX over ranks.  Before the `warmup` steps, untimed runs for >= --ramp-s seconds
        bring the GPU clock up from idle (a 0.1 ms step measured 20 % slow for the first ~20 ms
        of work: tools/dev/batch_geo.py rep 1 vs reps 2-3)."""
        t_ramp = time.perf_counter()
        while time.perf_counter() - t_ramp < args.ramp_s:
            run()
            torch.cuda.synchronize(dev)
        for _ in range(warmup):
            run()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(steps):
            run()
        e1.record()
        torch.cuda.synchronize(dev)
        wall_ = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t = torch.tensor([e0.elapsed_time(e1) / 1e3], dtype=torch.float64,
                         device=dev if backend == "nccl" else "cpu")
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item()), wall_

    G = graph_steps(args.steps) if use_graph else 1
    elapsed, wall = timed(make_runner(step_batched if batched else step_launches, G),
                          args.steps // G, max(1, -(-args.warmup // G)))

    flops = 2.0 * M * N * K
    nbytes = algo_bytes(M, N, K, bits, group)
    read_bytes = algo_bytes(M, N, K, bits, group, zb)
    products = args.steps * R  # (1 x M) x (N x K) products in the timed region
    kernel_launches = args.steps * (1 if batched else R)
    per_product_s = elapsed / products
    # whole job: weak = every rank's full ring; strong = the one shared ring (rows summed)
    job_flops = 2.0 * M * N_full * K if args.split else flops * world
    value = job_flops * products / elapsed / 1e12
    hbm_bound = kernel in ("gemv", "linear") or M <= 256

    def roofline(per_product, launch_products):
        if hbm_bound:
            r = {"bound": "hbm", "achieved": round(nbytes / per_product / 1e9, 1),
                 "peak": HBM_PEAK_GBS, "unit": "GB/s"}
        else:
            r = {"bound": "mfma", "achieved": round(flops / per_product / 1e12, 2),
                 "peak": MFMA_F16_PEAK_TFS, "unit": "TFLOP/s"}
        r["frac"] = round(r["achieved"] / r["peak"], 4)
        r["traffic"] = None
        pmc_name = args.workload + ("_batched" if launch_products > 1 else "")
        pmc = _pmc_traffic(pmc_name) if not (args.split and world > 1) else None
        _attach_traffic(r, pmc, nbytes * launch_products, launch_products)
        r["bytes_per_launch"] = nbytes * launch_products
        r["bytes_read_per_launch"] = read_bytes * launch_products
        r["us_per_launch"] = round(per_product * launch_products * 1e6, 3)
        r["products_per_launch"] = launch_products
        return r

    roof = roofline(per_product_s, R if batched else 1)
    if batched:
        roof["timing"] = ("HIP events over the timed region / launches (one strided-batch launch "
                          f"of {R} GEMVs per step; {G} steps per captured graph)")
    else:
        roof["timing"] = ("HIP events over the timed region / launches (graph replay of the ring, "
                          f"{G} steps per captured graph; includes the inter-kernel dispatch gap)"
                          if use_graph else
                          "HIP events over the timed region / launches (eager)")
    other = None
    if kernel == "gemv" and not args.no_other_mode:
        # the other mode, timed the same way, reported beside the headline
        o_steps = max(5, args.steps // 2)
        oG = graph_steps(o_steps) if use_graph else 1
        o_el, _ = timed(make_runner(step_launches if batched else step_batched, oG), o_steps // oG,
                        max(1, -(-max(2, args.warmup // 2) // oG)))
        o_per = o_el / (o_steps * R)
        other = roofline(o_per, 1 if batched else R)
        other["mode"] = "launches" if batched else "batched"
        other["value"] = round(job_flops / o_per / 1e12, 4)

    out = {
        "metric": "dequant-matmul TFLOP/s + HBM GB/s, int4 g128 4096x4096; LLaMA3-8B PPL delta",
        "value": round(value, 4),
        "unit": "TFLOP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "kernel_launches_per_step": kernel_launches // args.steps,
        "higher_is_better": True,
        "scaling": "strong" if args.split else "weak",
        "vs_baseline": None,
        "dtype": "f16",
        "data": "synthetic",
        "hbm_GBps_total": round(nbytes * products * world / elapsed / 1e9, 1),
        "config": {"workload": args.workload, "note": note, "M": M, "N": N_full, "K": K,
                   "N_per_rank": N, "bits": bits, "group_size": group, "ring": R,
                   "sz_bytes_per_group": 2 + zb, "graph": use_graph, "graph_steps": G,
                   "mode": ("batched" if batched else "launches") if kernel == "gemv" else kernel,
                   "parallelism": (f"strong x{world} (output rows split, no collective)"
                                   if args.split else f"weak x{world} (independent rings)")},
        "roofline": roof,
        "wall_s": round(wall, 4),
    }
    if other is not None:
        out["other_mode"] = other
    if kernel == "gemv" and args.workload == "gemv_int4_g128" and not args.no_decode_layer:
        out["decode_layer"] = decode_layer_bench(args, dev, timed)
    if args.pipeline == "on" or (args.pipeline == "auto" and world > 1):
        # configs[4]: the 32-layer pipeline over the same ranks (RCCL P2P between stages)
        out["pipeline"] = pipeline_bench(args, dev, world, rank, backend)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(M, N, K, bits, group, args.cpu_seconds) \
            if M <= 64 else cpu_baseline(min(M, 32), N, K, bits, group, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()  # no rank tears its transport down while a peer is still draining
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
