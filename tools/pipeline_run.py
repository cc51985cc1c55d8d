#!/usr/bin/env python3
"""Pipeline-sharded evaluation of a random-init LLaMA-architecture stack, one process per GPU
(RCCL send/recv between stages): python -m torch.distributed.run --nproc-per-node N
--master-addr 127.0.0.1 --master-port P tools/pipeline_run.py [--layers 32 --hidden 4096 ...].

Each rank builds (from the shared seed) only its own stage's layers, RTN-quantizes and packs them
(int4 g128 by default), then the pipeline runs W windows of T tokens; rank 0 prints per-window
NLL, the PPL, the wall time per window and (with --check) the max |difference| of the logits to a
single-process run of the same model on rank 0's GPU (only when every layer fits one GPU)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama3-quantization_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from models.pipeline import PipelineRunner, stage_info  # noqa: E402
from models.quant_llama import build_random_quant_llama, quant_args, rtn_quantize_  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--inter", type=int, default=14336)
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--kv-heads", type=int, default=8)
    ap.add_argument("--vocab", type=int, default=128256)
    ap.add_argument("--tokens", type=int, default=2048)
    ap.add_argument("--windows", type=int, default=4)
    ap.add_argument("--wbits", type=int, default=4)
    ap.add_argument("--group", type=int, default=128)
    ap.add_argument("--fake-quant", action="store_true", help="dense F.linear on W_dq instead of packed")
    ap.add_argument("--fused", action="store_true",
                    help="packed + fuse_packed_projections() (fused q/k/v, gate/up+SiLU, epilogues)")
    ap.add_argument("--decode", type=int, default=0,
                    help="also greedy-decode this many tokens for --micro sequences, eager and "
                         "with HIP-graph-replayed steps (decode "
                         "micro-batch mode: per-stage KV caches; fused layers use kv_cache=True)")
    ap.add_argument("--micro", type=int, default=0, help="decode sequences (default: world size)")
    ap.add_argument("--prompt", type=int, default=128, help="decode prompt length")
    a = ap.parse_args()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    from transformers import LlamaConfig
    cfg = LlamaConfig(hidden_size=a.hidden, intermediate_size=a.inter, num_attention_heads=a.heads,
                      num_key_value_heads=a.kv_heads, num_hidden_layers=a.layers,
                      vocab_size=a.vocab, max_position_embeddings=max(4096, a.tokens),
                      rms_norm_eps=1e-5, rope_theta=500000.0)
    info = stage_info(a.layers, rank, world)
    model = build_random_quant_llama(cfg, quant_args(a.wbits, a.group), seed=1, device=dev,
                                     dtype=torch.float16, layer_ids=range(info.lo, info.hi))
    rtn_quantize_(model, pack=not a.fake_quant)
    if a.fused and not a.fake_quant:
        for layer in model.layers:
            layer.fuse_packed_projections(kv_cache=a.decode > 0)
    g = torch.Generator(device=dev).manual_seed(123)
    wins = [torch.randint(0, a.vocab, (1, a.tokens), device=dev, generator=g)
            for _ in range(a.windows)] if info.first else None
    runner = PipelineRunner(model, info, (1, a.tokens, a.hidden), torch.float16, dev)
    runner.window_nlls(wins)  # warm
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    nll = runner.window_nlls(wins)
    torch.cuda.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
    dec = None
    if a.decode > 0:
        n_micro = a.micro or world
        prompts = [torch.randint(0, a.vocab, (1, a.prompt), device=dev, generator=g)
                   for _ in range(n_micro)] if info.first else None
        dr = PipelineRunner(model, info, (1, 1, a.hidden), torch.float16, dev)

        def timed(n, graphs):
            torch.cuda.synchronize()
            dist.barrier()
            t1 = time.perf_counter()
            toks = dr.generate(prompts, n, graphs=graphs)
            torch.cuda.synchronize()
            dist.barrier()
            return time.perf_counter() - t1, toks

        dec = {}
        for mode, graphs in (("eager", False), ("graphs", True)):
            timed(2, graphs)  # warm
            short = max(2, a.decode // 4)
            t_s, _ = timed(short, graphs)
            t_l, toks = timed(a.decode, graphs)
            # differential: the prefill step and the graph captures (first decode step of each
            # sequence) cancel between the two runs
            per_step = (t_l - t_s) / (a.decode - short)
            dec[mode] = {"sequences": n_micro, "prompt": a.prompt, "new_tokens": a.decode,
                         "ms_per_step": round(per_step * 1e3, 3),
                         "tokens_per_s": round(n_micro / per_step, 1),
                         "first_tokens": toks[:, 0, :8].tolist()}
    if rank == 0:
        ppl = float(torch.exp(nll.sum() / (a.windows * a.tokens)))
        print(json.dumps({"world": world, "layers": a.layers, "stages": [list(x) for x in
                          [(s.lo, s.hi) for s in [stage_info(a.layers, r, world) for r in range(world)]]],
                          "mode": "fake-quant" if a.fake_quant else
                          f"packed{' fused' if a.fused else ''} int{a.wbits} g{a.group}",
                          "windows": a.windows, "tokens": a.tokens, "ppl": ppl,
                          "ms_per_window": round(dt / a.windows * 1e3, 2),
                          "nll": [round(float(v), 4) for v in nll], "decode": dec}))
    dist.barrier()  # no rank tears its transport down while a peer is still draining
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
