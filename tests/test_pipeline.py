"""Pipeline sharding of the decoder stack (models/pipeline.py) with gloo, world size 2 and 3:
logits, per-window NLL and greedy decoding (the decode micro-batch mode: per-stage KV caches per
sequence) must equal the single-process model bit for bit (no cross-stage reduction exists), and
the stage split must cover every layer exactly once.

CPU tests: the layers run unquantized (QuantLinear with quant state off -> F.linear), so what is
under test is the stage orchestration and the send/recv plumbing, the same code the GPU run drives
over RCCL.  GPU test: both ranks on cuda:0 (gloo, hand-offs staged through host memory), every
stage running packed int4 layers through the gfx950 kernels, fused with the in-place KV cache."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from models.pipeline import PipelineRunner, greedy_generate, stage_bounds, stage_info
from models.quant_llama import build_random_quant_llama, quant_args, rtn_quantize_, window_nll

N_LAYERS = 5
T = 12
N_WIN = 3


def _cfg():
    from transformers import LlamaConfig
    return LlamaConfig(hidden_size=64, intermediate_size=96, num_attention_heads=4,
                       num_key_value_heads=2, num_hidden_layers=N_LAYERS, vocab_size=101,
                       max_position_embeddings=64, rms_norm_eps=1e-5, rope_theta=500000.0)


def _windows(vocab=101, n=N_WIN, T_=T):
    g = torch.Generator().manual_seed(7)
    return [torch.randint(0, vocab, (1, T_), generator=g) for _ in range(n)]


def _gpu_cfg():
    from transformers import LlamaConfig
    return LlamaConfig(hidden_size=512, intermediate_size=1408, num_attention_heads=4,
                       num_key_value_heads=2, num_hidden_layers=4, vocab_size=1000,
                       max_position_embeddings=256, rms_norm_eps=1e-5, rope_theta=500000.0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _prompts(vocab, n=2, B=1, T_=5, seed=8):
    g = torch.Generator().manual_seed(seed)
    return [torch.randint(0, vocab, (B, T_), generator=g) for _ in range(n)]


def _packed_model(cfg, device, layer_ids=None):
    """int4 g128 RTN, packed, fused with the in-place KV cache (the decode product path)."""
    model = build_random_quant_llama(cfg, quant_args(4, 128), seed=4, device=device,
                                     dtype=torch.float16, layer_ids=layer_ids)
    rtn_quantize_(model, pack=True)
    for layer in model.layers:
        layer.fuse_packed_projections(kv_cache=True)
    return model


N_NEW = 4


def _llama3_8b_cfg(layers=32):
    from transformers import LlamaConfig
    return LlamaConfig(hidden_size=4096, intermediate_size=14336, num_attention_heads=32,
                       num_key_value_heads=8, num_hidden_layers=layers, vocab_size=128256,
                       max_position_embeddings=8192, rms_norm_eps=1e-5, rope_theta=500000.0)


T_FULL = 128  # the full-shape case: one 128-token window


def _worker(rank, world, port, out_dir, kind="cpu"):
    """One pipeline stage.  kind: "cpu" (fp32, unquantized, gloo on CPU), "gpu" (packed int4
    stages at hidden 512 on cuda:0) or "gpu_full" (LLaMA3-8B widths, 32 layers, packed int4 g128
    + fused; every rank on cuda:0, hand-offs staged through host memory)."""
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        torch.manual_seed(0)
        gen_kw = {}
        if kind in ("gpu", "gpu_full"):
            full = kind == "gpu_full"
            cfg = _llama3_8b_cfg() if full else _gpu_cfg()
            T_ = T_FULL if full else T
            info = stage_info(cfg.num_hidden_layers, rank, world)
            dev = torch.device("cuda", 0)
            model = _packed_model(cfg, dev, layer_ids=range(info.lo, info.hi))
            runner = PipelineRunner(model, info, (1, T_, cfg.hidden_size), torch.float16, dev)
            wins = ([w.to(dev) for w in _windows(cfg.vocab_size, n=1 if full else N_WIN, T_=T_)]
                    if info.first else None)
            dtype_dev = dev
            n_win = 1 if full else N_WIN
            gen_kw = {"graphs": True} if full else {}
        else:
            cfg = _cfg()
            info = stage_info(N_LAYERS, rank, world)
            model = build_random_quant_llama(cfg, quant_args(wbits=16), seed=3, device="cpu",
                                             dtype=torch.float32,
                                             layer_ids=range(info.lo, info.hi))
            runner = PipelineRunner(model, info, (1, T, cfg.hidden_size), torch.float32, "cpu")
            wins = _windows() if info.first else None
            dtype_dev = "cpu"
            n_win = N_WIN
        logits = runner.forward(wins, n_micro=n_win)
        nll = runner.window_nlls(wins)
        prompts = [p.to(dtype_dev) for p in _prompts(cfg.vocab_size)] if info.first else None
        toks = runner.generate(prompts, N_NEW, **gen_kw)
        res = {"logits": None if logits is None else [x.cpu() for x in logits],
               "nll": nll.cpu(), "tokens": toks.cpu(), "lo": info.lo, "hi": info.hi}
        if kind == "gpu":
            # the same stages with each decode step captured once per micro-batch and replayed
            # (device-length attention, token hand-back on its own communicator)
            res["tokens_graphs"] = runner.generate(prompts, N_NEW, graphs=True).cpu()
        torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        # every rank past its last collective before any tears gloo down (a rank destroying its
        # group while a peer's transport is still draining aborted the peer now and then)
        dist.barrier()
        dist.destroy_process_group()


def test_stage_bounds_cover_all_layers():
    for n, w in ((32, 8), (32, 3), (5, 2), (7, 7), (12, 5)):
        b = stage_bounds(n, w)
        assert b[0][0] == 0 and b[-1][1] == n
        assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
        sizes = [hi - lo for lo, hi in b]
        assert max(sizes) - min(sizes) <= 1
    assert stage_bounds(32, 8)[3] == (12, 16)
    with pytest.raises(ValueError):
        stage_bounds(3, 4)


@pytest.mark.parametrize("world", [2, 3])
def test_pipeline_matches_single_process(tmp_path, world):
    cfg = _cfg()
    full = build_random_quant_llama(cfg, quant_args(wbits=16), seed=3, device="cpu",
                                    dtype=torch.float32)
    wins = _windows()
    with torch.no_grad():
        ref_logits = [full(w) for w in wins]
        ref_nll = torch.stack([window_nll(full, w) for w in wins])
    ref_tok = greedy_generate(full, _prompts(cfg.vocab_size), N_NEW)
    _check_pipeline(tmp_path, world, N_LAYERS, ref_logits, ref_nll, ref_tok)


def _check_pipeline(tmp_path, world, n_layers, ref_logits, ref_nll, ref_tok, kind="cpu",
                    ref_tok_graphs=None):
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, str(tmp_path), kind), nprocs=world, join=True,
                       start_method="spawn")
    outs = [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=True)
            for r in range(world)]
    assert [o["lo"] for o in outs] == [b[0] for b in stage_bounds(n_layers, world)]
    last = outs[-1]
    assert len(last["logits"]) == len(ref_logits)
    for got, ref in zip(last["logits"], ref_logits):
        assert torch.equal(got, ref.cpu())  # bit-identical: same ops on the same tensors
    for o in outs:  # every rank received the broadcast NLLs and the generated tokens
        assert torch.equal(o["nll"], ref_nll.cpu().to(o["nll"].dtype))
        assert torch.equal(o["tokens"], ref_tok.cpu())
        if ref_tok_graphs is not None:
            assert torch.equal(o["tokens_graphs"], ref_tok_graphs.cpu())
    for o in outs[:-1]:
        assert o["logits"] is None


def test_greedy_generate_uses_the_kv_cache():
    """The decode path (prefill + cached one-token steps) picks the same tokens as re-running the
    whole growing sequence without a cache."""
    cfg = _cfg()
    full = build_random_quant_llama(cfg, quant_args(wbits=16), seed=3, device="cpu",
                                    dtype=torch.float32)
    prompts = _prompts(cfg.vocab_size, n=2, B=2)
    got = greedy_generate(full, prompts, N_NEW)
    assert got.shape == (2, 2, N_NEW)
    with torch.no_grad():
        for i, p in enumerate(prompts):
            seq = p
            for s in range(N_NEW):
                nxt = full(seq)[:, -1].argmax(-1, keepdim=True)
                assert torch.equal(nxt[:, 0], got[i, :, s])
                seq = torch.cat([seq, nxt], 1)


@pytest.mark.gpu
def test_pipeline_packed_stages_on_gpu(tmp_path):
    """World 2 on one MI355X (gloo, host-staged hand-offs): each stage runs packed int4 layers
    through the gfx950 kernels (fused, in-place KV cache in decode) — logits, NLL and greedy
    tokens equal the single-process packed model bit for bit, eager and with every decode step
    replayed from per-micro-batch HIP graphs (graphs=True)."""
    cfg = _gpu_cfg()
    dev = torch.device("cuda", 0)
    full = _packed_model(cfg, dev)
    wins = [w.to(dev) for w in _windows(cfg.vocab_size)]
    with torch.no_grad():
        ref_logits = [full(w) for w in wins]
        ref_nll = torch.stack([window_nll(full, w) for w in wins])
    prompts = [p.to(dev) for p in _prompts(cfg.vocab_size)]
    ref_tok = greedy_generate(full, prompts, N_NEW)
    ref_tok_g = greedy_generate(full, prompts, N_NEW, graphs=True)
    _check_pipeline(tmp_path, 2, cfg.num_hidden_layers, ref_logits, ref_nll, ref_tok, kind="gpu",
                    ref_tok_graphs=ref_tok_g)


@pytest.mark.gpu
@pytest.mark.timeout(1200)
def test_pipeline_llama3_8b_full_shape_8_stages(tmp_path):
    """BASELINE configs[4] at its real shape on one MI355X: 32 LLaMA3-8B-width layers (hidden
    4096, intermediate 14336, 32 / 8 heads, vocab 128,256), int4 g128 RTN, packed + fused, as
    8 stages x 4 layers (8 rank processes, gloo, hand-offs staged through host memory; the
    driver's 8-GPU runs use RCCL, one rank per GPU).  The logits and NLL of one 128-token
    window and 4 greedy decode steps of two sequences with graphs=True (device-length
    attention, per-micro-batch graph replay, token hand-back) equal one process bit for bit
    (reference: parallel_utils.py:89-163, main.py:64-80)."""
    cfg = _llama3_8b_cfg()
    dev = torch.device("cuda", 0)
    full = _packed_model(cfg, dev)
    wins = [w.to(dev) for w in _windows(cfg.vocab_size, n=1, T_=T_FULL)]
    with torch.no_grad():
        ref_logits = [full(w) for w in wins]
        ref_nll = torch.stack([window_nll(full, w) for w in wins])
    prompts = [p.to(dev) for p in _prompts(cfg.vocab_size)]
    ref_tok = greedy_generate(full, prompts, N_NEW, graphs=True)
    assert torch.isfinite(ref_logits[0].float()).all()
    del full
    torch.cuda.empty_cache()
    _check_pipeline(tmp_path, 8, 32, ref_logits, ref_nll, ref_tok, kind="gpu_full")


def _teacher_forced_logits(model, prompt, tokens, device_len):
    """Per-step logits of one sequence fed ``tokens`` (teacher forcing: both paths see the same
    context at every step): prefill, then one token per step through the per-step-length decode
    (``device_len`` False) or the device-length launches (the ones graphs=True captures)."""
    from models.pipeline import StageInfo
    n = len(model.layers)
    run = PipelineRunner(model, StageInfo(0, 1, 0, n), (1, 1, model.config.hidden_size),
                         torch.float16, prompt.device)
    run._past, run._bufs, run._gstate = {}, {}, {}
    T_ = prompt.shape[1]
    out = []
    with torch.no_grad():
        h = run._layers_step(model.embed_tokens(prompt), 0, 0)
        out.append(model.head(h[:, -1:]).float())
        for s in range(tokens.shape[-1] - 1):
            h = model.embed_tokens(tokens[:, s:s + 1])
            pos0 = T_ + s
            if device_len:
                h = run._graph_step(h, 0, pos0, T_ + tokens.shape[-1], replay=False)
            else:
                h = run._layers_step(h, 0, pos0)
            out.append(model.head(h[:, -1:]).float())
    return torch.cat(out, 1)


@pytest.mark.gpu
def test_generate_graph_replay_matches_eager():
    """Decode steps captured once per sequence as HIP graphs (the cache length read on the device)
    give the same tokens, bit for bit, as the same device-length launches run eagerly.  Against
    the per-step-length path (whose attention splits the rows by the step's length, not the
    generation's maximum: fp32 summation order only) the device-length path is compared by its
    per-step logits with both fed the same tokens (teacher forcing), so every step is checked
    on the same context: max |d logit| <= 5e-3 x max |logit| at every step."""
    cfg = _gpu_cfg()
    dev = torch.device("cuda", 0)
    model = _packed_model(cfg, dev)
    prompts = [p.to(dev) for p in _prompts(cfg.vocab_size, n=3, B=1)]
    n_new = 12
    ref = greedy_generate(model, prompts, n_new)
    eager = greedy_generate(model, prompts, n_new, device_len=True)
    graph = greedy_generate(model, prompts, n_new, graphs=True)
    assert torch.equal(eager, graph)
    assert torch.equal(ref[:, :, 0], eager[:, :, 0])  # the prefill step is the same path
    for i, p in enumerate(prompts):
        a = _teacher_forced_logits(model, p, ref[i], device_len=False)
        b = _teacher_forced_logits(model, p, ref[i], device_len=True)
        assert torch.equal(a.argmax(-1)[0], ref[i, 0])  # per-step path reproduces its tokens
        scale = a.abs().amax(-1)
        rel = ((a - b).abs().amax(-1) / scale)[0]
        assert rel.max().item() <= 5e-3, rel


@pytest.mark.gpu
def test_generate_graphs_fall_back_past_attn_max_l():
    """A generation whose cache would pass qlin.ATTN_MAX_L rows cannot use the device-length
    attention (it serves at most that many rows): generate(graphs=True) takes the per-step
    path instead (PipelineRunner.generate), so its tokens equal the eager path's bit for bit
    rather than attending over a clamped prefix."""
    from quant import qlin
    cfg = _gpu_cfg()
    cfg.max_position_embeddings = 2 * qlin.ATTN_MAX_L
    dev = torch.device("cuda", 0)
    model = _packed_model(cfg, dev)
    T_ = qlin.ATTN_MAX_L - 2  # prompt + 4 new tokens passes ATTN_MAX_L
    prompts = [p.to(dev) for p in _prompts(cfg.vocab_size, n=1, B=1, T_=T_)]
    eager = greedy_generate(model, prompts, 4)
    graph = greedy_generate(model, prompts, 4, graphs=True)
    assert torch.equal(eager, graph)
