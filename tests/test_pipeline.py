"""Pipeline sharding of the decoder stack (models/pipeline.py) on CPU with gloo, world size 2 and
3: logits and per-window NLL must equal the single-process model bit for bit (no cross-stage
reduction exists), and the stage split must cover every layer exactly once.

The layers run unquantized here (QuantLinear with quant state off -> F.linear), which keeps the
test on CPU: what is under test is the stage orchestration and the send/recv plumbing, the same
code the GPU run drives over RCCL."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from models.pipeline import PipelineRunner, stage_bounds, stage_info
from models.quant_llama import build_random_quant_llama, quant_args, window_nll

N_LAYERS = 5
T = 12
N_WIN = 3


def _cfg():
    from transformers import LlamaConfig
    return LlamaConfig(hidden_size=64, intermediate_size=96, num_attention_heads=4,
                       num_key_value_heads=2, num_hidden_layers=N_LAYERS, vocab_size=101,
                       max_position_embeddings=64, rms_norm_eps=1e-5, rope_theta=500000.0)


def _windows():
    g = torch.Generator().manual_seed(7)
    return [torch.randint(0, 101, (1, T), generator=g) for _ in range(N_WIN)]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        torch.manual_seed(0)
        cfg = _cfg()
        info = stage_info(N_LAYERS, rank, world)
        model = build_random_quant_llama(cfg, quant_args(wbits=16), seed=3, device="cpu",
                                         dtype=torch.float32,
                                         layer_ids=range(info.lo, info.hi))
        runner = PipelineRunner(model, info, (1, T, cfg.hidden_size), torch.float32, "cpu")
        wins = _windows() if info.first else None
        logits = runner.forward(wins, n_micro=N_WIN)
        nll = runner.window_nlls(wins)
        torch.save({"logits": logits, "nll": nll, "lo": info.lo, "hi": info.hi},
                   os.path.join(out_dir, f"rank{rank}.pt"))
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

    port = _free_port()
    mp.start_processes(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    outs = [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=True)
            for r in range(world)]
    assert [o["lo"] for o in outs] == [b[0] for b in stage_bounds(N_LAYERS, world)]
    last = outs[-1]
    assert len(last["logits"]) == N_WIN
    for got, ref in zip(last["logits"], ref_logits):
        assert torch.equal(got, ref)  # bit-identical: same ops on the same tensors
    for o in outs:  # every rank received the broadcast NLLs
        assert torch.equal(o["nll"], ref_nll.to(o["nll"].dtype))
    for o in outs[:-1]:
        assert o["logits"] is None
