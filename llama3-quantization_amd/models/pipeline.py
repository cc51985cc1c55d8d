"""Pipeline sharding of the quantized decoder stack: one process per GPU, contiguous stages of
decoder layers, hidden states handed stage to stage with point-to-point send/recv (RCCL over xGMI
with the ``nccl`` backend on MI355X; gloo on CPU for the tests).

Replaces the reference's single-process layer placement (parallel_utils.py:89-131
``assign_layers_to_gpus`` + the forward pre-hooks of :135-159 that ``.to(device)`` every layer
input), used by main.py:66-86 when a model does not fit one GPU.  Differences, by design:
  * stages are contiguous and balanced by layer count (LLaMA layers are identical), instead of
    greedy free-memory placement; the reference's quirk of putting the LAST layer on the first
    layer's GPU (parallel_utils.py:103-107) is not reproduced — numerics are unaffected because
    no tensor is reduced across stages;
  * rank 0 owns the embedding, the last rank owns the final norm + lm_head;
  * several windows (micro-batches) are kept in flight (GPipe-style fill): stage r computes
    micro-batch i while stage r+1 computes micro-batch i-1; sends are asynchronous.

Stage outputs are bit-identical to the single-process model: each layer sees exactly the same
input tensor, only on another device.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist


def stage_bounds(n_layers: int, world: int):
    """Contiguous [lo, hi) layer ranges, sizes differing by at most one (earlier stages larger)."""
    if world < 1 or n_layers < world:
        raise ValueError(f"cannot split {n_layers} layers over {world} stages")
    base, extra = divmod(n_layers, world)
    out, lo = [], 0
    for r in range(world):
        hi = lo + base + (1 if r < extra else 0)
        out.append((lo, hi))
        lo = hi
    return out


@dataclass
class StageInfo:
    rank: int
    world: int
    lo: int
    hi: int

    @property
    def first(self):
        return self.rank == 0

    @property
    def last(self):
        return self.rank == self.world - 1


def stage_info(n_layers: int, rank: int | None = None, world: int | None = None) -> StageInfo:
    if rank is None:
        rank = dist.get_rank() if dist.is_initialized() else 0
    if world is None:
        world = dist.get_world_size() if dist.is_initialized() else 1
    lo, hi = stage_bounds(n_layers, world)[rank]
    return StageInfo(rank, world, lo, hi)


class PipelineRunner:
    """Runs ``model`` (a QuantLlamaForEval holding only this stage's layers, see
    ``build_random_quant_llama(layer_ids=...)``) as stage ``info.rank`` of the pipeline.

    ``model.layers`` must be exactly layers [info.lo, info.hi); the embedding is used on the first
    stage and norm + lm_head on the last.  ``hidden_shape`` is (batch, seq, hidden) of one
    micro-batch and ``dtype`` the hidden-state dtype: every stage knows them up front, so only the
    payload travels."""

    def __init__(self, model, info: StageInfo, hidden_shape, dtype, device):
        if len(model.layers) != info.hi - info.lo:
            raise ValueError(f"stage {info.rank} holds {len(model.layers)} layers, "
                             f"expected {info.hi - info.lo}")
        self.model = model
        self.info = info
        self.hidden_shape = tuple(hidden_shape)
        self.dtype = dtype
        self.device = torch.device(device)

    def _recv(self):
        buf = torch.empty(self.hidden_shape, dtype=self.dtype, device=self.device)
        dist.recv(buf, src=self.info.rank - 1)
        return buf

    @torch.no_grad()
    def forward(self, micro_batches=None, n_micro=None):
        """Pipelined forward of ``micro_batches`` (list of token tensors [B, T], needed on the
        first stage only; other stages pass ``n_micro``).  Returns the list of logits on the last
        stage and None elsewhere."""
        info = self.info
        if info.first:
            if micro_batches is None:
                raise ValueError("the first stage needs the input tokens")
            n_micro = len(micro_batches)
        elif n_micro is None:
            raise ValueError("non-first stages need n_micro")
        outs = []
        pending = []
        for i in range(n_micro):
            if info.first:
                h = self.model.embed_tokens(micro_batches[i].to(self.device))
            else:
                h = self._recv()
            h = self.model.run_layers(h)
            if info.last:
                outs.append(self.model.head(h))
            else:
                h = h.contiguous()
                pending.append((dist.isend(h, dst=info.rank + 1), h))
        for req, _ in pending:
            req.wait()
        return outs if info.last else None

    @torch.no_grad()
    def window_nlls(self, windows):
        """Σ NLL of each window (main.py:136-146) computed on the last stage and broadcast to all
        ranks, so every rank can form the perplexity."""
        n = len(windows) if windows is not None else None
        n_t = torch.tensor([n if n is not None else 0], dtype=torch.int64, device=self.device)
        dist.broadcast(n_t, src=0)
        n = int(n_t.item())
        logits = self.forward(windows if self.info.first else None, n_micro=n)
        from .quant_llama import nll_from_logits
        nll = torch.zeros(n, dtype=torch.float32, device=self.device)
        if self.info.last:
            labels = ([w.to(self.device) for w in windows] if self.info.first
                      else self._labels_from_first(n))
            for i, lg in enumerate(logits):
                nll[i] = nll_from_logits(lg, labels[i])
        elif self.info.first:
            self._send_labels(windows)
        dist.broadcast(nll, src=self.info.world - 1)
        return nll

    def _send_labels(self, windows):
        for w in windows:
            dist.send(w.to(self.device).contiguous(), dst=self.info.world - 1)

    def _labels_from_first(self, n):
        out = []
        for _ in range(n):
            buf = torch.empty(self.hidden_shape[:2], dtype=torch.int64, device=self.device)
            dist.recv(buf, src=0)
            out.append(buf)
        return out


def single_stage_nlls(model, windows):
    """The same Σ NLL per window without a pipeline (world size 1)."""
    from .quant_llama import window_nll
    return torch.stack([window_nll(model, w) for w in windows])
