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
    micro-batch i while stage r+1 computes micro-batch i-1; sends are asynchronous;
  * decode (``generate``): greedy autoregressive decoding of several independent sequences
    (micro-batches) — each stage keeps the KV cache of its own layers for every micro-batch
    (the reference's per-layer ``past_key_value``, models/int_llama_layer.py:130-135, or the fused
    layer's in-place cache buffers swapped in per micro-batch), the last stage picks each
    micro-batch's next token and sends it back to the first stage at once, on a communicator of
    its own, so stage 0 starts that micro-batch's next step while the later stages still run the
    current one (no per-step drain).
  * transport: RCCL point-to-point with ``nccl``; with ``gloo`` device tensors are staged through
    host memory (gloo's send / recv take CPU tensors), e.g. several ranks sharing one GPU in tests.

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
        self._tok_group = None

    def _host_staged(self):
        return dist.get_backend() == "gloo" and self.device.type != "cpu"

    def _recv(self, shape=None, dtype=None, src=None, group=None):
        shape = self.hidden_shape if shape is None else tuple(shape)
        dtype = self.dtype if dtype is None else dtype
        src = self.info.rank - 1 if src is None else src
        if self._host_staged():
            buf = torch.empty(shape, dtype=dtype)
            dist.recv(buf, src=src, group=group)
            return buf.to(self.device)
        buf = torch.empty(shape, dtype=dtype, device=self.device)
        dist.recv(buf, src=src, group=group)
        return buf

    def _bcast(self, t, src):
        """broadcast in place (through host memory for gloo with device tensors)"""
        if self._host_staged():
            h = t.cpu()
            dist.broadcast(h, src=src)
            t.copy_(h)
        else:
            dist.broadcast(t, src=src)
        return t

    def _isend(self, t, dst, group=None):
        """(request, the tensor kept alive until the request completes)"""
        t = t.contiguous()
        if self._host_staged():
            t = t.cpu()
        return dist.isend(t, dst=dst, group=group), t

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
                pending.append(self._isend(h, info.rank + 1))
        for req, _ in pending:
            req.wait()
        return outs if info.last else None

    # -- decode ----------------------------------------------------------------------------------
    def _layers_step(self, h, mb, pos0):
        """This stage's layers over h [B, T, H] of micro-batch ``mb`` at positions pos0..pos0+T-1,
        with that micro-batch's own KV cache per layer: the ``past_key_value`` each layer returned
        last time, and for layers in kv_cache mode (fuse_packed_projections(kv_cache=True)) their
        cache buffers, swapped in so the append stays in place."""
        B, T = h.shape[:2]
        from .quant_llama import causal_mask
        mask = causal_mask(B, T, h.dtype, h.device, past=pos0)
        pos = torch.arange(pos0, pos0 + T, device=h.device)[None].expand(B, T)
        n = len(self.model.layers)
        past = self._past.setdefault(mb, [None] * n)
        bufs = self._bufs.setdefault(mb, [None] * n)
        for j, layer in enumerate(self.model.layers):
            at = layer.self_attn
            own = bool(getattr(at, "kv_cache", False))
            if own:
                at._kv = bufs[j]
            h, past[j] = layer(h, attention_mask=mask, position_ids=pos, past_key_value=past[j],
                               use_cache=True)
            if own:
                bufs[j] = at._kv
        return h

    def _layers_step_len(self, h, mb, pos, length, max_len):
        """This stage's layers over one token per sequence with the cache length on the device
        (each layer's attention in its device-length mode over micro-batch ``mb``'s buffers, its
        grid sized for ``max_len``, the longest length of the generation): the launch sequence of
        every decode step, captured once per micro-batch."""
        bufs = self._bufs[mb]
        for j, layer in enumerate(self.model.layers):
            at = layer.self_attn
            at._kv = bufs[j]
            at._dyn_len, at._dyn_max = length, max_len
            try:
                h = layer(h, attention_mask=None, position_ids=pos, past_key_value=None,
                          use_cache=False)[0]
            finally:
                at._dyn_len = at._dyn_max = None
        return h

    def _graph_step(self, h, mb, pos0, cap_rows, replay):
        """Decode step of micro-batch ``mb`` at position pos0 through the device-length layers:
        replayed from its HIP graph (captured at its first step) when ``replay``, else eager —
        the same launches either way, so both give the same bits."""
        st = self._gstate.get(mb)
        if st is None:
            B, T, H = h.shape
            # every layer's cache buffers must hold all the steps: grow them once, here
            for j, layer in enumerate(self.model.layers):
                at = layer.self_attn
                kb, vb = self._bufs[mb][j]
                if kb.shape[2] < cap_rows:
                    at.adopt_kv_cache((kb[:, :, :pos0], vb[:, :, :pos0]), rows=cap_rows)
                    self._bufs[mb][j] = at._kv
            st = {"h": torch.empty_like(h), "pos": torch.empty(B, 1, dtype=torch.int64,
                                                                 device=h.device),
                  "len": torch.empty(1, dtype=torch.int32, device=h.device), "graph": None}
            self._gstate[mb] = st
        st["h"].copy_(h)
        st["pos"].fill_(pos0)
        st["len"].fill_(pos0 + 1)
        if not replay:
            return self._layers_step_len(st["h"], mb, st["pos"], st["len"], cap_rows)
        if st["graph"] is None:
            # one eager pass first (workspaces, rotary tables, the attention's merge counters,
            # which are kept per stream), then the capture ON THE SAME STREAM, so nothing is first
            # allocated inside the capture; both passes rewrite the same cache row pos0 with the
            # same values before the replay below
            s_ = torch.cuda.Stream(h.device)
            s_.wait_stream(torch.cuda.current_stream(h.device))
            with torch.cuda.stream(s_):
                self._layers_step_len(st["h"], mb, st["pos"], st["len"], cap_rows)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s_):
                st["out"] = self._layers_step_len(st["h"], mb, st["pos"], st["len"], cap_rows)
            torch.cuda.current_stream(h.device).wait_stream(s_)
            st["graph"] = g
        st["graph"].replay()
        return st["out"].clone()

    @torch.no_grad()
    def generate(self, prompts=None, n_new=8, graphs=False, device_len=None):
        """Greedy decoding of independent sequences through the pipeline.  ``prompts``: list of
        int64 token tensors [B, T] (one micro-batch each, same shape), needed on the first stage
        only.  Step 0 runs the prompts (prefill) and picks the first new token; each later step
        runs one token per sequence over the stages' KV caches.  Returns int64 [n_micro, B, n_new]
        on every rank.

        ``graphs`` (GPU, fused packed layers in kv_cache mode): decode steps run each stage's
        layers in their device-length form (the cache length read on the device), captured into
        one HIP graph per micro-batch at its first decode step and replayed after;
        ``device_len=True`` runs that form eagerly (same bits as the graphs)."""
        device_len = graphs if device_len is None else device_len
        info = self.info
        multi = info.world > 1
        meta = torch.zeros(3, dtype=torch.int64)
        if info.first:
            if not prompts:
                raise ValueError("the first stage needs the prompts")
            shapes = {tuple(p.shape) for p in prompts}
            if len(shapes) != 1 or len(next(iter(shapes))) != 2:
                raise ValueError("prompts must share one [B, T] shape")
            meta = torch.tensor([len(prompts), *prompts[0].shape], dtype=torch.int64)
        if multi:
            meta = self._bcast(meta.to(self.device), 0).cpu()
        n_micro, B, T = (int(v) for v in meta.tolist())
        H = self.hidden_shape[-1]
        from quant import qlin
        if device_len and T + n_new > qlin.ATTN_MAX_L:
            # the device-length attention serves at most ATTN_MAX_L cache rows: longer
            # generations take the per-step path (whose attention leaves the kernel there)
            device_len = graphs = False
        self._past, self._bufs, self._gstate = {}, {}, {}
        out = torch.zeros(n_micro, B, n_new, dtype=torch.int64, device=self.device)
        # next-token hand-back on a communicator of its own (first <-> last stage): each
        # micro-batch's token leaves the last stage as soon as it is picked, and the first stage
        # takes it just before that micro-batch's next step, so stage 0 starts micro-batch i of
        # step s + 1 while later stages still run step s; a separate communicator keeps these
        # transfers off the hidden-state stream's queue (RCCL runs one communicator's
        # point-to-point operations in order)
        if multi and getattr(self, "_tok_group", None) is None:
            self._tok_group = dist.new_group([0, info.world - 1])  # collective: every rank
        tok_group = self._tok_group if multi else None
        cur = [None] * n_micro  # next input tokens [B, 1] per micro-batch (first stage)
        tok_reqs, pending = [], []
        for step in range(n_new):
            # stages run ahead (no per-step drain), but sends that have completed are released
            # once per step, so held buffers stay bounded instead of growing with n_new * n_micro
            pending = [p for p in pending if not p[0].is_completed()]
            tok_reqs = [p for p in tok_reqs if not p[0].is_completed()]
            T_in, pos0 = (T, 0) if step == 0 else (1, T + step - 1)
            for i in range(n_micro):
                if info.first:
                    if step == 0:
                        ids = prompts[i].to(self.device)
                    elif info.last:
                        ids = cur[i]
                    else:
                        ids = self._recv((B, 1), torch.int64, src=info.world - 1, group=tok_group)
                    h = self.model.embed_tokens(ids)
                else:
                    h = self._recv((B, T_in, H))
                if step > 0 and device_len:
                    h = self._graph_step(h, i, pos0, T + n_new, replay=graphs)
                else:
                    h = self._layers_step(h, i, pos0)
                if info.last:
                    tok = self.model.head(h[:, -1:]).argmax(-1)  # [B, 1]
                    out[i, :, step] = tok[:, 0]
                    if info.first:
                        cur[i] = tok
                    elif step + 1 < n_new:
                        tok_reqs.append(self._isend(tok, 0, group=tok_group))
                else:
                    pending.append(self._isend(h, info.rank + 1))
        for req, _ in pending + tok_reqs:  # no per-step drain: stages run ahead
            req.wait()
        if multi:
            self._bcast(out, info.world - 1)
        return out

    @torch.no_grad()
    def window_nlls(self, windows):
        """Σ NLL of each window (main.py:136-146) computed on the last stage and broadcast to all
        ranks, so every rank can form the perplexity."""
        n = len(windows) if windows is not None else None
        if self.info.world > 1:
            n_t = torch.tensor([n if n is not None else 0], dtype=torch.int64, device=self.device)
            self._bcast(n_t, 0)
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
        if self.info.world > 1:
            self._bcast(nll, self.info.world - 1)
        return nll

    def _send_labels(self, windows):
        for w in windows:
            req, _ = self._isend(w.to(self.device), self.info.world - 1)
            req.wait()

    def _labels_from_first(self, n):
        out = []
        for _ in range(n):
            out.append(self._recv(self.hidden_shape[:2], torch.int64, src=0))
        return out


@torch.no_grad()
def greedy_generate(model, prompts, n_new, graphs=False, device_len=None):
    """The same greedy decoding in one process (world size 1): the reference's loop of
    QuantLlamaDecoderLayer.forward with use_cache=True over a prompt, then one token at a time
    (``graphs`` / ``device_len``: see PipelineRunner.generate)."""
    info = StageInfo(0, 1, 0, len(model.layers))
    H = model.config.hidden_size
    runner = PipelineRunner(model, info, (1, 1, H), model.embed_tokens.weight.dtype,
                            model.embed_tokens.weight.device)
    return runner.generate(prompts, n_new, graphs=graphs, device_len=device_len)


def single_stage_nlls(model, windows):
    """The same Σ NLL per window without a pipeline (world size 1)."""
    from .quant_llama import window_nll
    return torch.stack([window_nll(model, w) for w in windows])
