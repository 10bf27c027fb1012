"""Pipeline-parallel inference: contiguous layer stages, one process per GPU.

Reference: ``SRC/transformers/pipeline_parallel.py`` -- ``pipeline_parallel``
(166-234: slice layers, Dummy layers elsewhere, embedding on the first and
norm + lm_head on the last stage) and ``pipeline_parallel_generate``
(300-445: hidden states hop stage to stage with send/recv, the last rank
broadcasts ``next_ids``).

MI355X design: stages execute the native decoder (paged KV cache, fused
kernels) over their own layer range; the residual stream [T, hidden] is the
only thing crossing a stage boundary (RCCL send/recv over xGMI on GPU, gloo
on CPU).  Micro-batching across stages for serving is in
``serving/pp_worker.py``.  With 288 GB per MI355X, PP exists for capability
parity and for models whose INT4 weights exceed one GPU (e.g. 671B MoE).
"""
from __future__ import annotations

import time
import types
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist
import torch.nn as nn

from .comm import get_rank, get_world_size


class DummyLayer(nn.Module):
    """Stand-in for a module owned by another stage (reference: DummyLayer)."""

    def forward(self, x, *args, **kwargs):
        return x


class DummyDecoderLayer(nn.Module):
    def __init__(self):
        super().__init__()
        self.input_layernorm = DummyLayer()

    def forward(self, hidden_states, *args, **kwargs):
        return hidden_states


def stage_range(num_layers: int, stages: int, rank: int):
    per = (num_layers + stages - 1) // stages
    start = min(num_layers, per * rank)
    return start, min(num_layers, start + per)


def _decoder_root(model):
    for name in ("model", "transformer"):
        m = getattr(model, name, None)
        if m is not None and hasattr(m, "layers"):
            return m
    raise ValueError("pipeline_parallel: cannot find the decoder layer list")


def pipeline_parallel(model: nn.Module, stages: int, group=None, device=None) -> nn.Module:
    """Keep this rank's layer range of an (already low-bit) HF CausalLM,
    replace the rest with dummies and move it to this rank's GPU."""
    rank, world = get_rank(group), get_world_size(group)
    if world != stages:
        raise ValueError(f"pipeline_parallel_stages={stages} but the process group has {world} ranks")
    base = _decoder_root(model)
    L = len(base.layers)
    start, end = stage_range(L, stages, rank)
    for i in range(L):
        if not (start <= i < end):
            base.layers[i] = DummyDecoderLayer()
    if rank != 0 and hasattr(base, "embed_tokens"):
        base.embed_tokens = DummyLayer()
    if rank != stages - 1:
        if hasattr(base, "norm"):
            base.norm = DummyLayer()
        if hasattr(model, "lm_head"):
            model.lm_head = DummyLayer()
    model._pp = {"group": group, "rank": rank, "stages": stages, "start": start, "end": end}
    if device is None and torch.cuda.is_available():
        device = torch.device("cuda", torch.cuda.current_device())
    if device is not None:
        model.to(device)
    model.generate = types.MethodType(_pp_generate, model)
    return model


def _pp_generate(self, input_ids=None, max_new_tokens: int = 32, **kwargs):
    from ..transformers.hf_native import get_native
    native, _ = get_native(self)
    eng = PipelineEngine(native, self._pp["group"])
    prompts = input_ids.tolist() if torch.is_tensor(input_ids) else input_ids
    eos = kwargs.get("eos_token_id", getattr(getattr(self, "generation_config", None), "eos_token_id", None))
    t = eng.generate(prompts, max_new_tokens=max_new_tokens, eos_token_id=eos)
    self.first_token_time, self.rest_cost_mean = eng.first_cost, eng.rest_cost_mean
    width = max(len(x) for x in t)
    pad = getattr(getattr(self, "generation_config", None), "pad_token_id", None) or 0
    return torch.tensor([x + [pad] * (width - len(x)) for x in t], dtype=torch.long)


class PipelineEngine:
    """Runs prefill + decode across pipeline stages.  Call ``generate`` with
    the same prompts on every rank (as the reference does)."""

    def __init__(self, model, group=None, block_size: int = 64, kv_fp8: int = 0):
        from ..engine.runner import Engine
        self.model = model
        self.group = group
        self.rank, self.world = get_rank(group), get_world_size(group)
        self.prev = (self.rank - 1) % self.world
        self.next = (self.rank + 1) % self.world
        self.inner = Engine(model, block_size, kv_fp8)
        self.first_cost = 0.0
        self.rest_cost_mean = 0.0

    def _g(self, r):
        return dist.get_global_rank(self.group, r) if self.group is not None else r

    def _stage(self, ids, pos, slots, meta, logits_idx=None):
        m = self.model
        dev = m.device
        hidden = None
        if not m.first_stage:
            hidden = torch.empty(ids.numel(), m.spec.hidden_size, dtype=m.dtype, device=dev)
            dist.recv(hidden, src=self._g(self.prev), group=self.group)
        out = m.forward_tokens(ids, pos, slots, meta, self.inner.cache, logits_idx=logits_idx, hidden_in=hidden)
        if not m.last_stage:
            dist.send(out.contiguous(), dst=self._g(self.next), group=self.group)
            return None
        return out

    def _bcast_next(self, nxt: Optional[torch.Tensor], B: int):
        dev = self.model.device
        buf = nxt.to(dev, torch.long).contiguous() if nxt is not None else torch.empty(B, dtype=torch.long, device=dev)
        dist.broadcast(buf, src=self._g(self.world - 1), group=self.group)
        return buf

    @torch.no_grad()
    def generate(self, prompts: Sequence[Sequence[int]], max_new_tokens: int = 32, eos_token_id=None) -> List[List[int]]:
        from ..engine.runner import nsplit_for
        from ..models.cache import SequenceState, make_block_table, slots_for
        from ..models.decoder import AttnMeta
        m = self.model
        dev = m.device
        B = len(prompts)
        max_len = max(len(p) for p in prompts) + max_new_tokens + 1
        cache = self.inner._ensure_cache(B, max_len)
        nblk = (max_len + cache.bs - 1) // cache.bs
        seqs = [SequenceState(cache.allocator.alloc(nblk)) for _ in range(B)]
        eos = set([eos_token_id] if isinstance(eos_token_id, int) else (eos_token_id or []))
        sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
        t0 = time.perf_counter()
        firsts = []
        for b, p in enumerate(prompts):
            n = len(p)
            ids = torch.tensor(list(p), dtype=torch.long, device=dev)
            pos = torch.arange(n, device=dev)
            slots = slots_for(seqs[b], 0, n, cache.bs).to(dev)
            bt = make_block_table([seqs[b]], nblk, dev)
            meta = AttnMeta(1, n, bt, torch.tensor([n], dtype=torch.int32, device=dev), nsplit_for(n), [n])
            lg = self._stage(ids, pos, slots, meta, logits_idx=torch.tensor([n - 1], device=dev))
            firsts.append(torch.argmax(lg, -1) if lg is not None else None)
            seqs[b].length = n
        nxt = torch.cat(firsts) if m.last_stage else None
        cur = self._bcast_next(nxt, B)
        sync()
        self.first_cost = time.perf_counter() - t0
        out = [list(p) for p in prompts]
        done = [False] * B
        toks = cur.tolist()
        for b in range(B):
            out[b].append(toks[b])
            done[b] = toks[b] in eos
        bt = make_block_table(seqs, nblk, dev)
        costs = []
        for _ in range(1, max_new_tokens):
            if all(done):
                break
            t1 = time.perf_counter()
            pos = torch.tensor([s.length for s in seqs], device=dev)
            blk = torch.gather(bt, 1, (pos // cache.bs).unsqueeze(1)).squeeze(1).long()
            slots = blk * cache.bs + pos % cache.bs
            meta = AttnMeta(B, 1, bt, (pos + 1).to(torch.int32), nsplit_for(max_len))
            lg = self._stage(cur, pos, slots, meta)
            cur = self._bcast_next(torch.argmax(lg, -1) if lg is not None else None, B)
            for s in seqs:
                s.length += 1
            toks = cur.tolist()
            costs.append(time.perf_counter() - t1)
            for b in range(B):
                if not done[b]:
                    out[b].append(toks[b])
                    done[b] = toks[b] in eos
        self.rest_cost_mean = sum(costs) / max(1, len(costs))
        for s in seqs:
            cache.allocator.release(s.blocks)
        return out
