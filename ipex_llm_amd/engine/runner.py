"""Decode-step execution with hipGraph capture + a generate() loop.

The reference issues ~300 kernel launches per token eagerly from Python and
has no graph capture (vLLM runs --enforce-eager).  Here the
whole decode step -- embedding, all layers, lm_head and greedy argmax --
is captured once per (batch, max_blocks) into a hipGraph via
``torch.cuda.CUDAGraph`` (HIP graphs on ROCm) and replayed per token.  The
step advances its own position counter on the device, derives the KV slot
from the block table on the device, and feeds its argmax back as the next
input, so back-to-back replays need no host<->device traffic at all.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..models.cache import PagedKVCache, SequenceState, make_block_table, slots_for
from ..models.decoder import AttnMeta, NativeCausalLM

SPLIT = 64


def nsplit_for(max_len: int) -> int:
    return max(1, (max_len + SPLIT - 1) // SPLIT)


_ARGMAX_EPI = __import__("os").environ.get("ILLM_ARGMAX_EPI", "1") != "0"


def _argmax_head_ok(head, h: torch.Tensor, spec) -> bool:
    """greedy decode through the lm_head GEMV's argmax epilogue (ops_hip.cpp
    gemv_argmax): a plain single-device low-bit head on the v5 GEMV formats"""
    from ..transformers.low_bit_linear import LowBitLinear
    from ..quantize import qtypes as Q
    return (_ARGMAX_EPI and isinstance(head, LowBitLinear) and head.mp_group is None
            and getattr(head, "g_idx_map", None) is None and getattr(head, "compute_dtype", None) in (None, h.dtype)
            and not spec.final_softcap and h.dim() == 2 and h.shape[0] <= 16
            and h.dtype in (torch.bfloat16, torch.float16)
            and head.fmt in (Q.FMT_SYM_INT4, Q.FMT_ASYM_INT4, Q.FMT_NF4, Q.FMT_NF3, Q.FMT_FP4, Q.FMT_SYM_INT8,
                             Q.FMT_SYM_INT5, Q.FMT_ASYM_INT5, Q.FMT_FP8E4, Q.FMT_FP8E5, Q.FMT_FP6)
            and (head.bias is None or head.bias.dtype == h.dtype))


class DecodeStep:
    """Static-buffer decode step (B sequences, 1 new token each).

    On the GPU the step is: native forward (qkv GEMV -> fused RoPE/KV over
    its split-K partials with device-side slots -> fused flash-decoding ->
    ...) -> lm_head GEMV -> ``decode_advance`` (greedy argmax, feed back the
    token, advance positions and precompute the next step's slots / key
    counts).  No framework glue kernels remain inside the captured graph."""

    def __init__(self, model: NativeCausalLM, cache: PagedKVCache, block_tables: torch.Tensor,
                 max_len: int, greedy: bool = True, use_graph: bool = True):
        from .. import ops
        self.model, self.cache = model, cache
        dev = model.device
        self.B = block_tables.shape[0]
        self.block_tables = block_tables.to(dev, torch.int32).contiguous()
        self.ids = torch.zeros(self.B, dtype=torch.long, device=dev)
        self.pos = torch.zeros(self.B, dtype=torch.long, device=dev)
        self.slots = torch.zeros(self.B, dtype=torch.long, device=dev)
        self.off = torch.zeros(self.B, dtype=torch.long, device=dev)      # compressed-KV position offsets
        self.seq_lens = torch.ones(self.B, dtype=torch.int32, device=dev)
        self.nsplit = nsplit_for(max_len)
        self.greedy = greedy
        self.logits: Optional[torch.Tensor] = None
        self.next_ids = torch.zeros(self.B, dtype=torch.long, device=dev)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.use_graph = use_graph and dev.type == "cuda"
        self.native_glue = dev.type == "cuda" and ops.native_gpu(self.ids)

    def _refresh(self):
        """slots / key counts for the current positions (eager, outside the graph)"""
        bs = self.cache.bs
        ci = self.pos - self.off
        blk = torch.gather(self.block_tables, 1, (ci // bs).unsqueeze(1)).squeeze(1).long()
        self.slots.copy_(blk * bs + ci % bs)
        self.seq_lens.copy_((ci + 1).to(torch.int32))

    def _body(self):
        meta = AttnMeta(self.B, 1, self.block_tables, self.seq_lens, self.nsplit, pos_offset=self.off)
        m = self.model
        if self.native_glue:
            h = m.forward_tokens(self.ids, self.pos, self.slots, meta, self.cache, return_hidden=True)
            head = m.lm_head
            if self.greedy and _argmax_head_ok(head, h, m.spec):
                # the lm_head GEMV writes per-wave argmax partials next to the
                # logits: decode_advance reduces ~V / 16 pairs, not V logits
                logits, parts = torch.ops.ipex_llm_amd.gemv_argmax(h.contiguous(), head.weight, head.fmt,
                                                                  head.out_features, head.in_features, head.bias)
                self.logits = logits
                torch.ops.ipex_llm_amd.decode_advance(None, self.ids, self.next_ids, self.pos, self.block_tables,
                                                      self.cache.bs, self.slots, self.seq_lens, self.off, parts)
                return
            logits = head(h.contiguous())
            if m.spec.final_softcap:
                logits = (torch.tanh(logits.float() / m.spec.final_softcap) * m.spec.final_softcap).to(h.dtype)
            self.logits = logits
            torch.ops.ipex_llm_amd.decode_advance(logits if self.greedy else None, self.ids, self.next_ids,
                                                  self.pos, self.block_tables, self.cache.bs, self.slots,
                                                  self.seq_lens, self.off)
            return
        logits = m.forward_tokens(self.ids, self.pos, self.slots, meta, self.cache)
        self.logits = logits
        if self.greedy:
            nxt = torch.argmax(logits, dim=-1)
            self.next_ids.copy_(nxt)
            self.ids.copy_(nxt)
        self.pos.add_(1)
        self._refresh()

    def capture(self):
        if not self.use_graph:
            return
        # warm up on a side stream (allocator + kernel JIT), then capture.
        # The warm-up really executes (writes K/V): point it at the last slot
        # of each sequence's allocation, which generation never reaches.
        ids0, pos0 = self.ids.clone(), self.pos.clone()
        last = self.block_tables.shape[1] * self.cache.bs - 2
        self.pos.fill_(last)
        self._refresh()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._body()
        torch.cuda.current_stream().wait_stream(s)
        self.ids.copy_(ids0)
        self.pos.fill_(last)
        self._refresh()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._body()
        # capture does not execute; restore the state written by the warm-up
        self.ids.copy_(ids0)
        self.pos.copy_(pos0)
        self._refresh()

    def set_state(self, ids: torch.Tensor, pos: torch.Tensor, off: Optional[torch.Tensor] = None):
        self.ids.copy_(ids)
        self.pos.copy_(pos)
        if off is not None:
            self.off.copy_(off)
        else:
            self.off.zero_()
        self._refresh()

    def step(self):
        from ..utils.trace import trace_range
        with trace_range("decode_step"):
            if self.graph is not None:
                self.graph.replay()
            else:
                self._body()
        from .. import ops
        if ops.api.CHECK_KERNELS and self.native_glue:
            ops.check_kernel_errors(self.ids.device)          # debug: surface skipped bad indices
        return self.next_ids


@dataclass
class GenTiming:
    first_cost: float = 0.0            # s, prefill + first token
    rest_costs: List[float] = field(default_factory=list)

    @property
    def rest_cost_mean(self) -> float:
        return sum(self.rest_costs) / max(1, len(self.rest_costs))


def _sample(logits: torch.Tensor, do_sample: bool, temperature: float, top_k: int, top_p: float,
            generator=None) -> torch.Tensor:
    if not do_sample:
        return torch.argmax(logits, dim=-1)
    x = logits.float() / max(temperature, 1e-5)
    if top_k and top_k > 0:
        kth = torch.topk(x, min(top_k, x.shape[-1]), dim=-1).values[..., -1:]
        x = x.masked_fill(x < kth, float("-inf"))
    if top_p and top_p < 1.0:
        sx, si = torch.sort(x, descending=True, dim=-1)
        cp = torch.softmax(sx, -1).cumsum(-1)
        drop = cp - torch.softmax(sx, -1) > top_p
        sx = sx.masked_fill(drop, float("-inf"))
        x = torch.full_like(x, float("-inf")).scatter(-1, si, sx)
    return torch.multinomial(torch.softmax(x, -1), 1, generator=generator).squeeze(-1)


def apply_repetition_penalty(logits, seqs, penalty):
    if penalty == 1.0:
        return logits
    for b, s in enumerate(seqs):
        idx = torch.tensor(sorted(set(s)), device=logits.device, dtype=torch.long)
        sc = logits[b, idx]
        logits[b, idx] = torch.where(sc > 0, sc / penalty, sc * penalty)
    return logits


class Engine:
    """Owns a model + KV cache; runs prefill and (graph) decode."""

    def __init__(self, model: NativeCausalLM, block_size: int = 64, kv_fp8: int = 0):
        self.model = model
        self.block_size = block_size
        self.kv_fp8 = kv_fp8
        self._steps: Dict[Tuple[int, int], DecodeStep] = {}
        self._pf_graphs: Dict[Tuple[int, int, int], tuple] = {}
        self.cache: Optional[PagedKVCache] = None
        self._cache_key = None
        # prefill GEMMs on a resident dequantized shadow when HBM allows
        # (ops/gemm.py auto_dense_budget; ILLM_PREFILL_DENSE_GB overrides)
        self.prefill_dense_gb = 0.0
        p = next(iter(model.parameters()), None) if hasattr(model, "parameters") else None
        if p is None and hasattr(model, "buffers"):
            p = next(iter(model.buffers()), None)
        if p is not None and p.is_cuda:
            # bounded by half of the free HBM (as serving.engine.LLMEngine does)
            from ..ops.gemm import auto_dense_budget
            free, _ = torch.cuda.mem_get_info(p.device)
            self.prefill_dense_gb = auto_dense_budget(p.device, cap_gb=0.5 * free / 2 ** 30)

    def _ensure_cache(self, batch: int, max_len: int):
        blocks = batch * ((max_len + self.block_size - 1) // self.block_size)
        if self.cache is None or self.cache.num_blocks < blocks:
            self.cache = self.model.make_cache(max_len, batch, self.block_size, self.kv_fp8, num_blocks=blocks)
            self._steps.clear()
            self._pf_graphs.clear()
        else:
            self.cache.allocator = type(self.cache.allocator)(self.cache.num_blocks)
        return self.cache

    @torch.no_grad()
    def prefill(self, seq: SequenceState, ids: torch.Tensor, start: int = 0) -> torch.Tensor:
        """Run ids (1-D) for one sequence from position ``start``; returns last logits [1, V]."""
        from ..utils.trace import trace_range
        with trace_range(f"prefill[{ids.numel()}]"):
            return self._prefill(seq, ids, start)

    def _prefill(self, seq: SequenceState, ids: torch.Tensor, start: int = 0) -> torch.Tensor:
        m, c = self.model, self.cache
        dev = m.device
        n = ids.numel()
        pos = torch.arange(start, start + n, device=dev)
        slots = slots_for(seq, start, n, c.bs).to(dev)
        L = start + n
        bt = make_block_table([seq], len(seq.blocks), dev)
        meta = AttnMeta(1, n, bt, torch.tensor([L], dtype=torch.int32, device=dev), nsplit_for(L), [L])
        logits = m.forward_tokens(ids.to(dev), pos, slots, meta, c,
                                  logits_idx=torch.tensor([n - 1], device=dev))
        seq.length = L
        return logits

    @torch.no_grad()
    def prefill_batch(self, seqs: List[SequenceState], ids: torch.Tensor, use_graph: bool = False) -> torch.Tensor:
        """Prefill B equal-length prompts (ids [B, n]) in ONE forward: the
        projections run as [B*n, K] GEMMs (weights read once for the whole
        batch), attention per sequence.  Returns last-token logits [B, V].

        ``use_graph``: the forward is captured once per (B, n, blocks) shape
        as a hipGraph and replayed (token ids, cache slots and block table
        copied into its static inputs): the ~15 launches per layer leave the
        host path -- the first-token analogue of the decode-step graph.
        Dense native decoders on one GPU only (no MoE routing / TP / EP)."""
        m, c = self.model, self.cache
        dev = m.device
        B, n = ids.shape
        nb = max(len(s.blocks) for s in seqs)
        if use_graph and self._pf_graph_ok():
            key = (B, n, nb)
            ent = self._pf_graphs.get(key)
            fresh = ent is None
            if fresh:
                ent = self._prefill_buffers(B, n, nb)
            graph, ids_s, slots_s, bt_s, out, meta, pos, lidx = ent[:8]
            ids_s.copy_(ids.reshape(-1).to(dev), non_blocking=True)
            slots_s.copy_(torch.cat([slots_for(s, 0, n, c.bs) for s in seqs]).to(dev), non_blocking=True)
            bt_s.copy_(make_block_table(seqs, nb, dev))
            if fresh:
                # warm-up (lazy library state) writes exactly these sequences'
                # KV, then the capture (which does not execute)
                side = torch.cuda.Stream(device=dev)
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side):
                    m.forward_tokens(ids_s, pos, slots_s, meta, c, logits_idx=lidx)
                torch.cuda.current_stream(dev).wait_stream(side)
                graph = torch.cuda.CUDAGraph()
                from ..ops.gemm import pin_dense_shadows
                # the resident dequantized shadows the graph reads are pinned in its
                # entry: a later cache drop cannot free memory the replay still reads
                with pin_dense_shadows() as pins, torch.cuda.graph(graph):
                    out = m.forward_tokens(ids_s, pos, slots_s, meta, c, logits_idx=lidx)
                ent = (graph, ids_s, slots_s, bt_s, out, meta, pos, lidx, pins)
                self._pf_graphs[key] = ent
            graph.replay()
            for s in seqs:
                s.length = n
            return out.clone()
        pos = torch.arange(n, device=dev).repeat(B)
        slots = torch.cat([slots_for(s, 0, n, c.bs) for s in seqs]).to(dev)
        bt = make_block_table(seqs, nb, dev)
        meta = AttnMeta(B, n, bt, torch.full((B,), n, dtype=torch.int32, device=dev), nsplit_for(n), [n] * B)
        logits = m.forward_tokens(ids.reshape(-1).to(dev), pos, slots, meta, c,
                                  logits_idx=torch.arange(B, device=dev) * n + (n - 1))
        for s in seqs:
            s.length = n
        return logits

    def _pf_graph_ok(self) -> bool:
        m = self.model
        dev = getattr(m, "device", None)
        if dev is None or dev.type != "cuda" or getattr(m, "tp_group", None) is not None:
            return False
        from ..models.decoder import NativeMLP
        return all(isinstance(L.mlp, NativeMLP) for L in getattr(m, "layers", [])) and m.graph_max_batch() > 0

    def _prefill_buffers(self, B: int, n: int, nb: int):
        """static inputs of a captured prefill (graph / output filled on first use)"""
        dev = self.model.device
        ids_s = torch.zeros(B * n, dtype=torch.long, device=dev)
        slots_s = torch.zeros(B * n, dtype=torch.long, device=dev)
        bt_s = torch.zeros(B, nb, dtype=torch.int32, device=dev)
        pos = torch.arange(n, device=dev).repeat(B)
        meta = AttnMeta(B, n, bt_s, torch.full((B,), n, dtype=torch.int32, device=dev), nsplit_for(n), [n] * B)
        lidx = torch.arange(B, device=dev) * n + (n - 1)
        return None, ids_s, slots_s, bt_s, None, meta, pos, lidx

    @torch.no_grad()
    def forward_chunk(self, seq: SequenceState, tokens: Sequence[int], start: int) -> torch.Tensor:
        """Run ``tokens`` of one sequence at positions start.. (KV written,
        ``seq.length`` = start + n); returns f32 logits for every token [n, V].
        Used by speculative / lookup verification: rejected tail positions are
        simply overwritten later (the paged cache is position-addressed)."""
        m, c = self.model, self.cache
        dev = m.device
        n = len(tokens)
        pos = torch.arange(start, start + n, device=dev)
        slots = slots_for(seq, start, n, c.bs).to(dev)
        L = start + n
        bt = make_block_table([seq], len(seq.blocks), dev)
        meta = AttnMeta(1, n, bt, torch.tensor([L], dtype=torch.int32, device=dev), nsplit_for(L), [L])
        logits = m.forward_tokens(torch.tensor(list(tokens), dtype=torch.long, device=dev), pos, slots, meta, c,
                                  logits_idx=torch.arange(n, device=dev))
        seq.length = L
        return logits

    def new_sequence(self, max_len: int) -> SequenceState:
        return SequenceState(self.cache.allocator.alloc((max_len + self.block_size - 1) // self.block_size))

    @torch.no_grad()
    def decode_step_obj(self, seqs: List[SequenceState], max_len: int, greedy: bool, use_graph: bool):
        gmax = self.model.graph_max_batch() if hasattr(self.model, "graph_max_batch") else 16
        use_graph = use_graph and len(seqs) <= gmax
        key = (len(seqs), max(len(s.blocks) for s in seqs), greedy, use_graph)
        st = self._steps.get(key)
        bt = make_block_table(seqs, key[1], self.model.device)
        if st is None:
            st = DecodeStep(self.model, self.cache, bt, key[1] * self.block_size, greedy, use_graph)
            st.capture()
            self._steps[key] = st
        else:
            st.block_tables.copy_(bt)
        return st

    @torch.no_grad()
    def generate(self, prompts: Sequence[Sequence[int]], max_new_tokens: int = 32, min_new_tokens: int = 0,
                 do_sample: bool = False, temperature: float = 1.0, top_k: int = 0, top_p: float = 1.0,
                 repetition_penalty: float = 1.0, eos_token_id=None, streamer=None, use_graph: bool = True,
                 timing: Optional[GenTiming] = None, generator=None, compress_kv: Optional[bool] = None,
                 compress_capacity: Optional[int] = None, compress_window: Optional[int] = None,
                 logits_processor=None) -> List[List[int]]:
        dev = self.model.device
        B = len(prompts)
        max_len = max(len(p) for p in prompts) + max_new_tokens + 1
        self._ensure_cache(B, max_len)
        nblk = (max_len + self.block_size - 1) // self.block_size
        seqs = [SequenceState(self.cache.allocator.alloc(nblk)) for _ in range(B)]
        eos = set([eos_token_id] if isinstance(eos_token_id, int) else (eos_token_id or []))
        sync = (lambda: torch.cuda.synchronize()) if dev.type == "cuda" else (lambda: None)
        from ..utils.settings import get_settings
        cfg = get_settings()
        compress = cfg.compress_kv_cache if compress_kv is None else compress_kv
        cap = compress_capacity or cfg.compress_kv_capacity
        win = compress_window or cfg.compress_kv_window
        offs = [0] * B
        t0 = time.perf_counter()
        last = []
        for b, p in enumerate(prompts):
            snap = compress and len(p) > cap
            if snap:
                self.model._capture_q, self.model._capture_w = {}, win
            try:
                lg = self.prefill(seqs[b], torch.tensor(list(p), dtype=torch.long))
            finally:
                qw, self.model._capture_q = self.model._capture_q, None
            if snap:
                from .compress_kv import snapkv_compress
                snapkv_compress(self.model, self.cache, seqs[b], len(p), qw, cap, win)
                offs[b] = len(p) - cap
            lg = apply_repetition_penalty(lg, [list(p)], repetition_penalty)
            if logits_processor is not None:
                lg = logits_processor(torch.tensor([list(p)], device=lg.device), lg.float())
            last.append(_sample(lg, do_sample, temperature, top_k, top_p, generator))
        cur = torch.cat(last).to(dev)
        out = [list(p) for p in prompts]
        done = [False] * B
        toks = cur.tolist()
        for b in range(B):
            out[b].append(toks[b])
            done[b] = toks[b] in eos and min_new_tokens <= 1
        sync()
        if timing is not None:
            timing.first_cost = time.perf_counter() - t0
        if streamer is not None:
            streamer.put(torch.tensor(toks))
        greedy = not do_sample and repetition_penalty == 1.0 and logits_processor is None
        st = self.decode_step_obj(seqs, max_len, greedy, use_graph)
        st.set_state(cur, torch.tensor([s.length + o for s, o in zip(seqs, offs)], device=dev),
                     torch.tensor(offs, device=dev))
        for i in range(1, max_new_tokens):
            if all(done):
                break
            t1 = time.perf_counter()
            nxt = st.step()
            if not greedy:
                lg = apply_repetition_penalty(st.logits.float().clone(), out, repetition_penalty)
                if logits_processor is not None:
                    width = max(len(o) for o in out)
                    ids_t = torch.tensor([o + [o[-1]] * (width - len(o)) for o in out], device=lg.device)
                    lg = logits_processor(ids_t, lg)
                nxt = _sample(lg, do_sample, temperature, top_k, top_p, generator)
                st.ids.copy_(nxt)
            toks = nxt.tolist()
            if timing is not None:
                timing.rest_costs.append(time.perf_counter() - t1)
            for b in range(B):
                if not done[b]:
                    out[b].append(toks[b])
                    if toks[b] in eos and i + 1 >= min_new_tokens:
                        done[b] = True
            if streamer is not None:
                streamer.put(torch.tensor(toks))
        if streamer is not None:
            streamer.end()
        for s in seqs:
            self.cache.allocator.release(s.blocks)
        return out
