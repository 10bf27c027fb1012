"""Self-speculative decoding as ONE hipGraph per draft length.

Reference: ``SRC/transformers/speculative.py:805-1271`` (draft with the
INT4 copy, verify with the fp16/bf16 target, crop the caches).  The
reference loop synchronises with the host for every drafted token (its stop
threshold reads the draft probability) and again for acceptance.

MI355X design: the whole iteration lives on the device and is captured once:

    draft   k forwards of the INT4 model: [token at p - 1, last], then
            d1 .. d(k-1) -- re-feeding position p - 1 writes d_k's KV when
            the previous round accepted everything, so no catch-up forward
    verify  one target forward over [last, d1 .. dk] (k + 1 query rows:
            skinny GEMV projections, flash-decoding / prefill attention
            reading the paged cache, device-side slots)
    accept  pred = argmax(logits); m = leading matches of d vs pred;
            emitted = pred[0 .. m]; positions, ``last`` and the output ring
            advance by m + 1 -- all tensor ops on device scalars

Both caches are position-addressed, so rejected tails are simply overwritten
by later rounds (no crop).  The host replays the graph and reads one int per
round (tokens emitted so far) to stop at ``max_new_tokens`` / EOS.  Greedy
output equals the target model's greedy decoding (up to ties between the
T = 1 and T = k + 1 GEMV reductions).
"""
from __future__ import annotations

import time
from typing import List, Optional, Sequence

import torch

from ..engine.runner import nsplit_for
from ..models.cache import SequenceState, make_block_table
from ..models.decoder import AttnMeta


class GraphSpeculator:
    """``k``: initial draft length; ``adaptive``: grow k after a fully
    accepted round, shrink it after a round that kept less than half (the
    reference's max_step_draft auto-tuning, speculative.py:1010-1040) --
    one captured graph per k in [1, k_max]."""

    def __init__(self, target_engine, draft_engine, k: int, max_len: int, use_graph: bool = True,
                 k_max: Optional[int] = None, adaptive: bool = True):
        self.te, self.de = target_engine, draft_engine
        self.tm, self.dm = target_engine.model, draft_engine.model
        self.k = k
        self.k_max = k_max or k
        self.adaptive = adaptive
        self.max_len = max_len
        dev = self.tm.device
        self.dev = dev
        self.use_graph = use_graph and dev.type == "cuda"
        self.graphs = {}
        self.warm = set()
        self.p = torch.zeros(1, dtype=torch.long, device=dev)          # position of `last`
        self.last = torch.zeros(1, dtype=torch.long, device=dev)
        self.prev = torch.zeros(1, dtype=torch.long, device=dev)      # token at position p - 1
        self.ar1 = torch.arange(2, device=dev)
        self.one = torch.ones(1, dtype=torch.long, device=dev)
        self.n_out = torch.zeros((), dtype=torch.long, device=dev)
        self.n_match = torch.zeros((), dtype=torch.long, device=dev)
        self.rounds = 0
        self.drafted = 0
        self.out = torch.zeros(max_len + 2 * self.k_max + 2, dtype=torch.long, device=dev)
        self.ars = {j: torch.arange(j + 1, device=dev) for j in range(1, self.k_max + 1)}

    def _slots(self, bt, pos, bs):
        return bt[0].long()[pos // bs] * bs + pos % bs

    def _iter(self, k: int):
        bs_t, bs_d = self.te.cache.bs, self.de.cache.bs
        ar = self.ars[k]
        # draft step 0 feeds [token at p - 1, last]: re-writing p - 1 is a no-op
        # unless the previous round accepted every draft (then d_k's KV was
        # never written) -- so k draft forwards suffice, no catch-up step
        ids0 = torch.cat([self.prev, self.last])
        pos0 = self.p - 1 + self.ar1
        meta = AttnMeta(1, 2, self.bt_d, (self.p + 1).to(torch.int32), self.ns)
        lg = self.dm.forward_tokens(ids0, pos0, self._slots(self.bt_d, pos0, bs_d), meta, self.de.cache,
                                    logits_idx=self.one)
        tok = torch.argmax(lg, dim=-1)
        drafts = [tok]
        for j in range(1, k):
            pos = self.p + j
            meta = AttnMeta(1, 1, self.bt_d, (pos + 1).to(torch.int32), self.ns)
            lg = self.dm.forward_tokens(tok, pos, self._slots(self.bt_d, pos, bs_d), meta, self.de.cache)
            tok = torch.argmax(lg, dim=-1)
            drafts.append(tok)
        d = torch.cat(drafts)                                         # d1 .. dk
        ids = torch.cat([self.last, d])
        pos = self.p + ar
        meta = AttnMeta(1, k + 1, self.bt_t, (self.p + k + 1).to(torch.int32), self.ns)
        lg = self.tm.forward_tokens(ids, pos, self._slots(self.bt_t, pos, bs_t), meta, self.te.cache)
        pred = torch.argmax(lg, dim=-1)                              # [k + 1]
        m = torch.cumprod((d == pred[:k]).long(), 0).sum()
        self.out.index_copy_(0, self.n_out + ar, pred)
        self.n_out.add_(m + 1)
        self.n_match.add_(m)
        self.p.add_(m + 1)
        self.prev.copy_(ids.gather(0, m.view(1)))                    # token now at p - 1
        self.last.copy_(pred.gather(0, m.view(1)))

    @torch.no_grad()
    def generate(self, prompt: Sequence[int], max_new_tokens: int, eos=(), timing=None, streamer=None,
                 min_new_tokens: int = 0) -> List[int]:
        """Greedy speculative generation of one prompt.  Stops like the eager
        path (generation/speculative.py): at ``max_new_tokens``, or at an EOS
        once ``min_new_tokens`` tokens exist; only the tokens kept are
        streamed.  The caller ends the streamer."""
        te, de = self.te, self.de
        te._ensure_cache(1, self.max_len)
        de._ensure_cache(1, self.max_len)
        st, sd = te.new_sequence(self.max_len), de.new_sequence(self.max_len)
        bt_t = make_block_table([st], len(st.blocks), self.dev)
        bt_d = make_block_table([sd], len(sd.blocks), self.dev)
        key = (id(te.cache), id(de.cache), bt_t.shape, bt_d.shape)
        if getattr(self, "_key", None) != key:
            # graphs bake in the cache tensors and block-table buffers
            self._key = key
            self.graphs, self.warm = {}, set()
            self.bt_t, self.bt_d = bt_t, bt_d
            self.pool = torch.cuda.graph_pool_handle() if self.use_graph else None
        else:
            self.bt_t.copy_(bt_t)
            self.bt_d.copy_(bt_d)
        self.ns = nsplit_for(self.max_len)
        sync = torch.cuda.synchronize if self.dev.type == "cuda" else (lambda: None)
        p = list(prompt)
        t0 = time.perf_counter()
        first = torch.argmax(te.forward_chunk(st, p, 0)[-1])
        de.forward_chunk(sd, p, 0)
        self.p.fill_(len(p))
        self.prev.fill_(p[-1])
        self.last.copy_(first.view(1))
        self.n_out.zero_()
        self.n_match.zero_()
        self.out[0] = first
        self.n_out.fill_(1)
        sync()
        if timing is not None:
            timing.first_cost = time.perf_counter() - t0
        eos = set(eos or ())
        got, emitted = 1, [int(first)]
        done = max_new_tokens <= 1 or (emitted[-1] in eos and 1 >= min_new_tokens)
        if streamer is not None:
            streamer.put(first.view(1).cpu())
        self.rounds = self.drafted = 0
        while not done:
            t1 = time.perf_counter()
            k = self.k
            g = self.graphs.get(k)
            if g is not None:
                g.replay()
            elif self.use_graph and k in self.warm:
                # this k ran once eagerly (allocator / kernel warm-up): capture now
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self.pool):
                    self._iter(k)
                self.graphs[k] = g
                g.replay()
            elif self.use_graph:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    self._iter(k)
                torch.cuda.current_stream().wait_stream(s)
                self.warm.add(k)
            else:
                self._iter(k)
            self.rounds += 1
            self.drafted += k
            n = int(self.n_out)                                      # the round's one host read
            new = self.out[got:n].tolist()
            if self.adaptive:
                m = len(new) - 1
                if m >= k and k < self.k_max:
                    self.k = k + 1
                elif m < k // 2 and k > 1:
                    self.k = k - 1
            got = n
            kept = []
            for t in new:                       # the eager path's stop rule, token by token
                kept.append(t)
                if len(emitted) + len(kept) >= max_new_tokens or (t in eos and len(emitted) + len(kept) >= min_new_tokens):
                    done = True
                    break
            emitted.extend(kept)
            if timing is not None:
                dt = time.perf_counter() - t1
                timing.rest_costs.extend([dt / max(1, len(kept))] * len(kept))
            if streamer is not None and kept:
                streamer.put(torch.tensor(kept))
        te.cache.allocator.release(st.blocks)
        de.cache.allocator.release(sd.blocks)
        return p + emitted

    @property
    def acceptance(self) -> float:
        return float(self.n_match) / max(1, self.drafted)


def max_graph_draft(model) -> int:
    """largest k for which the k + 1-row verify stays on capture-safe kernels"""
    s = model.spec
    group = max(1, s.num_heads // s.num_kv_heads)
    if s.head_dim in (64, 128):
        return 15                         # attn_decode (<= 16 rows x group) or the paged prefill kernel
    return max(1, 16 // group - 1)
