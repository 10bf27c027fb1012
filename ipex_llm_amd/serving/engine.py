"""Continuous-batching LLM engine for serving.

Reference: ``SRC/serving/fastapi/model_worker.py`` (one request at a time
through HF ``generate`` + ``TextIteratorStreamer``) and the vLLM engine
integration (``SRC/vllm/xpu/engine/engine.py``).

MI355X design: requests share one paged KV pool sized from free HBM (288 GB
holds thousands of 8K-token Llama-3-8B sequences); the C++ scheduler
(``csrc/runtime/scheduler.cpp``) decides per step which sequences are
prefilled / decoded / preempted; every decode step is ONE batched native
forward over all running sequences (flash-decoding over their own block
tables), so throughput scales with concurrency instead of serialising
requests.
"""
from __future__ import annotations

import itertools
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import torch

from .. import ops
from ..engine.runner import _sample, apply_repetition_penalty, nsplit_for
from ..models.cache import PagedKVCache
from ..models.decoder import AttnMeta, NativeCausalLM


@dataclass
class SamplingParams:
    max_new_tokens: int = 32
    min_new_tokens: int = 0
    temperature: float = 1.0
    top_k: int = 0
    top_p: float = 1.0
    do_sample: bool = False
    repetition_penalty: float = 1.0
    stop_token_ids: List[int] = field(default_factory=list)
    seed: Optional[int] = None
    ignore_eos: bool = False          # run to max_new_tokens through EOS (stop_token_ids still stop)


@dataclass
class Request:
    rid: int
    prompt: List[int]
    params: SamplingParams
    tokens: List[int] = field(default_factory=list)     # prompt + generated
    generated: List[int] = field(default_factory=list)
    finished: bool = False
    finish_reason: Optional[str] = None
    arrival: float = 0.0
    first_token_time: Optional[float] = None
    on_token: Optional[Callable[[int, "Request"], None]] = None
    generator: Optional[torch.Generator] = None


class LLMEngine:
    def __init__(self, model: NativeCausalLM, max_batch: int = 64, block_size: int = 64,
                 num_blocks: Optional[int] = None, max_model_len: int = 8192, max_prefill_tokens: int = 8192,
                 kv_fp8: int = 0, memory_fraction: float = 0.5, eos_token_id=None, use_graph: bool = True,
                 enable_prefix_caching: bool = True, tp_group="auto"):
        ops.require() if model.device.type == "cuda" else None
        self.model = model
        s = model.spec
        # tensor-parallel serving (reference: vLLM --tensor-parallel-size,
        # SRC/vllm/xpu/model_convert.py:36-75): one process per GPU, each with its
        # shard of the model and of the KV cache.  Rank 0 (the driver) owns the
        # requests and the C++ scheduler and broadcasts each step's plan (token
        # ids, positions, block tables); every rank runs the same forwards --
        # the row-parallel all-reduces and the vocab-parallel logits gather
        # happen inside them -- and only the driver samples.  Ranks > 0 sit in
        # run_worker().
        self.tp_group = getattr(model, "tp_group", None) if tp_group == "auto" else tp_group
        self.tp_world, self.tp_rank = 1, 0
        if self.tp_group is not None:
            import torch.distributed as dist
            self.tp_world, self.tp_rank = dist.get_world_size(self.tp_group), dist.get_rank(self.tp_group)
            if self.tp_world == 1:
                self.tp_group = None
        self.is_driver = self.tp_rank == 0
        self._stopped = False
        if num_blocks is None:
            per_tok = PagedKVCache.bytes_per_token(len(model.layers), s.num_kv_heads, s.head_dim, model.dtype, kv_fp8)
            if model.device.type == "cuda":
                free, _ = torch.cuda.mem_get_info(model.device)
                budget = int(free * memory_fraction)
            else:
                budget = per_tok * max_batch * max_model_len // 4
            num_blocks = max(max_batch, budget // (per_tok * block_size))
            num_blocks = min(num_blocks, max_batch * ((max_model_len + block_size - 1) // block_size))
            if self.tp_group is not None:      # one block layout on every rank: the smallest pool
                num_blocks = int(self._tp_reduce_min(num_blocks))
        # one extra block past the scheduler's pool: the scratch target of the
        # padding rows of a captured decode step
        self.cache = model.make_cache(max_model_len, max_batch, block_size, kv_fp8, num_blocks=num_blocks + 1)
        self._scratch = num_blocks
        self.num_blocks = num_blocks
        # prefill GEMMs on a resident dequantized shadow (ops/gemm.py
        # auto_dense_budget), bounded by half of what the KV pool left free
        self.prefill_dense_gb = 0.0
        if model.device.type == "cuda":
            from ..ops.gemm import auto_dense_budget
            free, _ = torch.cuda.mem_get_info(model.device)
            self.prefill_dense_gb = auto_dense_budget(model.device, cap_gb=0.5 * free / 2 ** 30)
        from .metrics import EngineMetrics
        self.metrics = EngineMetrics()
        self.use_graph = use_graph and model.device.type == "cuda" and ops.native_gpu(self.cache.k[0])
        self._graphs: Dict[tuple, dict] = {}
        # every captured (batch, width) bucket allocates from ONE private pool,
        # and only buckets whose forward is capture-safe are captured (MoE
        # routing / SDPA fallbacks above the model's limit run eagerly)
        self._graph_pool = None
        self._graph_max_b = model.graph_max_batch() if hasattr(model, "graph_max_batch") else 16
        model.ensure_rope_cache(max_model_len + 1)
        self.sched = torch.classes.ipex_llm_amd.Scheduler(num_blocks, block_size, max_batch, max_prefill_tokens)
        # automatic prefix caching: full KV blocks are shared by content hash
        # (C++ scheduler); a request prefills only its uncached suffix
        self.prefix_caching = bool(enable_prefix_caching)
        self.sched.enable_prefix_caching(self.prefix_caching)
        self.block_size, self.max_model_len = block_size, max_model_len
        eos = eos_token_id if eos_token_id is not None else []
        self.eos = set([eos] if isinstance(eos, int) else eos)
        self.requests: Dict[int, Request] = {}
        self._ids = itertools.count()
        self.lock = threading.Lock()
        self.stats = {"steps": 0, "prefill_tokens": 0, "decode_tokens": 0, "preemptions": 0,
                      "prefix_hit_tokens": 0}

    # ------------------------------------------------------------ API
    def add_request(self, prompt: List[int], params: Optional[SamplingParams] = None,
                    on_token: Optional[Callable] = None) -> int:
        params = params or SamplingParams()
        if len(prompt) + params.max_new_tokens > self.max_model_len:
            raise ValueError(f"prompt ({len(prompt)}) + max_new_tokens exceeds max_model_len={self.max_model_len}")
        with self.lock:
            rid = next(self._ids)
            g = None
            if params.seed is not None:
                g = torch.Generator(device=self.model.device).manual_seed(params.seed)
            r = Request(rid, list(prompt), params, tokens=list(prompt), arrival=time.perf_counter(),
                        on_token=on_token, generator=g)
            self.requests[rid] = r
            if self.prefix_caching:
                self.sched.add_tokens(rid, [int(t) for t in prompt])
            else:
                self.sched.add(rid, len(prompt))
        self.metrics.on_request(len(prompt))
        return rid

    def abort(self, rid: int):
        with self.lock:
            r = self.requests.get(rid)
            if r is not None and not r.finished:
                self._finish(r, "abort")

    def has_work(self) -> bool:
        # a snapshot: request threads add / pop entries while the loop polls
        return any(not r.finished for r in list(self.requests.values()))

    # ------------------------------------------------------------ step
    def _finish(self, r: Request, reason: str):
        r.finished, r.finish_reason = True, reason
        self.metrics.on_finish(reason, time.perf_counter() - r.arrival, len(r.generated), r.first_token_time)
        try:
            self.sched.finish(r.rid)
        except RuntimeError:
            pass
        if r.on_token is not None:
            r.on_token(-1, r)

    def _emit(self, r: Request, tok: int):
        r.tokens.append(tok)
        r.generated.append(tok)
        if r.first_token_time is None:
            r.first_token_time = time.perf_counter() - r.arrival
            self.metrics.on_first_token(r.first_token_time)
        if self.prefix_caching:
            self.sched.append(r.rid, int(tok))
        else:
            self.sched.grow(r.rid)
        if r.on_token is not None:
            r.on_token(tok, r)
        p = r.params
        n = len(r.generated)
        if n >= p.max_new_tokens:
            self._finish(r, "length")
        elif n >= p.min_new_tokens and ((tok in self.eos and not p.ignore_eos) or tok in p.stop_token_ids):
            self._finish(r, "stop")

    def _pick(self, logits: torch.Tensor, r: Request) -> int:
        p = r.params
        if p.repetition_penalty != 1.0:
            logits = apply_repetition_penalty(logits.clone(), [r.tokens], p.repetition_penalty)
        return int(_sample(logits, p.do_sample, p.temperature, p.top_k, p.top_p, r.generator)[0])

    def _block_table(self, rids: List[int]) -> torch.Tensor:
        rows = [list(self.sched.blocks(r)) for r in rids]
        w = max(len(x) for x in rows)
        t = torch.zeros(len(rows), w, dtype=torch.int32)
        for i, x in enumerate(rows):
            t[i, :len(x)] = torch.tensor(x, dtype=torch.int32)
        return t.to(self.model.device)

    # ------------------------------------------------------------ tensor parallel
    def _tp_device(self):
        import torch.distributed as dist
        return self.model.device if dist.get_backend(self.tp_group) == "nccl" else torch.device("cpu")

    def _tp_reduce_min(self, v: int) -> int:
        import torch.distributed as dist
        t = torch.tensor([int(v)], dtype=torch.int64, device=self._tp_device())
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.tp_group)
        return int(t.item())

    def _tp_bcast(self, plan: Optional[List[int]]) -> List[int]:
        """the driver's step plan to every rank (length, then the int64 words)"""
        import torch.distributed as dist
        dev, src = self._tp_device(), dist.get_global_rank(self.tp_group, 0)
        n = torch.tensor([len(plan) if plan is not None else 0], dtype=torch.int64, device=dev)
        dist.broadcast(n, src, group=self.tp_group)
        buf = torch.tensor(plan, dtype=torch.int64, device=dev) if plan is not None else \
            torch.empty(int(n.item()), dtype=torch.int64, device=dev)
        dist.broadcast(buf, src, group=self.tp_group)
        return buf.tolist() if plan is None else plan

    @staticmethod
    def encode_plan(prefill, decode) -> List[int]:
        """[1, #prefill, #decode, (n, start, #blocks, tokens[start:n], blocks)...,
        (id, pos, #blocks, blocks)...]; [0] stops the workers"""
        out = [1, len(prefill), len(decode)]
        for toks, start, blocks in prefill:
            out += [len(toks), start, len(blocks)] + list(toks[start:]) + list(blocks)
        for tok, pos, blocks in decode:
            out += [tok, pos, len(blocks)] + list(blocks)
        return out

    @staticmethod
    def decode_plan(words: List[int]):
        if not words or words[0] == 0:
            return None
        i, prefill, decode = 3, [], []
        for _ in range(words[1]):
            n, start, nb = words[i:i + 3]
            i += 3
            suffix = words[i:i + n - start]
            i += n - start
            prefill.append(([0] * start + suffix, start, words[i:i + nb]))
            i += nb
        for _ in range(words[2]):
            tok, pos, nb = words[i:i + 3]
            i += 3
            decode.append((tok, pos, words[i:i + nb]))
            i += nb
        return prefill, decode

    @torch.no_grad()
    def run_worker(self):
        """ranks > 0: execute the driver's plans until it stops the group"""
        assert self.tp_group is not None and not self.is_driver, "run_worker: tensor-parallel ranks > 0 only"
        while True:
            plan = self.decode_plan(self._tp_bcast(None))
            if plan is None:
                return
            prefill, decode = plan
            for toks, start, blocks in prefill:
                self._exec_prefill(toks, start, blocks)
            if decode:
                self._exec_decode([d[0] for d in decode], [d[1] for d in decode], [d[2] for d in decode])

    def shutdown(self):
        """driver: release the tensor-parallel workers (idempotent)"""
        if self.tp_group is not None and self.is_driver and not self._stopped:
            self._stopped = True
            self._tp_bcast([0])

    # ------------------------------------------------------------ graph decode
    @staticmethod
    def _bucket(x: int, lo: int = 1) -> int:
        b = lo
        while b < x:
            b *= 2
        return b

    def _capture(self, Bb: int, Wb: int) -> dict:
        """hipGraph of one decode forward for Bb sequences (padded) with block
        tables of Wb blocks: slots / key counts are derived on the device from
        the positions, so a replay needs only ids, positions and tables."""
        m, bs, dev = self.model, self.block_size, self.model.device
        g = {"ids": torch.zeros(Bb, dtype=torch.long, device=dev),
             "pos": torch.zeros(Bb, dtype=torch.long, device=dev),
             "bt": torch.full((Bb, Wb), self._scratch, dtype=torch.int32, device=dev)}

        def body():
            pos, bt = g["pos"], g["bt"]
            blk = torch.gather(bt, 1, (pos // bs).unsqueeze(1)).squeeze(1).long()
            slots = blk * bs + pos % bs
            seq_lens = (pos + 1).to(torch.int32)
            meta = AttnMeta(Bb, 1, bt, seq_lens, nsplit_for(Wb * bs))
            return m.forward_tokens(g["ids"], pos, slots, meta, self.cache)

        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):            # warm-up (writes only the scratch block)
            body()
        torch.cuda.current_stream().wait_stream(s)
        g["graph"] = torch.cuda.CUDAGraph()
        if self._graph_pool is None:
            self._graph_pool = torch.cuda.graph_pool_handle()
        with torch.cuda.graph(g["graph"], pool=self._graph_pool):
            g["logits"] = body()
        self._graphs[(Bb, Wb)] = g
        return g

    def _decode_graph(self, ids_l: List[int], pos_l: List[int], rows: List[List[int]]) -> torch.Tensor:
        B = len(ids_l)
        Bb = self._bucket(B)
        Wb = self._bucket(max(len(x) for x in rows), 4)
        g = self._graphs.get((Bb, Wb)) or self._capture(Bb, Wb)
        bt = torch.full((Bb, Wb), self._scratch, dtype=torch.int32)
        for i, x in enumerate(rows):
            bt[i, :len(x)] = torch.tensor(x, dtype=torch.int32)
        pos = torch.zeros(Bb, dtype=torch.long)
        pos[:B] = torch.tensor(pos_l)
        ids = torch.zeros(Bb, dtype=torch.long)
        ids[:B] = torch.tensor(ids_l)
        g["bt"].copy_(bt, non_blocking=True)
        g["pos"].copy_(pos, non_blocking=True)
        g["ids"].copy_(ids, non_blocking=True)
        g["graph"].replay()
        return g["logits"][:B]

    def _exec_prefill(self, toks: List[int], start: int, blocks: List[int]) -> torch.Tensor:
        """forward of toks[start:] over the cached prefix; last-position logits"""
        m, dev, bs = self.model, self.model.device, self.block_size
        n = len(toks)
        tq = n - start
        bt = torch.tensor([list(blocks)], dtype=torch.int32).to(dev)
        pos_h = torch.arange(start, n)
        bl = torch.tensor(list(blocks), dtype=torch.long)
        slots = (bl[pos_h // bs] * bs + pos_h % bs).to(dev)
        meta = AttnMeta(1, tq, bt, torch.tensor([n], dtype=torch.int32, device=dev), nsplit_for(n), [n])
        return m.forward_tokens(torch.tensor(toks[start:], device=dev), pos_h.to(dev), slots, meta,
                                self.cache, logits_idx=torch.tensor([tq - 1], device=dev))

    def _exec_decode(self, ids_l: List[int], pos_l: List[int], rows: List[List[int]]) -> torch.Tensor:
        """one decode forward of len(ids_l) sequences (graph bucket or eager)"""
        m, dev, bs = self.model, self.model.device, self.block_size
        B = len(ids_l)
        if self.use_graph and self._bucket(B) <= self._graph_max_b:
            return self._decode_graph(ids_l, pos_l, rows)
        w = max(len(x) for x in rows)
        bt = torch.zeros(B, w, dtype=torch.int32)
        for i, x in enumerate(rows):
            bt[i, :len(x)] = torch.tensor(list(x), dtype=torch.int32)
        bt = bt.to(dev)
        pos = torch.tensor(pos_l, device=dev)
        blk = torch.gather(bt, 1, (pos // bs).unsqueeze(1).to(torch.int64)).squeeze(1).long()
        slots = blk * bs + pos % bs
        seq_lens = (pos + 1).to(torch.int32)
        meta = AttnMeta(B, 1, bt, seq_lens, nsplit_for(max(pos_l) + 1), [p + 1 for p in pos_l])
        return m.forward_tokens(torch.tensor(ids_l, device=dev), pos, slots, meta, self.cache)

    @torch.no_grad()
    def step(self) -> int:
        """One scheduler step: prefill admitted requests, decode all running
        ones.  Returns the number of tokens produced."""
        from ..utils.trace import trace_range
        with trace_range("engine_step"):
            return self._step()

    def _step(self) -> int:
        if not self.is_driver:
            raise RuntimeError("LLMEngine.step: tensor-parallel ranks > 0 run run_worker(), not step()")
        t_step = time.perf_counter()
        with self.lock:
            plan = list(self.sched.schedule())
            i1 = plan.index(-1)
            i2 = plan.index(-1, i1 + 1)
            i3 = plan.index(-1, i2 + 1)
            prefill, decode, preempted, failed = plan[:i1], plan[i1 + 1:i2], plan[i2 + 1:i3], plan[i3 + 1:]
            self.stats["preemptions"] += len(preempted)
            for rid in failed:
                r = self.requests[rid]
                r.finished, r.finish_reason = True, "error: request does not fit in the KV cache"
                if r.on_token is not None:
                    r.on_token(-1, r)
            produced = 0
            pre = []
            for rid in prefill:
                toks = self.requests[rid].tokens
                pre.append((toks, int(self.sched.cached(rid)), list(self.sched.blocks(rid))))
            dec = [(self.requests[rid].tokens[-1], int(self.sched.cached(rid)), list(self.sched.blocks(rid)))
                   for rid in decode]
            if self.tp_group is not None and (pre or dec):
                self._tp_bcast(self.encode_plan(pre, dec))
            for rid, (toks, start, blocks) in zip(prefill, pre):
                r = self.requests[rid]
                n = len(toks)
                tq = n - start                               # prefix already in cached KV blocks
                lg = self._exec_prefill(toks, start, blocks)
                self.sched.advance(rid, tq)
                self.stats["prefill_tokens"] += tq
                self.stats["prefix_hit_tokens"] += start
                self.metrics.on_prefill(tq)
                self.metrics.on_prefix_hit(start)
                self._emit(r, self._pick(lg, r))
                produced += 1
            if decode:
                rs = [self.requests[rid] for rid in decode]
                B = len(rs)
                lg = self._exec_decode([d[0] for d in dec], [d[1] for d in dec], [d[2] for d in dec])
                greedy = all(not r.params.do_sample and r.params.repetition_penalty == 1.0 for r in rs)
                nxt = torch.argmax(lg, -1).tolist() if greedy else None
                for i, r in enumerate(rs):
                    self.sched.advance(r.rid, 1)
                    self._emit(r, nxt[i] if greedy else self._pick(lg[i:i + 1], r))
                produced += B
                self.stats["decode_tokens"] += B
            self.stats["steps"] += 1
            self.metrics.on_tokens(produced)
            self.metrics.on_step(time.perf_counter() - t_step, int(self.sched.num_running()),
                                 int(self.sched.num_waiting()),
                                 1.0 - int(self.sched.num_free_blocks()) / max(1, self.num_blocks), len(preempted))
            return produced

    def generate(self, prompts: List[List[int]], params: Optional[SamplingParams] = None) -> List[List[int]]:
        """Offline batch: submit everything, run until done (continuous batching)."""
        rids = [self.add_request(p, params) for p in prompts]
        while any(not self.requests[r].finished for r in rids):
            self.step()
        out = [self.requests[r].generated for r in rids]
        for r in rids:
            self.requests.pop(r, None)
        return out


class EngineLoop:
    """Background thread driving ``LLMEngine.step`` for the API server."""

    def __init__(self, engine: LLMEngine, idle_sleep: float = 0.002):
        self.engine, self.idle = engine, idle_sleep
        self._stop = threading.Event()
        self.thread = threading.Thread(target=self._run, daemon=True)
        self.error: Optional[BaseException] = None

    def start(self):
        self.thread.start()
        return self

    def _run(self):
        while not self._stop.is_set():
            try:
                if self.engine.has_work():
                    self.engine.step()
                else:
                    time.sleep(self.idle)
            except BaseException as e:  # pragma: no cover - surfaced to requests
                self.error = e
                for r in list(self.engine.requests.values()):
                    if not r.finished:
                        r.finished, r.finish_reason = True, f"error: {e}"
                        if r.on_token is not None:
                            r.on_token(-1, r)

    def stop(self):
        self._stop.set()
        self.thread.join(timeout=5)
