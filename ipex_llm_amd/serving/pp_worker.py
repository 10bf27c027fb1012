"""Pipeline-parallel serving worker: continuously batched micro-batches kept
in flight across pipeline stages (one process per GPU).

Reference: ``SRC/transformers/pipeline_parallel.py:448-927`` -- ``PPModelWorker``
(rank 0 tokenizes and forms a ``BatchTask``, broadcasts it with
``broadcast_object_list``, keeps ``world_size`` batches in flight in
``on_going_batches``, partial prefill through ``max_prefilled_seqs``,
streamed output through per-request queues).

MI355X design: a global *tick* clock shared by every rank.  At tick t stage r
runs the micro-batch that entered the pipeline at tick t - r, so once W
micro-batches are in flight every stage is busy every tick.  A micro-batch owns
pipeline slot s = t mod W and re-enters stage 0 exactly W ticks after it
entered -- the tick right after the last stage sampled its next tokens.  Per
tick there are two small collectives (rank 0's control object, the last
stage's sampled tokens) and one point-to-point residual-stream hop per stage
boundary: the ``isend`` is posted this tick and received by the next stage on
the next tick, so no stage waits for its successor's compute.  Every stage owns
a paged KV cache for its own layer range (``models/cache.py``); sequence
membership and lengths are mirrored on every rank from the control stream, so
no KV metadata crosses a link.
"""
from __future__ import annotations

import itertools
import queue
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..engine.runner import _sample, apply_repetition_penalty, nsplit_for
from ..models.cache import SequenceState, make_block_table, slots_for
from ..models.decoder import AttnMeta
from ..parallel.comm import get_rank, get_world_size, is_dist
from .engine import SamplingParams


@dataclass
class _Seq:
    rid: int
    prompt_len: int
    tokens: List[int]
    params: SamplingParams
    state: SequenceState
    prefilled: int = 0                     # prompt tokens scheduled into the pipeline
    generated: List[int] = field(default_factory=list)
    done: bool = False
    finish_reason: Optional[str] = None
    arrival: float = 0.0
    first_token_time: Optional[float] = None
    generator: Optional[torch.Generator] = None


class PPModelWorker:
    """Micro-batched pipeline-parallel serving over a model already split by
    :func:`ipex_llm_amd.parallel.pipeline.pipeline_parallel` (or a native
    stage model with ``first_stage`` / ``last_stage`` set).

    Rank 0 drives: :meth:`add_request`, :meth:`process_step`,
    :meth:`generate`, :meth:`stop`.  Every other rank calls
    :meth:`serve_forever`, which returns when rank 0 calls :meth:`stop`.
    """

    def __init__(self, model, tokenizer=None, group=None, max_num_seqs: int = 8, max_prefilled_seqs: int = 0,
                 prefill_chunk: int = 0, max_model_len: int = 2048, block_size: int = 64, kv_fp8: int = 0,
                 num_blocks: Optional[int] = None, eos_token_id=None):
        from ..transformers.hf_native import get_native
        native = model if hasattr(model, "forward_tokens") else get_native(model)[0]
        self.model, self.tokenizer, self.group = native, tokenizer, group
        self.rank, self.world = get_rank(group), get_world_size(group)
        self.dev = native.device
        self.max_num_seqs, self.max_prefilled_seqs = max_num_seqs, max_prefilled_seqs
        self.prefill_chunk, self.max_model_len, self.bs = prefill_chunk, max_model_len, block_size
        per_seq = (max_model_len + block_size - 1) // block_size
        self.num_blocks = num_blocks or per_seq * max_num_seqs * self.world
        self.cache = native.make_cache(max_model_len, 1, block_size, kv_fp8, num_blocks=self.num_blocks)
        if eos_token_id is None and tokenizer is not None:
            eos_token_id = getattr(tokenizer, "eos_token_id", None)
        self.eos = set([eos_token_id] if isinstance(eos_token_id, int) else (eos_token_id or []))
        self.seqs: Dict[int, _Seq] = {}
        self.on_going: List[List[int]] = [[] for _ in range(self.world)]    # rids per pipeline slot
        self.waiting: deque = deque()
        self.pending: Dict[int, list] = {}          # tick -> calls that entered stage 0 at that tick
        self.tick = 0
        self.streamer: Dict[int, "queue.Queue[int]"] = {}
        self._sends: List[tuple] = []
        self._ids = itertools.count()
        self._lock = threading.Lock()
        self._stopped = False
        self.stats = {"ticks": 0, "bubbles": 0, "prefill_tokens": 0, "decode_tokens": 0}
        self.monitor = None                          # parallel.health.RankMonitor (rank 0)
        self.heartbeat = None
        self.failed: Optional[str] = None

    def enable_failure_detection(self, timeout: float = 5.0, interval: float = 0.5):
        """heartbeats on every rank, a monitor on rank 0 (parallel/health.py)"""
        from ..parallel.health import Heartbeat, RankMonitor, default_store
        store = default_store()
        if store is None or self.world == 1:
            return self
        self.heartbeat = Heartbeat(store, self._g(self.rank), interval).start()
        if self.is_head:
            self.monitor = RankMonitor(store, [self._g(r) for r in range(1, self.world)], timeout,
                                       poll=interval)
        return self

    def fail_all(self, reason: str):
        """finish every in-flight request with an error (streams woken)"""
        self.failed = reason
        for sq in list(self.seqs.values()):
            if not sq.done:
                sq.done, sq.finish_reason = True, f"error: {reason}"
                if self.is_head and sq.rid in self.streamer:
                    self.streamer[sq.rid].put(-1)
        while self.waiting:
            rid = self.waiting.popleft()
            sq = self.seqs.get(rid)
            if sq is not None and not sq.done:
                sq.done, sq.finish_reason = True, f"error: {reason}"
                if rid in self.streamer:
                    self.streamer[rid].put(-1)

    # ----------------------------------------------------------------- helpers
    @property
    def is_head(self) -> bool:
        return self.rank == 0

    @property
    def is_tail(self) -> bool:
        return self.rank == self.world - 1

    def _g(self, r: int) -> int:
        return dist.get_global_rank(self.group, r) if self.group is not None else r

    def _bcast(self, obj, src: int):
        if self.world == 1 or not is_dist():
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=self._g(src), group=self.group,
                                   device=self.dev if self.dev.type == "cuda" else None)
        return box[0]

    def _blocks_for(self, n_prompt: int, params: SamplingParams) -> int:
        return (n_prompt + params.max_new_tokens + self.bs - 1) // self.bs

    # ----------------------------------------------------------------- API (rank 0)
    def add_request(self, prompt, params: Optional[SamplingParams] = None, request_id: Optional[int] = None) -> int:
        """Queue a prompt (token ids, or text when a tokenizer was given).
        Tokens stream into ``self.streamer[rid]`` (-1 marks the end)."""
        if not self.is_head:
            raise RuntimeError("requests are submitted on pipeline rank 0")
        ids = self.tokenizer.encode(prompt) if isinstance(prompt, str) else [int(t) for t in prompt]
        params = params or SamplingParams()
        if len(ids) + params.max_new_tokens > self.max_model_len:
            raise ValueError(f"prompt ({len(ids)}) + max_new_tokens exceeds max_model_len={self.max_model_len}")
        if self._blocks_for(len(ids), params) > self.num_blocks:
            raise ValueError("request does not fit in the KV cache")
        with self._lock:
            rid = next(self._ids) if request_id is None else int(request_id)
            self.streamer[rid] = queue.Queue()
            self.waiting.append((rid, ids, params, time.perf_counter()))
        return rid

    def has_work(self) -> bool:
        return bool(self.waiting) or any(not s.done for s in self.seqs.values())

    def _schedule(self) -> dict:
        """Rank 0: the control object of this tick -- sequences admitted into
        the slot entering stage 0 and the forward calls it runs."""
        slot = self.tick % self.world
        live = [r for r in self.on_going[slot] if r in self.seqs and not self.seqs[r].done]
        new = []
        free = len(self.cache.allocator.free)
        with self._lock:
            while self.waiting and len(live) < self.max_num_seqs:
                rid, ids, params, t0 = self.waiting[0]
                nb = self._blocks_for(len(ids), params)
                if nb > free:
                    break
                free -= nb
                self.waiting.popleft()
                pd = dict(params.__dict__)
                pd["stop_token_ids"] = list(pd.get("stop_token_ids") or [])
                new.append((rid, ids, pd, t0))
                live.append(rid)
        plen = {n[0]: len(n[1]) for n in new}
        calls, dec = [], []
        budget = self.max_prefilled_seqs or len(live)
        for rid in live:
            sq = self.seqs.get(rid)
            n_prompt = sq.prompt_len if sq is not None else plen[rid]
            done_pre = sq.prefilled if sq is not None else 0
            if done_pre >= n_prompt:
                dec.append(rid)
            elif budget > 0:
                n = n_prompt - done_pre
                if self.prefill_chunk:
                    n = min(n, self.prefill_chunk)
                calls.append(("p", rid, done_pre, n))
                budget -= 1
        if dec:
            calls.insert(0, ("d", dec))
        return {"stop": False, "new": new, "calls": calls, "slot": live}

    def _apply_ctrl(self, ctrl: dict):
        for rid, ids, pd, t0 in ctrl["new"]:
            params = SamplingParams(**pd)
            g = torch.Generator(device=self.dev).manual_seed(params.seed) if params.seed is not None else None
            st = SequenceState(self.cache.allocator.alloc(self._blocks_for(len(ids), params)))
            self.seqs[rid] = _Seq(rid, len(ids), list(ids), params, st, arrival=t0, generator=g)
        self.on_going[self.tick % self.world] = list(ctrl["slot"])
        for c in ctrl["calls"]:
            if c[0] == "p":
                self.seqs[c[1]].prefilled = c[2] + c[3]
        self.pending[self.tick] = ctrl["calls"]

    # ----------------------------------------------------------------- stage execution
    def _inputs(self, c):
        dev, bs = self.dev, self.bs
        if c[0] == "p":
            _, rid, start, n = c
            sq = self.seqs[rid]
            ids = torch.tensor(sq.tokens[start:start + n], dtype=torch.long, device=dev)
            pos = torch.arange(start, start + n, device=dev)
            slots = slots_for(sq.state, start, n, bs).to(dev)
            L = start + n
            bt = make_block_table([sq.state], len(sq.state.blocks), dev)
            meta = AttnMeta(1, n, bt, torch.tensor([L], dtype=torch.int32, device=dev), nsplit_for(L), [L])
            return ids, pos, slots, meta, torch.tensor([n - 1], device=dev), [sq], n
        sqs = [self.seqs[r] for r in c[1]]
        pos_l = [sq.state.length for sq in sqs]
        ids = torch.tensor([sq.tokens[-1] for sq in sqs], dtype=torch.long, device=dev)
        pos = torch.tensor(pos_l, device=dev)
        slots = torch.tensor([sq.state.blocks[p // bs] * bs + p % bs for sq, p in zip(sqs, pos_l)], device=dev)
        bt = make_block_table([sq.state for sq in sqs], max(len(sq.state.blocks) for sq in sqs), dev)
        lens = [p + 1 for p in pos_l]
        meta = AttnMeta(len(sqs), 1, bt, torch.tensor(lens, dtype=torch.int32, device=dev),
                        nsplit_for(max(lens)), lens)
        return ids, pos, slots, meta, None, sqs, 1

    def _pick(self, logits: torch.Tensor, sq: _Seq) -> int:
        p = sq.params
        if p.repetition_penalty != 1.0:
            logits = apply_repetition_penalty(logits.clone(), [sq.tokens], p.repetition_penalty)
        return int(_sample(logits, p.do_sample, p.temperature, p.top_k, p.top_p, sq.generator)[0])

    def _run_stage(self, calls) -> Dict[int, int]:
        m = self.model
        sampled: Dict[int, int] = {}
        for c in calls:
            ids, pos, slots, meta, lidx, sqs, per = self._inputs(c)
            hidden = None
            if not self.is_head:
                hidden = torch.empty(ids.numel(), m.spec.hidden_size, dtype=m.dtype, device=self.dev)
                dist.recv(hidden, src=self._g(self.rank - 1), group=self.group)
            out = m.forward_tokens(ids, pos, slots, meta, self.cache, logits_idx=lidx, hidden_in=hidden)
            for sq in sqs:
                sq.state.length += per
            if c[0] == "p":
                self.stats["prefill_tokens"] += per
            else:
                self.stats["decode_tokens"] += len(sqs)
            if not self.is_tail:
                out = out.contiguous()
                self._sends.append((dist.isend(out, dst=self._g(self.rank + 1), group=self.group), out, self.tick))
                continue
            if c[0] == "p" and c[2] + c[3] < sqs[0].prompt_len:
                continue                            # partial prefill: no token yet
            for i, sq in enumerate(sqs):
                sampled[sq.rid] = self._pick(out[i:i + 1], sq)
        return sampled

    def _finish(self, sq: _Seq, reason: str):
        sq.done, sq.finish_reason = True, reason
        self.cache.allocator.release(sq.state.blocks)
        if self.is_head and sq.rid in self.streamer:
            self.streamer[sq.rid].put(-1)

    def _apply_tokens(self, sampled: Dict[int, int]):
        now = time.perf_counter()
        for rid, tok in sampled.items():
            sq = self.seqs[rid]
            sq.tokens.append(tok)
            sq.generated.append(tok)
            if sq.first_token_time is None:
                sq.first_token_time = now - sq.arrival
            if self.is_head and rid in self.streamer:
                self.streamer[rid].put(tok)
            p, n = sq.params, len(sq.generated)
            if n >= p.max_new_tokens:
                self._finish(sq, "length")
            elif n >= p.min_new_tokens and (tok in self.eos or tok in (p.stop_token_ids or [])):
                self._finish(sq, "stop")

    def _tick(self, ctrl: dict):
        self._apply_ctrl(ctrl)
        calls = self.pending.pop(self.tick - self.rank, None) if self.tick >= self.rank else None
        if calls:
            sampled = self._run_stage(calls)
        else:
            sampled = {}
            self.stats["bubbles"] += 1
        sampled = self._bcast(sampled if self.is_tail else None, self.world - 1)
        self._apply_tokens(sampled)
        # a send of an earlier tick was received by the successor before it
        # reached the token broadcast above, so waiting on it cannot block
        keep = []
        for h, buf, t in self._sends:
            if t < self.tick:
                h.wait()
            else:
                keep.append((h, buf, t))
        self._sends = keep
        self.tick += 1
        self.stats["ticks"] += 1

    # ----------------------------------------------------------------- drivers
    @torch.no_grad()
    def process_step(self) -> None:
        """Rank 0: one pipeline tick (schedule, broadcast, execute).  A dead
        peer (heartbeat monitor) or a failed collective fails every in-flight
        request and raises RankFailureError instead of blocking."""
        from ..parallel.health import RankFailureError, abort_process_group
        if self.failed:
            raise RankFailureError(self.failed)
        try:
            if self.monitor is not None:
                self.monitor.check()
            ctrl = self._bcast(self._schedule(), 0)
            self._tick(ctrl)
        except RankFailureError as e:
            abort_process_group(self.group)
            self.fail_all(str(e))
            raise
        except RuntimeError as e:                   # collective error: a peer vanished mid-tick
            if self.world == 1:
                raise
            self.fail_all(f"collective failed: {e}")
            raise RankFailureError(self.failed) from e

    @torch.no_grad()
    def serve_forever(self) -> None:
        """Ranks > 0: execute ticks until rank 0 calls :meth:`stop`."""
        if self.is_head:
            raise RuntimeError("rank 0 drives the pipeline with process_step() / generate()")
        while True:
            ctrl = self._bcast(None, 0)
            if ctrl["stop"]:
                break
            self._tick(ctrl)
        self._drain()

    def _drain(self):
        for h, _, _ in self._sends:
            h.wait()
        self._sends = []

    def stop(self) -> None:
        if self.heartbeat is not None:
            self.heartbeat.stop()
        if self.is_head and not self._stopped and not self.failed:
            self._stopped = True
            self._bcast({"stop": True}, 0)
            self._drain()

    def health(self) -> dict:
        """/health payload: ok, or the failure (dead ranks) that stopped serving"""
        if self.failed:
            return {"status": "error", "error": self.failed}
        if self.monitor is not None and not self.monitor.healthy:
            return {"status": "error", "error": self.monitor.reason}
        return {"status": "ok", "ticks": self.stats["ticks"]}

    def generate(self, prompts, params: Optional[SamplingParams] = None) -> List[List[int]]:
        """Rank 0 offline batch: submit everything, tick until done; returns
        the generated tokens of each prompt."""
        rids = [self.add_request(p, params) for p in prompts]
        while any(r not in self.seqs or not self.seqs[r].done for r in rids):
            self.process_step()                     # (raises RankFailureError on a dead peer)
        out = [list(self.seqs[r].generated) for r in rids]
        for r in rids:
            self.seqs.pop(r, None)
            self.streamer.pop(r, None)
        return out

    def stream(self, rid: int):
        """Rank 0: yield the tokens of request ``rid`` while another thread
        ticks the pipeline (:class:`PPEngineLoop`)."""
        q = self.streamer[rid]
        while True:
            t = q.get()
            if t < 0:
                return
            yield t


class PPEngineLoop:
    """Background thread on rank 0 that ticks the pipeline while there is
    work (the reference's ``process_step`` loop of its API server)."""

    def __init__(self, worker: PPModelWorker, idle_sleep: float = 0.002):
        self.worker, self.idle = worker, idle_sleep
        self._stop = threading.Event()
        self.thread = threading.Thread(target=self._run, daemon=True)
        self.error: Optional[BaseException] = None

    def start(self):
        self.thread.start()
        return self

    def _run(self):
        last = time.perf_counter()
        try:
            while not self._stop.is_set():
                # idle ticks once a second keep the other ranks' collectives
                # well inside the process-group timeout
                if self.worker.has_work() or time.perf_counter() - last > 1.0:
                    self.worker.process_step()
                    last = time.perf_counter()
                else:
                    time.sleep(self.idle)
        except BaseException as e:      # surfaced to the caller through .error / worker.health()
            self.error = e
            if not self.worker.failed:
                self.worker.fail_all(repr(e))

    def stop(self):
        self._stop.set()
        self.thread.join(timeout=30)
        self.worker.stop()
