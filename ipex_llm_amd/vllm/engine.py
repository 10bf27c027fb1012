"""vLLM-style engine surface over the native serving engine.

Reference: ``SRC/vllm/xpu/engine/engine.py`` -- ``IPEXLLMClass`` (offline
``LLM``), ``IPEXLLMLLMEngine`` (``LLMEngine.from_engine_args(...,
load_in_low_bit=...)``) and ``IPEXLLMAsyncLLMEngine``, which subclass vLLM's
engines and convert the loaded model's linears to low-bit.  vLLM is not a
dependency here (and not importable in this image), so the same class names
and call shapes are provided directly on ``serving.engine.LLMEngine``: the
C++ continuous-batching scheduler, the paged KV cache, captured decode
graphs and the low-bit HIP kernels.  A script written against the
reference's vLLM path -- ``IPEXLLMClass(model=path, load_in_low_bit="sym_int4")
.generate(prompts, SamplingParams(max_tokens=64))`` -- runs unchanged; the
outputs are vLLM-shaped ``RequestOutput`` / ``CompletionOutput`` records.
"""
from __future__ import annotations

import asyncio
import itertools
import threading
from dataclasses import dataclass, field
from typing import AsyncIterator, Dict, List, Optional, Sequence, Union

import torch

from ..serving import engine as _srv


@dataclass
class SamplingParams:
    """vLLM field names (``max_tokens``, ``min_tokens``, ``stop_token_ids``,
    ``ignore_eos``, ``n`` = 1); ``to_native`` maps onto the serving engine's"""
    n: int = 1
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = -1
    max_tokens: int = 16
    min_tokens: int = 0
    repetition_penalty: float = 1.0
    stop_token_ids: List[int] = field(default_factory=list)
    ignore_eos: bool = False
    seed: Optional[int] = None
    skip_special_tokens: bool = True

    def to_native(self) -> _srv.SamplingParams:
        if self.n != 1:
            raise ValueError("SamplingParams.n > 1 is not supported (one completion per request)")
        greedy = self.temperature <= 1e-5
        return _srv.SamplingParams(max_new_tokens=self.max_tokens, min_new_tokens=self.min_tokens,
                                   temperature=1.0 if greedy else self.temperature,
                                   top_k=max(0, self.top_k), top_p=self.top_p, do_sample=not greedy,
                                   repetition_penalty=self.repetition_penalty,
                                   stop_token_ids=list(self.stop_token_ids), seed=self.seed,
                                   ignore_eos=self.ignore_eos)


@dataclass
class CompletionOutput:
    index: int
    text: str
    token_ids: List[int]
    finish_reason: Optional[str] = None


@dataclass
class RequestOutput:
    request_id: str
    prompt: Optional[str]
    prompt_token_ids: List[int]
    outputs: List[CompletionOutput]
    finished: bool


@dataclass
class EngineArgs:
    """the subset of vLLM's EngineArgs this engine honours (others are
    accepted through ``**kwargs`` of the classes below and ignored)"""
    model: Union[str, torch.nn.Module]
    tokenizer: Optional[str] = None
    dtype: str = "auto"
    tensor_parallel_size: int = 1
    max_model_len: int = 4096
    max_num_seqs: int = 64
    block_size: int = 64
    gpu_memory_utilization: float = 0.9
    enforce_eager: bool = False
    enable_prefix_caching: bool = True
    seed: Optional[int] = None
    device: Optional[str] = None
    trust_remote_code: bool = False


def _finish_reason(r) -> Optional[str]:
    if not r.finished:
        return None
    return {"stop": "stop", "eos": "stop", "length": "length"}.get(r.finish_reason, r.finish_reason)


class IPEXLLMLLMEngine:
    """``LLMEngine``-shaped: ``add_request`` / ``step`` / ``has_unfinished_requests``"""

    def __init__(self, engine: _srv.LLMEngine, tokenizer=None):
        self.engine = engine
        self.tokenizer = tokenizer
        self._rid: Dict[str, int] = {}           # request_id -> native id
        self._text: Dict[str, Optional[str]] = {}

    @classmethod
    def from_engine_args(cls, engine_args: EngineArgs, load_in_low_bit: str = "sym_int4", **_):
        a = engine_args
        tp_group = None
        if a.tensor_parallel_size != 1:
            # one process per GPU (torchrun --nproc-per-node N ...): every rank
            # loads its AutoTP shard (the reference's per-rank low-bit convert,
            # SRC/vllm/xpu/model_convert.py:36-75); rank 0 serves, the others
            # run engine.run_worker() (see tp_worker_or_driver)
            import torch.distributed as dist
            from ..parallel.comm import init_distributed
            init_distributed()
            if dist.get_world_size() != a.tensor_parallel_size:
                raise ValueError(f"tensor_parallel_size={a.tensor_parallel_size} but {dist.get_world_size()} "
                                 "ranks are running: launch with torchrun --nproc-per-node "
                                 f"{a.tensor_parallel_size}")
            tp_group = dist.group.WORLD
        tok = None
        if isinstance(a.model, torch.nn.Module):
            model = a.model
        else:
            from transformers import AutoTokenizer
            from ..transformers import AutoModelForCausalLM
            dt = {"auto": torch.bfloat16, "bfloat16": torch.bfloat16, "float16": torch.float16,
                  "half": torch.float16}.get(a.dtype, torch.bfloat16)
            kw = {"tp_group": tp_group} if tp_group is not None else {}
            model = AutoModelForCausalLM.from_pretrained(a.model, load_in_low_bit=load_in_low_bit, torch_dtype=dt,
                                                         trust_remote_code=a.trust_remote_code, **kw)
            dev = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
            model = model.to(dev)
            tok = AutoTokenizer.from_pretrained(a.tokenizer or a.model, trust_remote_code=a.trust_remote_code)
        if a.tokenizer is not None and tok is None:
            from transformers import AutoTokenizer
            tok = AutoTokenizer.from_pretrained(a.tokenizer)
        if a.seed is not None:
            torch.manual_seed(a.seed)
        native = model
        if not hasattr(model, "forward_tokens"):
            from ..transformers.hf_native import get_native
            native = get_native(model)[0]
        eos = getattr(tok, "eos_token_id", None) if tok is not None else None
        if eos is None:
            eos = getattr(getattr(native, "config", None), "eos_token_id", None)
        eng = _srv.LLMEngine(native, max_batch=a.max_num_seqs, block_size=a.block_size,
                             max_model_len=a.max_model_len, memory_fraction=min(0.95, a.gpu_memory_utilization),
                             eos_token_id=eos, use_graph=not a.enforce_eager,
                             enable_prefix_caching=a.enable_prefix_caching)
        return cls(eng, tok)

    def get_tokenizer(self):
        return self.tokenizer

    @property
    def is_driver(self) -> bool:
        return self.engine.is_driver

    def run_worker(self):
        """tensor-parallel ranks > 0: replay the driver's steps until it shuts down"""
        self.engine.run_worker()

    def shutdown(self):
        self.engine.shutdown()

    def _ids(self, prompt: Optional[str], prompt_token_ids: Optional[Sequence[int]]) -> List[int]:
        if prompt_token_ids is not None:
            return [int(t) for t in prompt_token_ids]
        if self.tokenizer is None:
            raise ValueError("text prompts need a tokenizer (pass prompt_token_ids or tokenizer=...)")
        return list(self.tokenizer(prompt)["input_ids"])

    def add_request(self, request_id: str, prompt: Optional[str] = None,
                    sampling_params: Optional[SamplingParams] = None,
                    prompt_token_ids: Optional[Sequence[int]] = None, on_token=None):
        sp = sampling_params or SamplingParams()
        ids = self._ids(prompt, prompt_token_ids)
        rid = self.engine.add_request(ids, sp.to_native(), on_token=on_token)
        self._rid[str(request_id)] = rid
        self._text[str(request_id)] = prompt

    def abort_request(self, request_id: Union[str, Sequence[str]]):
        """stop and forget the requests (as in vLLM, an aborted request
        produces no further output)"""
        for q in ([request_id] if isinstance(request_id, str) else request_id):
            rid = self._rid.pop(str(q), None)
            self._text.pop(str(q), None)
            if rid is not None:
                self.engine.abort(rid)
                with self.engine.lock:          # the engine loop thread walks requests
                    self.engine.requests.pop(rid, None)

    def has_unfinished_requests(self) -> bool:
        return self.engine.has_work()

    def _output(self, request_id: str, release: bool) -> RequestOutput:
        rid = self._rid[request_id]
        r = self.engine.requests[rid]
        text = ""
        if self.tokenizer is not None:
            text = self.tokenizer.decode(r.generated, skip_special_tokens=True)
        out = RequestOutput(request_id, self._text.get(request_id), list(r.prompt),
                            [CompletionOutput(0, text, list(r.generated), _finish_reason(r))], r.finished)
        if release and r.finished:
            self.engine.requests.pop(rid, None)
            self._rid.pop(request_id, None)
            self._text.pop(request_id, None)
        return out

    def step(self) -> List[RequestOutput]:
        """one scheduler iteration; the outputs of every tracked request
        (finished ones are released after being reported once)"""
        if self.engine.has_work():
            self.engine.step()
        return [self._output(q, release=True) for q in list(self._rid)]


class IPEXLLMClass:
    """offline ``LLM``: ``generate(prompts, sampling_params)`` runs every
    request to completion through continuous batching"""

    def __init__(self, model, tokenizer: Optional[str] = None, tensor_parallel_size: int = 1, dtype: str = "auto",
                 seed: Optional[int] = None, gpu_memory_utilization: float = 0.9, enforce_eager: Optional[bool] = None,
                 max_model_len: int = 4096, max_num_seqs: int = 64, load_in_low_bit: str = "sym_int4",
                 device: Optional[str] = None, **kwargs):
        args = EngineArgs(model=model, tokenizer=tokenizer, dtype=dtype, tensor_parallel_size=tensor_parallel_size,
                          max_model_len=max_model_len, max_num_seqs=max_num_seqs, seed=seed,
                          gpu_memory_utilization=gpu_memory_utilization, enforce_eager=bool(enforce_eager),
                          device=device, trust_remote_code=bool(kwargs.get("trust_remote_code", False)))
        self.llm_engine = IPEXLLMLLMEngine.from_engine_args(args, load_in_low_bit=load_in_low_bit)
        self._counter = itertools.count()
        if tensor_parallel_size > 1:
            # the same script on every rank (torchrun): ranks > 0 serve the
            # driver's forwards here and leave when it exits; the driver
            # releases them at interpreter exit (or llm.shutdown())
            if not self.llm_engine.is_driver:
                self.llm_engine.run_worker()
                raise SystemExit(0)
            import atexit
            atexit.register(self.llm_engine.shutdown)

    def shutdown(self):
        self.llm_engine.shutdown()

    def get_tokenizer(self):
        return self.llm_engine.get_tokenizer()

    def generate(self, prompts: Union[str, Sequence[str], None] = None,
                 sampling_params: Union[SamplingParams, Sequence[SamplingParams], None] = None,
                 prompt_token_ids: Optional[Sequence[Sequence[int]]] = None, use_tqdm: bool = False) -> List[RequestOutput]:
        if isinstance(prompts, str):
            prompts = [prompts]
        n = len(prompts) if prompts is not None else len(prompt_token_ids)
        sps = (list(sampling_params) if isinstance(sampling_params, (list, tuple))
               else [sampling_params or SamplingParams()] * n)
        ids = []
        for i in range(n):
            q = str(next(self._counter))
            self.llm_engine.add_request(q, prompts[i] if prompts is not None else None, sps[i],
                                        prompt_token_ids[i] if prompt_token_ids is not None else None)
            ids.append(q)
        done: Dict[str, RequestOutput] = {}
        while len(done) < n:
            for o in self.llm_engine.step():
                if o.finished:
                    done[o.request_id] = o
        return [done[q] for q in ids]


class IPEXLLMAsyncLLMEngine:
    """``AsyncLLMEngine``-shaped: ``async for out in engine.generate(prompt,
    sampling_params, request_id)`` streams cumulative outputs while a
    background thread drives the scheduler (serving.engine.EngineLoop)"""

    def __init__(self, llm_engine: IPEXLLMLLMEngine):
        self.engine = llm_engine
        self.loop = _srv.EngineLoop(llm_engine.engine).start()
        self._lock = threading.Lock()

    @classmethod
    def from_engine_args(cls, engine_args: EngineArgs, load_in_low_bit: str = "sym_int4", **kw):
        return cls(IPEXLLMLLMEngine.from_engine_args(engine_args, load_in_low_bit=load_in_low_bit, **kw))

    async def generate(self, prompt: Optional[str], sampling_params: SamplingParams, request_id: str,
                       prompt_token_ids: Optional[Sequence[int]] = None) -> AsyncIterator[RequestOutput]:
        aloop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        tok = self.engine.tokenizer

        def on_token(t, r):
            aloop.call_soon_threadsafe(q.put_nowait, (list(r.generated), r.finished, _finish_reason(r)))

        with self._lock:
            self.engine.add_request(request_id, prompt, sampling_params, prompt_token_ids, on_token=on_token)
            rid = self.engine._rid[str(request_id)]
            pids = list(self.engine.engine.requests[rid].prompt)
        while True:
            gen, fin, why = await q.get()
            text = tok.decode(gen, skip_special_tokens=True) if tok is not None else ""
            yield RequestOutput(str(request_id), prompt, pids, [CompletionOutput(0, text, gen, why)], fin)
            if fin:
                # under the serving engine's own lock: its loop thread walks requests
                with self._lock, self.engine.engine.lock:
                    self.engine.engine.requests.pop(rid, None)
                    self.engine._rid.pop(str(request_id), None)
                    self.engine._text.pop(str(request_id), None)
                return

    async def abort(self, request_id: str):
        with self._lock:
            self.engine.abort_request(request_id)

    def shutdown(self):
        self.loop.stop()
