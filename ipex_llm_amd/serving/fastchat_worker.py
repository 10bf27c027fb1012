"""FastChat-protocol model worker over the continuous-batching engine.

Reference: ``SRC/serving/fastchat/ipex_llm_worker.py`` (``BigDLLLMWorker``:
``/worker_generate_stream`` with NUL-delimited JSON chunks,
``/worker_generate``, ``/worker_get_embeddings``, ``/worker_get_status``,
``/count_token``, ``/worker_get_conv_template``, ``/model_details``;
controller registration and heartbeats from FastChat's ``BaseModelWorker``).

The reference runs one HF ``generate`` per request in a thread; here every
request joins the shared :class:`LLMEngine` (paged KV pool, one batched
native decode step for all running requests).  The FastChat package is not
required: the worker speaks its wire protocol directly (controller calls go
through ``requests`` when a controller address is given).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import queue
import threading
import uuid
from typing import Iterator, List, Optional

import torch

from .engine import EngineLoop, LLMEngine, SamplingParams

try:                                 # module level: endpoint annotations are resolved from globals
    from fastapi import Request
except ImportError:                  # pragma: no cover - the worker class works without fastapi
    Request = None

WORKER_HEART_BEAT_INTERVAL = 45
SERVER_ERROR_MSG = "**NETWORK ERROR DUE TO HIGH TRAFFIC. PLEASE REGENERATE OR REFRESH THIS PAGE.**"
ERROR_INTERNAL = 50001
ERROR_CONTEXT_OVERFLOW = 40303


def is_partial_stop(output: str, stop_str: str) -> bool:
    """True when a suffix of ``output`` is a proper prefix of ``stop_str``."""
    for i in range(0, min(len(output), len(stop_str))):
        if stop_str.startswith(output[-i - 1:]):
            return True
    return False


class IPEXLLMWorker:
    def __init__(self, engine: LLMEngine, tokenizer, model_names: List[str], controller_addr: Optional[str] = None,
                 worker_addr: Optional[str] = None, worker_id: Optional[str] = None,
                 limit_worker_concurrency: int = 1024, conv_template: Optional[str] = None,
                 context_len: Optional[int] = None, stream_interval: int = 2, no_register: bool = True):
        self.engine, self.tokenizer = engine, tokenizer
        self.model_names = list(model_names)
        self.controller_addr, self.worker_addr = controller_addr, worker_addr
        self.worker_id = worker_id or uuid.uuid4().hex[:8]
        self.limit_worker_concurrency = limit_worker_concurrency
        self.conv_template = conv_template
        self.context_len = context_len or engine.max_model_len
        self.stream_interval = max(1, stream_interval)
        self.call_ct = 0
        self.semaphore: Optional[asyncio.Semaphore] = None
        self._stop_hb = threading.Event()
        if not no_register and controller_addr:
            self.register_to_controller()
            threading.Thread(target=self._heart_beat_loop, daemon=True).start()

    # ----------------------------------------------------------------- controller
    def register_to_controller(self):
        import requests
        r = requests.post(self.controller_addr + "/register_worker",
                          json={"worker_name": self.worker_addr, "check_heart_beat": True,
                                "worker_status": self.get_status()}, timeout=10)
        r.raise_for_status()

    def send_heart_beat(self):
        import requests
        r = requests.post(self.controller_addr + "/receive_heart_beat",
                          json={"worker_name": self.worker_addr, "queue_length": self.get_queue_length()},
                          timeout=10)
        if not r.json().get("exist", True):
            self.register_to_controller()

    def _heart_beat_loop(self):
        while not self._stop_hb.wait(WORKER_HEART_BEAT_INTERVAL):
            try:
                self.send_heart_beat()
            except Exception:          # a restarting controller is retried on the next beat
                pass

    # ----------------------------------------------------------------- status
    def get_queue_length(self) -> int:
        return sum(1 for r in list(self.engine.requests.values()) if not r.finished)

    def get_status(self) -> dict:
        return {"model_names": self.model_names, "speed": 1, "queue_length": self.get_queue_length()}

    def count_token(self, params: dict) -> dict:
        return {"count": len(self.tokenizer(params["prompt"]).input_ids), "error_code": 0}

    def get_conv_template(self) -> dict:
        return {"conv": self.conv_template}

    # ----------------------------------------------------------------- generation
    def _params(self, params: dict, n_prompt: int) -> SamplingParams:
        temperature = float(params.get("temperature", 1.0))
        top_k = int(params.get("top_k", -1))
        max_new = max(1, min(int(params.get("max_new_tokens", 256)), self.context_len - n_prompt))
        stop_ids = [int(t) for t in (params.get("stop_token_ids") or []) if t is not None]
        eos = getattr(self.tokenizer, "eos_token_id", None)
        if eos is not None and eos not in stop_ids:
            stop_ids.append(eos)
        sample = temperature > 1e-5 and bool(params.get("do_sample", True))
        return SamplingParams(max_new_tokens=max_new, temperature=max(temperature, 1e-5),
                              top_k=top_k if top_k > 0 else 0, top_p=float(params.get("top_p", 1.0)),
                              do_sample=sample, repetition_penalty=float(params.get("repetition_penalty", 1.0)),
                              stop_token_ids=stop_ids, seed=params.get("seed"))

    @staticmethod
    def _chunk(text, finish, n_prompt, n_out, code=0) -> bytes:
        return json.dumps({"text": text, "error_code": code, "finish_reason": finish,
                           "usage": {"prompt_tokens": n_prompt, "completion_tokens": n_out,
                                     "total_tokens": n_prompt + n_out}}).encode() + b"\0"

    def generate_stream_gate(self, params: dict) -> Iterator[bytes]:
        self.call_ct += 1
        try:
            prompt = params["prompt"]
            ids = self.tokenizer.encode(prompt)
            if len(ids) >= self.context_len:
                yield self._chunk(f"{SERVER_ERROR_MSG}\n\n(prompt of {len(ids)} tokens exceeds the context "
                                  f"length {self.context_len})", None, len(ids), 0, ERROR_CONTEXT_OVERFLOW)
                return
            sp = self._params(params, len(ids))
            stop = params.get("stop")
            stops = {stop} if isinstance(stop, str) and stop else set(stop or [])
            q: "queue.Queue[int]" = queue.Queue()
            rid = self.engine.add_request(ids, sp, on_token=lambda t, r: q.put(t))
        except (ValueError, RuntimeError, KeyError) as e:
            yield self._chunk(f"{SERVER_ERROR_MSG}\n\n({e})", None, 0, 0, ERROR_INTERNAL)
            return
        base = prompt if bool(params.get("echo", True)) else ""
        out: List[int] = []
        text, finish, r = base, None, None
        try:
            while True:
                t = q.get()
                if t < 0:
                    break
                out.append(t)
                text = base + self.tokenizer.decode(out, skip_special_tokens=True)
                cut = [c for c in (text.rfind(s, len(base)) for s in stops) if c >= 0]
                if cut:
                    text, finish = text[:min(cut)], "stop"
                    break
                if len(out) % self.stream_interval == 0 and not any(is_partial_stop(text, s) for s in stops):
                    yield self._chunk(text, None, len(ids), len(out))
        finally:
            r = self.engine.requests.get(rid)
            if r is not None and not r.finished:
                self.engine.abort(rid)          # client went away / stop string hit
            self.engine.requests.pop(rid, None)
        if finish is None:
            finish = "length" if r is not None and r.finish_reason == "length" else "stop"
        yield self._chunk(text, finish, len(ids), len(out))

    def generate_gate(self, params: dict) -> dict:
        last = None
        for last in self.generate_stream_gate(params):
            pass
        return json.loads(last[:-1].decode())

    @torch.no_grad()
    def get_embeddings(self, params: dict) -> dict:
        """Mean-pooled, L2-normalised final hidden states (reference
        get_embeddings: masked sum / token count, then F.normalize)."""
        self.call_ct += 1
        from ..engine.runner import nsplit_for
        from ..models.cache import SequenceState, make_block_table, slots_for
        from ..models.decoder import AttnMeta
        eng, m = self.engine, self.engine.model
        dev, bs = m.device, self.engine.block_size
        embs, total = [], 0
        try:
            with eng.lock:        # shares the KV pool with the engine thread
                for text in params["input"]:
                    ids = self.tokenizer.encode(text)[:self.context_len]
                    n = len(ids)
                    blocks = eng.cache.allocator.alloc((n + bs - 1) // bs)
                    try:
                        seq = SequenceState(blocks)
                        meta = AttnMeta(1, n, make_block_table([seq], len(blocks), dev),
                                        torch.tensor([n], dtype=torch.int32, device=dev), nsplit_for(n), [n])
                        h = m.forward_tokens(torch.tensor(ids, device=dev), torch.arange(n, device=dev),
                                             slots_for(seq, 0, n, bs).to(dev), meta, eng.cache, return_hidden=True)
                    finally:
                        eng.cache.allocator.release(blocks)
                    embs.append(torch.nn.functional.normalize(h.float().mean(0), dim=0).cpu().tolist())
                    total += n
        except (RuntimeError, ValueError) as e:
            return {"text": f"{SERVER_ERROR_MSG}\n\n({e})", "error_code": ERROR_INTERNAL}
        return {"embedding": embs, "token_num": total}


def build_worker_app(worker: IPEXLLMWorker, loop_thread: Optional[EngineLoop] = None):
    import contextlib

    from fastapi import FastAPI
    from fastapi.responses import JSONResponse, StreamingResponse
    from starlette.background import BackgroundTask
    runner = loop_thread or EngineLoop(worker.engine)

    @contextlib.asynccontextmanager
    async def lifespan(_app):
        worker.semaphore = asyncio.Semaphore(worker.limit_worker_concurrency)
        if not runner.thread.is_alive():
            runner.start()
        yield
        runner.stop()
        worker._stop_hb.set()

    app = FastAPI(lifespan=lifespan)

    @app.post("/worker_generate_stream")
    async def api_generate_stream(request: Request):
        params = await request.json()
        await worker.semaphore.acquire()
        return StreamingResponse(worker.generate_stream_gate(params),
                                 background=BackgroundTask(worker.semaphore.release))

    async def _call(fn, params):
        await worker.semaphore.acquire()
        try:
            return JSONResponse(await asyncio.to_thread(fn, params))
        finally:
            worker.semaphore.release()

    @app.post("/worker_generate")
    async def api_generate(request: Request):
        return await _call(worker.generate_gate, await request.json())

    @app.post("/worker_get_embeddings")
    async def api_get_embeddings(request: Request):
        return await _call(worker.get_embeddings, await request.json())

    @app.post("/worker_get_status")
    async def api_get_status(request: Request):
        return worker.get_status()

    @app.post("/count_token")
    async def api_count_token(request: Request):
        return worker.count_token(await request.json())

    @app.post("/worker_get_conv_template")
    async def api_get_conv(request: Request):
        return worker.get_conv_template()

    @app.post("/model_details")
    async def api_model_details(request: Request):
        return {"context_length": worker.context_len}

    app.state.worker = worker
    return app


def main(argv=None):
    ap = argparse.ArgumentParser(description="ipex_llm_amd FastChat-protocol worker")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=21002)
    ap.add_argument("--worker-address", default="http://127.0.0.1:21002")
    ap.add_argument("--controller-address", default="http://127.0.0.1:21001")
    ap.add_argument("--model-path", required=True)
    ap.add_argument("--model-names", type=lambda s: s.split(","), default=None)
    ap.add_argument("--limit-worker-concurrency", type=int, default=1024)
    ap.add_argument("--no-register", action="store_true")
    ap.add_argument("--conv-template", default=None)
    ap.add_argument("--stream-interval", type=int, default=2)
    ap.add_argument("--low-bit", default="sym_int4")
    ap.add_argument("--load-low-bit-model", action="store_true")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--max-batch", type=int, default=64)
    ap.add_argument("--max-model-len", type=int, default=8192)
    a = ap.parse_args(argv)
    import uvicorn
    from transformers import AutoTokenizer

    from ..transformers import AutoModelForCausalLM
    from ..transformers.hf_native import get_native
    if a.load_low_bit_model:
        model = AutoModelForCausalLM.load_low_bit(a.model_path)
    else:
        model = AutoModelForCausalLM.from_pretrained(a.model_path, load_in_low_bit=a.low_bit,
                                                     torch_dtype=torch.bfloat16)
    model = model.to(a.device)
    tok = AutoTokenizer.from_pretrained(a.model_path)
    eng = LLMEngine(get_native(model)[0], max_batch=a.max_batch, max_model_len=a.max_model_len,
                    eos_token_id=tok.eos_token_id)
    names = a.model_names or [a.model_path.rstrip("/").split("/")[-1]]
    w = IPEXLLMWorker(eng, tok, names, a.controller_address, a.worker_address,
                      limit_worker_concurrency=a.limit_worker_concurrency, conv_template=a.conv_template,
                      stream_interval=a.stream_interval, no_register=a.no_register)
    uvicorn.run(build_worker_app(w), host=a.host, port=a.port)


if __name__ == "__main__":
    main()
