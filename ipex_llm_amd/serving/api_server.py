"""OpenAI / TGI-compatible HTTP server over the continuous-batching engine.

Reference: ``SRC/serving/fastapi/api_server.py`` -- ``FastApp`` with
``/generate``, ``/generate_stream``, ``/v1/chat/completions``,
``/v1/completions`` (103-437); ``openai_protocol.py`` / ``tgi_protocol.py``
request and response models; ``model_worker.py`` (one request at a time).

Here every request is submitted to :class:`LLMEngine` (continuous batching
over the paged KV pool) and tokens are streamed back as they are produced
(Server-Sent Events, OpenAI ``data: ... [DONE]`` framing).
Run: ``python -m ipex_llm_amd.serving.api_server --model PATH --low-bit sym_int4``.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import time
import uuid
from typing import Dict, List, Optional, Union

from pydantic import BaseModel

from .engine import EngineLoop, LLMEngine, SamplingParams


# ------------------------------------------------------------------ protocol
class Parameters(BaseModel):
    max_new_tokens: int = 32
    do_sample: Optional[bool] = None
    min_new_tokens: Optional[int] = None
    repetition_penalty: Optional[float] = None
    temperature: Optional[float] = None
    top_k: Optional[int] = None
    top_p: Optional[float] = None
    seed: Optional[int] = None


class InputsRequest(BaseModel):
    inputs: str
    parameters: Optional[Parameters] = None
    stream: Optional[bool] = False


class ChatCompletionRequest(BaseModel):
    messages: Union[str, List[Dict[str, str]]]
    model: str = ""
    max_tokens: Optional[int] = None
    min_tokens: Optional[int] = None
    stream: Optional[bool] = False
    top_p: Optional[float] = None
    top_k: Optional[int] = None
    repetition_penalty: Optional[float] = None
    presence_penalty: Optional[float] = None
    temperature: Optional[float] = None
    seed: Optional[int] = None


class CompletionRequest(BaseModel):
    prompt: Union[List[int], List[List[int]], str, List[str]]
    model: str = ""
    max_tokens: Optional[int] = None
    min_tokens: Optional[int] = None
    stream: Optional[bool] = False
    top_p: Optional[float] = None
    top_k: Optional[int] = None
    repetition_penalty: Optional[float] = None
    presence_penalty: Optional[float] = None
    temperature: Optional[float] = None
    seed: Optional[int] = None


def _params(max_tokens, min_tokens, temperature, top_k, top_p, repetition_penalty, do_sample=None, seed=None,
            default_max=256) -> SamplingParams:
    t = 1.0 if temperature is None else float(temperature)
    sample = do_sample if do_sample is not None else (temperature is not None and t > 0)
    return SamplingParams(max_new_tokens=int(max_tokens or default_max), min_new_tokens=int(min_tokens or 0),
                          temperature=max(t, 1e-5), top_k=int(top_k or 0), top_p=float(top_p or 1.0),
                          do_sample=bool(sample), repetition_penalty=float(repetition_penalty or 1.0), seed=seed)


class _Stream:
    """per-request token queue fed from the engine thread"""

    def __init__(self, loop: asyncio.AbstractEventLoop):
        self.loop, self.q = loop, asyncio.Queue()

    def __call__(self, tok, req):
        self.loop.call_soon_threadsafe(self.q.put_nowait, tok)


class _Detok:
    """incremental detokenization: emit only the new text"""

    def __init__(self, tok):
        self.tok, self.ids, self.text = tok, [], ""

    def push(self, t: int) -> str:
        self.ids.append(t)
        s = self.tok.decode(self.ids, skip_special_tokens=True)
        if s.endswith("�"):           # incomplete multi-byte char: wait
            return ""
        d, self.text = s[len(self.text):], s
        return d


def build_app(engine: LLMEngine, tokenizer, model_name: str = "ipex-llm-amd", loop_thread: Optional[EngineLoop] = None,
              asr=None):
    """``asr``: a :class:`serving.asr.WhisperTranscriber` serving
    ``/v1/audio/transcriptions`` (501 without one)."""
    from fastapi import FastAPI, HTTPException, Request
    from fastapi.middleware.cors import CORSMiddleware
    from fastapi.responses import JSONResponse, StreamingResponse

    import contextlib
    runner = loop_thread or EngineLoop(engine)
    state = {"runner": runner}

    @contextlib.asynccontextmanager
    async def lifespan(_app):
        if not runner.thread.is_alive():
            runner.start()
        yield
        runner.stop()

    app = FastAPI(title="ipex_llm_amd serving", lifespan=lifespan)
    app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_methods=["*"], allow_headers=["*"])

    def encode(text: str) -> List[int]:
        return tokenizer.encode(text, add_special_tokens=True) if isinstance(text, str) else list(text)

    def chat_prompt(messages) -> List[int]:
        if isinstance(messages, str):
            return encode(messages)
        if getattr(tokenizer, "chat_template", None):
            return list(tokenizer.apply_chat_template(messages, add_generation_prompt=True, tokenize=True))
        text = "".join(f"{m.get('role', 'user')}: {m.get('content', '')}\n" for m in messages) + "assistant:"
        return encode(text)

    async def run(prompt_ids: List[int], params: SamplingParams):
        s = _Stream(asyncio.get_running_loop())
        try:
            rid = engine.add_request(prompt_ids, params, on_token=s)
        except ValueError as e:
            raise HTTPException(status_code=400, detail=str(e))
        return rid, s

    async def tokens(rid, s: _Stream):
        try:
            while True:
                t = await s.q.get()
                if t < 0:
                    break
                yield t
        finally:
            r = engine.requests.get(rid)
            if r is not None and not r.finished:
                engine.abort(rid)

    def done(rid):
        r = engine.requests.pop(rid, None)
        return r

    def usage(r, n_prompt):
        return {"prompt_tokens": n_prompt, "completion_tokens": len(r.generated) if r else 0,
                "total_tokens": n_prompt + (len(r.generated) if r else 0)}

    @app.get("/health")
    async def health():
        from fastapi.responses import JSONResponse
        err = runner.error if runner is not None else None
        if err is not None:           # the engine loop died (device fault / dead rank): not ready
            return JSONResponse({"status": "error", "error": repr(err)}, status_code=503)
        return {"status": "ok", "running": int(engine.sched.num_running()), "waiting": int(engine.sched.num_waiting())}

    @app.get("/metrics")
    async def metrics():
        from fastapi.responses import Response
        from .metrics import CONTENT_TYPE_LATEST
        return Response(engine.metrics.render(), media_type=CONTENT_TYPE_LATEST)

    @app.get("/v1/models")
    async def models():
        return {"object": "list", "data": [{"id": model_name, "object": "model", "owned_by": "ipex_llm_amd"}]}

    # ---- TGI-style
    @app.post("/generate")
    async def generate(req: InputsRequest):
        if req.stream:
            return await generate_stream(req)
        p = req.parameters or Parameters()
        rid, s = await run(encode(req.inputs), _params(p.max_new_tokens, p.min_new_tokens, p.temperature, p.top_k,
                                                       p.top_p, p.repetition_penalty, p.do_sample, p.seed))
        ids = [t async for t in tokens(rid, s)]
        done(rid)
        return [str(rid), tokenizer.decode(ids, skip_special_tokens=True)]

    @app.post("/generate_stream")
    async def generate_stream(req: InputsRequest):
        p = req.parameters or Parameters()
        rid, s = await run(encode(req.inputs), _params(p.max_new_tokens, p.min_new_tokens, p.temperature, p.top_k,
                                                       p.top_p, p.repetition_penalty, p.do_sample, p.seed))

        async def gen():
            d = _Detok(tokenizer)
            idx = 0
            async for t in tokens(rid, s):
                idx += 1
                yield "data: " + json.dumps({"index": idx, "token": {"id": t, "text": d.push(t)},
                                             "generated_text": None, "details": None}) + "\n\n"
            r = done(rid)
            yield "data: " + json.dumps({"index": idx + 1, "token": None, "generated_text": d.text,
                                         "details": {"finish_reason": r.finish_reason if r else None,
                                                     "generated_tokens": idx}}) + "\n\n"
        return StreamingResponse(gen(), media_type="text/event-stream")

    # ---- OpenAI
    async def _openai(prompt_ids, params, stream, chat: bool):
        rid, s = await run(prompt_ids, params)
        oid = ("chatcmpl-" if chat else "cmpl-") + uuid.uuid4().hex[:24]
        created = int(time.time())
        obj = "chat.completion" if chat else "text_completion"
        if not stream:
            ids = [t async for t in tokens(rid, s)]
            r = done(rid)
            text = tokenizer.decode(ids, skip_special_tokens=True)
            choice = {"index": 0, "finish_reason": r.finish_reason if r else None}
            if chat:
                choice["message"] = {"role": "assistant", "content": text}
            else:
                choice["text"] = text
            return JSONResponse({"id": oid, "object": obj, "created": created, "model": model_name,
                                 "choices": [choice], "usage": usage(r, len(prompt_ids))})

        async def gen():
            d = _Detok(tokenizer)
            if chat:
                first = {"id": oid, "object": "chat.completion.chunk", "created": created, "model": model_name,
                         "choices": [{"index": 0, "delta": {"role": "assistant"}, "finish_reason": None}]}
                yield "data: " + json.dumps(first) + "\n\n"
            async for t in tokens(rid, s):
                delta = d.push(t)
                ch = {"index": 0, "finish_reason": None}
                if chat:
                    ch["delta"] = {"content": delta}
                else:
                    ch["text"] = delta
                yield "data: " + json.dumps({"id": oid, "object": obj + (".chunk" if chat else ""),
                                             "created": created, "model": model_name, "choices": [ch]}) + "\n\n"
            r = done(rid)
            ch = {"index": 0, "finish_reason": r.finish_reason if r else "stop"}
            if chat:
                ch["delta"] = {}
            else:
                ch["text"] = ""
            yield "data: " + json.dumps({"id": oid, "object": obj + (".chunk" if chat else ""), "created": created,
                                         "model": model_name, "choices": [ch]}) + "\n\n"
            yield "data: [DONE]\n\n"
        return StreamingResponse(gen(), media_type="text/event-stream")

    @app.post("/v1/chat/completions")
    async def chat_completions(req: ChatCompletionRequest):
        params = _params(req.max_tokens, req.min_tokens, req.temperature, req.top_k, req.top_p,
                         req.repetition_penalty, seed=req.seed)
        return await _openai(chat_prompt(req.messages), params, req.stream, True)

    @app.post("/v1/completions")
    async def completions(req: CompletionRequest):
        prompt = req.prompt
        if isinstance(prompt, list) and prompt and isinstance(prompt[0], (list, str)):
            prompt = prompt[0]                     # one prompt per request (like the reference)
        ids = encode(prompt) if isinstance(prompt, str) else list(prompt)
        params = _params(req.max_tokens, req.min_tokens, req.temperature, req.top_k, req.top_p,
                         req.repetition_penalty, seed=req.seed, default_max=16)
        return await _openai(ids, params, req.stream, False)

    async def transcriptions(request):
        # reference SRC/serving/fastapi/api_server.py:404-428: multipart upload
        # (file, model, language, prompt, response_format) -> {"text": ...}
        if asr is None:
            raise HTTPException(status_code=501, detail="no speech model loaded (start with --asr-model)")
        from fastapi.responses import PlainTextResponse
        from .asr import decode_wav, parse_multipart, srt_or_vtt
        try:
            form = parse_multipart(await request.body(), request.headers.get("content-type", ""))
            f = form.get("file")
            if not isinstance(f, tuple):
                raise ValueError("missing 'file' upload")
            audio, sr = decode_wav(f[1])
        except ValueError as e:
            raise HTTPException(status_code=400, detail=str(e))
        lang = form.get("language") or None
        fmt = form.get("response_format") or "json"
        try:
            text = await asyncio.get_running_loop().run_in_executor(
                None, lambda: asr.transcribe(audio, sr, lang, form.get("prompt") or None))
        except ValueError as e:
            raise HTTPException(status_code=400, detail=str(e))
        if fmt == "text":
            return PlainTextResponse(text)
        if fmt in ("srt", "vtt"):
            return PlainTextResponse(srt_or_vtt(text, fmt, len(audio) / sr))
        if fmt == "verbose_json":
            return {"task": "transcribe", "language": lang, "duration": len(audio) / sr, "text": text}
        return {"text": text}

    transcriptions.__annotations__["request"] = Request     # (postponed annotations: give FastAPI the class)
    app.post("/v1/audio/transcriptions")(transcriptions)

    app.state.engine = engine
    app.state.runner = state["runner"]
    return app


class FastApp:
    """Reference-compatible wrapper: ``FastApp(model, tokenizer).app``."""

    def __init__(self, model, tokenizer, max_batch: int = 32, max_model_len: int = 4096, asr=None, **kw):
        from ..transformers.hf_native import get_native
        native = get_native(model)[0] if not hasattr(model, "forward_tokens") else model
        eos = getattr(tokenizer, "eos_token_id", None)
        self.engine = LLMEngine(native, max_batch=max_batch, max_model_len=max_model_len, eos_token_id=eos, **kw)
        self.app = build_app(self.engine, tokenizer, getattr(getattr(model, "config", None), "_name_or_path", "model"),
                             asr=asr)


def main(argv=None):
    ap = argparse.ArgumentParser(description="ipex_llm_amd OpenAI-compatible server")
    ap.add_argument("--model", required=True, help="HF checkpoint or low-bit directory")
    ap.add_argument("--low-bit", default="sym_int4")
    ap.add_argument("--load-low-bit", action="store_true", help="--model was written by save_low_bit")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--max-batch", type=int, default=64)
    ap.add_argument("--max-model-len", type=int, default=8192)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--asr-model", default=None, help="Whisper checkpoint served at /v1/audio/transcriptions")
    a = ap.parse_args(argv)
    import torch
    import uvicorn
    from transformers import AutoTokenizer
    from ..transformers import AutoModelForCausalLM
    if a.load_low_bit:
        model = AutoModelForCausalLM.load_low_bit(a.model)
    else:
        model = AutoModelForCausalLM.from_pretrained(a.model, load_in_low_bit=a.low_bit, torch_dtype=torch.bfloat16)
    model = model.to(a.device)
    tok = AutoTokenizer.from_pretrained(a.model)
    asr = None
    if a.asr_model:
        from .asr import WhisperTranscriber
        asr = WhisperTranscriber.from_pretrained(a.asr_model, a.low_bit, a.device)
    fa = FastApp(model, tok, max_batch=a.max_batch, max_model_len=a.max_model_len, asr=asr)
    uvicorn.run(fa.app, host=a.host, port=a.port)


if __name__ == "__main__":
    main()
