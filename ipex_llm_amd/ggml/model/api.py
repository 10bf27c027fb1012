"""``Llama`` (llama-cpp-python surface) and its family wrappers.

Reference: ``SRC/ggml/model/llama/llama.py:123-1419`` (``Llama``: tokenize,
eval, sample, generate, create_completion / __call__, create_chat_completion,
create_embedding / embed, save_state / load_state, n_ctx / n_embd / n_vocab,
token_eos / token_bos / token_nl), ``SRC/ggml/model/generation/utils.py``
(HF-like ``generate`` / ``decode`` / ``batch_decode``), the ``Gptneox`` /
``Bloom`` / ``Starcoder`` wrappers and ``SRC/transformers/modelling_bigdl.py``
(``from_pretrained(..., model_family=...)``).
"""
from __future__ import annotations

import os
import time
import uuid
from typing import Dict, Iterator, List, Optional, Sequence, Union

import torch

from ...engine.runner import _sample, apply_repetition_penalty
from .llama import LlamaCache, LlamaContext, LlamaState, load_model_and_tokenizer, longest_token_prefix


class Llama:
    """High-level model wrapper with the llama-cpp-python API."""

    def __init__(self, model_path: Optional[str] = None, n_ctx: int = 512, n_batch: int = 512, seed: int = -1,
                 logits_all: bool = False, embedding: bool = False, last_n_tokens_size: int = 64,
                 low_bit: str = "sym_int4", device: Optional[str] = None, verbose: bool = False,
                 model=None, tokenizer=None, **kwargs):
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        if model is None:
            if model_path is None or not os.path.exists(model_path):
                raise ValueError(f"Model path does not exist: {model_path}")
            model, tokenizer = load_model_and_tokenizer(model_path, low_bit, device)
        self.model, self.tokenizer, self.model_path = model, tokenizer, model_path
        self.verbose, self.embedding = verbose, embedding
        self.last_n_tokens_size = last_n_tokens_size
        self.ctx = LlamaContext(model, n_ctx, n_batch, logits_all)
        self.cache: Optional[LlamaCache] = None
        self._gen = torch.Generator().manual_seed(seed if seed >= 0 else int(time.time()))

    # ----------------------------------------------------------------- tokens
    @property
    def eval_tokens(self):
        return self.ctx.eval_tokens

    @property
    def eval_logits(self):
        return self.ctx.eval_logits

    def _tokenize(self, text: bytes, add_bos: bool = True) -> List[int]:
        s = text.decode("utf-8", errors="ignore") if isinstance(text, (bytes, bytearray)) else text
        return list(self.tokenizer.encode(s, add_special_tokens=add_bos))

    def tokenize(self, text, add_bos: bool = True):
        if isinstance(text, (list, tuple)):
            return [self._tokenize(t, add_bos) for t in text]
        return self._tokenize(text, add_bos)

    def detokenize(self, tokens: List[int]) -> bytes:
        return self.tokenizer.decode(list(tokens), skip_special_tokens=True).encode("utf-8")

    def decode(self, tokens: List[int]) -> str:
        return self.detokenize(tokens).decode("utf-8", errors="ignore")

    def batch_decode(self, tokens):
        if not tokens:
            return None
        if isinstance(tokens[0], (list, tuple)):
            return [self.decode(t) for t in tokens]
        return self.decode(tokens)

    # ----------------------------------------------------------------- context
    def set_cache(self, cache: Optional[LlamaCache]):
        self.cache = cache

    def reset(self):
        self.ctx.reset()

    def eval(self, tokens: Sequence[int]):
        self.ctx.eval(tokens)

    def sample(self, top_k: int = 40, top_p: float = 0.95, temp: float = 0.80, repeat_penalty: float = 1.1,
               frequency_penalty: float = 0.0, presence_penalty: float = 0.0, logits_processor=None, **kw) -> int:
        if self.ctx._scores is None:
            raise RuntimeError("sample() before eval()")
        lg = self.ctx._scores.clone().unsqueeze(0)
        last = list(self.eval_tokens)[-self.last_n_tokens_size:]
        lg = apply_repetition_penalty(lg, [last], repeat_penalty)
        if (frequency_penalty or presence_penalty) and last:
            ids, counts = torch.tensor(last).unique(return_counts=True)
            lg[0, ids] -= counts.float() * frequency_penalty + presence_penalty
        if logits_processor is not None:
            lg = logits_processor(torch.tensor([list(self.eval_tokens)]), lg)
        if temp <= 0:
            return int(torch.argmax(lg, -1)[0])
        return int(_sample(lg, True, temp, top_k, top_p, self._gen)[0])

    def _generate(self, tokens: Sequence[int], top_k: int = 40, top_p: float = 0.95, temp: float = 0.80,
                  repeat_penalty: float = 1.1, reset: bool = True, **kw) -> Iterator[int]:
        """Endless token generator; reuses the longest already-evaluated prefix."""
        tokens = list(tokens)
        if reset and len(self.eval_tokens) > 0:
            pre = longest_token_prefix(self.eval_tokens, tokens)
            if pre == len(tokens):
                pre -= 1                       # re-evaluate the last token for fresh logits
            if pre > 0:
                self.ctx.rewind(pre)
                tokens = tokens[pre:]
            else:
                self.reset()
        while True:
            self.eval(tokens)
            tok = self.sample(top_k=top_k, top_p=top_p, temp=temp, repeat_penalty=repeat_penalty, **kw)
            yield tok
            tokens = [tok]

    def generate(self, inputs=None, max_new_tokens: int = 128, top_k: int = 40, top_p: float = 0.95,
                 temperature: float = 0.80, repetition_penalty: float = 1.1, reset: bool = True,
                 frequency_penalty: float = 0.0, presence_penalty: float = 0.0, stop=None, **kw):
        """HF-like generate: the generated token ids of each input."""
        if isinstance(inputs, torch.Tensor):
            inputs = inputs.tolist()
        batched = bool(inputs) and isinstance(inputs[0], (list, tuple))
        eos = self.token_eos()
        outs = []
        for row in (inputs if batched else [inputs]):
            gen = []
            for tok in self._generate(row, top_k, top_p, temperature, repetition_penalty, reset,
                                      frequency_penalty=frequency_penalty, presence_penalty=presence_penalty):
                if tok == eos:
                    break
                gen.append(tok)
                if len(gen) >= max_new_tokens:
                    break
            outs.append(gen)
        return outs if batched else outs[0]

    def save_state(self) -> LlamaState:
        return self.ctx.save()

    def load_state(self, state: LlamaState) -> None:
        self.ctx.load(state)

    # ----------------------------------------------------------------- completions
    def _completion(self, prompt, suffix, max_tokens, temperature, top_p, echo, stop, frequency_penalty,
                    presence_penalty, repeat_penalty, top_k, stream, model) -> Iterator[dict]:
        cid, created = f"cmpl-{uuid.uuid4()}", int(time.time())
        name = model or self.model_path or "model"
        ptoks = self.tokenize(prompt) if isinstance(prompt, (str, bytes)) else list(prompt)
        ptext = prompt if isinstance(prompt, str) else self.decode(ptoks)
        if len(ptoks) + max_tokens > self.n_ctx():
            raise ValueError(f"Requested tokens exceed context window of {self.n_ctx()}")
        stops = [stop] if isinstance(stop, str) else list(stop or [])
        if self.cache is not None and ptoks in self.cache:
            self.load_state(self.cache[ptoks])
        eos = self.token_eos()
        gen: List[int] = []
        sent, text, finish = "", "", "length"

        def chunk(t, fin):
            return {"id": cid, "object": "text_completion", "created": created, "model": name,
                    "choices": [{"text": t, "index": 0, "logprobs": None, "finish_reason": fin}]}

        for tok in self._generate(ptoks, top_k, top_p, temperature, repeat_penalty,
                                  frequency_penalty=frequency_penalty, presence_penalty=presence_penalty):
            if tok == eos:
                finish = "stop"
                break
            gen.append(tok)
            text = self.decode(gen)
            hit = [text.index(s) for s in stops if s and s in text]
            if hit:
                text, finish = text[:min(hit)], "stop"
                break
            if stream:
                # hold back a tail that could still become a stop string / a partial char
                hold = max([len(s) - 1 for s in stops if s] + [0])
                safe = text[:len(text) - hold] if hold else text
                if safe.endswith("�"):
                    safe = safe[:-1]
                if len(safe) > len(sent):
                    yield chunk(safe[len(sent):], None)
                    sent = safe
            if len(gen) >= max_tokens:
                break
        if self.cache is not None:
            self.cache[ptoks + gen] = self.save_state()
        if stream:
            yield chunk(text[len(sent):], finish)
            return
        r = chunk((ptext if echo else "") + text + (suffix or ""), finish)
        r["usage"] = {"prompt_tokens": len(ptoks), "completion_tokens": len(gen),
                      "total_tokens": len(ptoks) + len(gen)}
        yield r

    def create_completion(self, prompt, suffix=None, max_tokens: int = 128, temperature: float = 0.8,
                          top_p: float = 0.95, logprobs=None, echo: bool = False, stop=None,
                          frequency_penalty: float = 0.0, presence_penalty: float = 0.0,
                          repeat_penalty: float = 1.1, top_k: int = 40, stream: bool = False, model=None, **kw):
        it = self._completion(prompt, suffix, max_tokens, temperature, top_p, echo, stop, frequency_penalty,
                              presence_penalty, repeat_penalty, top_k, stream, model)
        return it if stream else next(iter(it))

    __call__ = create_completion

    def _chat_prompt(self, messages):
        if getattr(self.tokenizer, "chat_template", None):
            return list(self.tokenizer.apply_chat_template(messages, add_generation_prompt=True, tokenize=True))
        text = "".join(f"### {m.get('role', 'user').capitalize()}:\n{m.get('content', '')}\n" for m in messages)
        return text + "### Assistant:\n"

    def create_chat_completion(self, messages: List[Dict[str, str]], temperature: float = 0.2, top_p: float = 0.95,
                               top_k: int = 40, stream: bool = False, stop=None, max_tokens: int = 256,
                               repeat_penalty: float = 1.1, **kw):
        stops = ([stop] if isinstance(stop, str) else list(stop or [])) + ["### Human:"]
        r = self.create_completion(self._chat_prompt(messages), max_tokens=max_tokens, temperature=temperature,
                                   top_p=top_p, top_k=top_k, stream=stream, stop=stops,
                                   repeat_penalty=repeat_penalty, **kw)
        if stream:
            def chunks():
                first = True
                for c in r:
                    ch = c["choices"][0]
                    delta = {"role": "assistant"} if first else {}
                    first = False
                    if ch["text"]:
                        delta["content"] = ch["text"]
                    yield {"id": "chat" + c["id"], "object": "chat.completion.chunk", "created": c["created"],
                           "model": c["model"],
                           "choices": [{"index": 0, "delta": delta, "finish_reason": ch["finish_reason"]}]}
            return chunks()
        ch = r["choices"][0]
        return {"id": "chat" + r["id"], "object": "chat.completion", "created": r["created"], "model": r["model"],
                "choices": [{"index": 0, "message": {"role": "assistant", "content": ch["text"]},
                             "finish_reason": ch["finish_reason"]}], "usage": r["usage"]}

    # ----------------------------------------------------------------- embeddings
    def embed(self, input: str) -> List[float]:
        """Mean-pooled final hidden state (resets the context)."""
        toks = self.tokenize(input)
        if len(toks) > self.n_ctx():
            raise ValueError(f"Requested tokens exceed context window of {self.n_ctx()}")
        return self.ctx.hidden(toks).float().mean(0).cpu().tolist()

    def create_embedding(self, input: Union[str, List[str]], model=None) -> dict:
        inputs = [input] if isinstance(input, str) else list(input)
        data, total = [], 0
        for i, t in enumerate(inputs):
            total += len(self.tokenize(t))
            data.append({"object": "embedding", "embedding": self.embed(t), "index": i})
        return {"object": "list", "data": data, "model": model or self.model_path or "model",
                "usage": {"prompt_tokens": total, "total_tokens": total}}

    # ----------------------------------------------------------------- info
    def n_ctx(self) -> int:
        return self.ctx._n_ctx

    def n_embd(self) -> int:
        return int(self.model.config.hidden_size)

    def n_vocab(self) -> int:
        return int(self.model.config.vocab_size)

    def token_eos(self) -> int:
        e = getattr(self.tokenizer, "eos_token_id", None)
        return -1 if e is None else int(e)

    def token_bos(self) -> int:
        b = getattr(self.tokenizer, "bos_token_id", None)
        return -1 if b is None else int(b)

    def token_nl(self) -> int:
        ids = self.tokenizer.encode("\n", add_special_tokens=False)
        return int(ids[-1]) if ids else -1

    @staticmethod
    def logits_to_logprobs(logits: List[float]) -> List[float]:
        return torch.log_softmax(torch.tensor(logits, dtype=torch.float64), -1).tolist()

    longest_token_prefix = staticmethod(longest_token_prefix)


# family wrappers: the engine underneath serves any supported architecture
class Gptneox(Llama):
    pass


class Bloom(Llama):
    pass


class Starcoder(Llama):
    pass


_FAMILIES = {"llama": Llama, "gptneox": Gptneox, "bloom": Bloom, "starcoder": Starcoder}


class AutoModelForCausalLM:
    """``from_pretrained(path, model_family=...)`` -> a family wrapper."""

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path: str, model_family: str = "llama", **kwargs):
        if model_family not in _FAMILIES:
            raise ValueError(f"model_family must be one of {sorted(_FAMILIES)}, got {model_family}")
        return _FAMILIES[model_family](pretrained_model_name_or_path, **kwargs)
