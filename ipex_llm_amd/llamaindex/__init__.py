"""LlamaIndex-style LLM wrapper (reference ``SRC/llamaindex/llms/bigdlllm.py``:
``IpexLLM`` with complete / stream_complete / chat).  Standalone when
``llama_index`` is not installed."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterator, List, Optional


@dataclass
class CompletionResponse:
    text: str
    delta: Optional[str] = None


class IpexLLM:
    def __init__(self, model=None, tokenizer=None, max_new_tokens: int = 128, generate_kwargs=None,
                 messages_to_prompt=None, completion_to_prompt=None):
        self.model, self.tokenizer = model, tokenizer
        self.max_new_tokens = max_new_tokens
        self.generate_kwargs = generate_kwargs or {}
        self.messages_to_prompt = messages_to_prompt or (
            lambda msgs: "".join(f"{m['role']}: {m['content']}\n" for m in msgs) + "assistant:")
        self.completion_to_prompt = completion_to_prompt or (lambda s: s)

    @classmethod
    def from_model_id(cls, model_name: str, device_map: str = "cuda", low_bit: str = "sym_int4", **kw):
        from transformers import AutoTokenizer
        from ..transformers import AutoModelForCausalLM
        m = AutoModelForCausalLM.from_pretrained(model_name, load_in_low_bit=low_bit).to(device_map)
        return cls(m, AutoTokenizer.from_pretrained(model_name), **kw)

    def complete(self, prompt: str, formatted: bool = False, **kwargs) -> CompletionResponse:
        p = prompt if formatted else self.completion_to_prompt(prompt)
        dev = next(self.model.parameters()).device
        ids = self.tokenizer(p, return_tensors="pt").input_ids.to(dev)
        out = self.model.generate(ids, max_new_tokens=self.max_new_tokens, **{**self.generate_kwargs, **kwargs})
        return CompletionResponse(self.tokenizer.decode(out[0][ids.shape[1]:], skip_special_tokens=True))

    def stream_complete(self, prompt: str, formatted: bool = False, **kwargs) -> Iterator[CompletionResponse]:
        import threading
        from transformers import TextIteratorStreamer
        p = prompt if formatted else self.completion_to_prompt(prompt)
        dev = next(self.model.parameters()).device
        ids = self.tokenizer(p, return_tensors="pt").input_ids.to(dev)
        st = TextIteratorStreamer(self.tokenizer, skip_prompt=True, skip_special_tokens=True)
        th = threading.Thread(target=self.model.generate, args=(ids,),
                              kwargs={"max_new_tokens": self.max_new_tokens, "streamer": st, **kwargs})
        th.start()
        text = ""
        for d in st:
            text += d
            yield CompletionResponse(text, d)
        th.join()

    def chat(self, messages: List[dict], **kwargs) -> CompletionResponse:
        return self.complete(self.messages_to_prompt(messages), formatted=True, **kwargs)
