from __future__ import annotations

from typing import Any, Iterator, List, Optional

try:  # optional dependency
    from langchain_core.language_models.llms import LLM as _Base
except ImportError:  # pragma: no cover - not installed in this image
    _Base = object


class TransformersLLM(_Base):
    """Text generation on the native engine (reference langchain/llms/transformersllm.py)."""

    model_id: str = ""
    model: Any = None
    tokenizer: Any = None
    model_kwargs: Optional[dict] = None
    generate_kwargs: Optional[dict] = None

    def __init__(self, model=None, tokenizer=None, model_id: str = "", generate_kwargs=None, **kw):
        if _Base is not object:
            super().__init__(**kw)
        self.model, self.tokenizer, self.model_id = model, tokenizer, model_id
        self.generate_kwargs = generate_kwargs or {"max_new_tokens": 64}

    @classmethod
    def from_model_id(cls, model_id: str, model_kwargs: Optional[dict] = None, device: str = "cuda",
                      low_bit: str = "sym_int4", **kwargs):
        from transformers import AutoTokenizer
        from ..transformers import AutoModelForCausalLM
        mk = dict(model_kwargs or {})
        model = AutoModelForCausalLM.from_pretrained(model_id, load_in_low_bit=low_bit, **mk).to(device)
        tok = AutoTokenizer.from_pretrained(model_id)
        return cls(model=model, tokenizer=tok, model_id=model_id, **kwargs)

    @classmethod
    def from_model_id_low_bit(cls, model_id: str, device: str = "cuda", **kwargs):
        from transformers import AutoTokenizer
        from ..transformers import AutoModelForCausalLM
        model = AutoModelForCausalLM.load_low_bit(model_id).to(device)
        return cls(model=model, tokenizer=AutoTokenizer.from_pretrained(model_id), model_id=model_id, **kwargs)

    @property
    def _llm_type(self) -> str:
        return "ipex_llm_amd"

    def _call(self, prompt: str, stop: Optional[List[str]] = None, run_manager=None, **kwargs) -> str:
        dev = next(self.model.parameters()).device
        ids = self.tokenizer(prompt, return_tensors="pt").input_ids.to(dev)
        gk = {**self.generate_kwargs, **kwargs}
        out = self.model.generate(ids, **gk)
        text = self.tokenizer.decode(out[0][ids.shape[1]:], skip_special_tokens=True)
        for s in stop or []:
            i = text.find(s)
            if i >= 0:
                text = text[:i]
        return text

    if _Base is object:
        def invoke(self, prompt: str, stop: Optional[List[str]] = None, **kwargs) -> str:
            return self._call(prompt, stop, **kwargs)

        def __call__(self, prompt: str, stop: Optional[List[str]] = None, **kwargs) -> str:
            return self._call(prompt, stop, **kwargs)

    def stream(self, prompt: str, **kwargs) -> Iterator[str]:
        import threading
        from transformers import TextIteratorStreamer
        dev = next(self.model.parameters()).device
        ids = self.tokenizer(prompt, return_tensors="pt").input_ids.to(dev)
        st = TextIteratorStreamer(self.tokenizer, skip_prompt=True, skip_special_tokens=True)
        th = threading.Thread(target=self.model.generate, args=(ids,),
                              kwargs={**self.generate_kwargs, **kwargs, "streamer": st})
        th.start()
        yield from st
        th.join()


class TransformersPipelineLLM(TransformersLLM):
    """reference TransformersPipelineLLM: same engine, pipeline-style construction"""

    @classmethod
    def from_model_id(cls, model_id: str, task: str = "text-generation", **kwargs):
        if task != "text-generation":
            raise ValueError("only text-generation is supported")
        return super().from_model_id(model_id, **kwargs)
