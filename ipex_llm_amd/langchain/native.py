"""LangChain wrappers over the llama.cpp-style native model API
(``ipex_llm_amd.ggml.Llama`` / ``Gptneox`` / ``Bloom`` / ``Starcoder``) and a
vLLM-style offline batch LLM over the continuous-batching engine.

Reference: ``SRC/langchain/llms/bigdlllm.py`` (``BigdlNativeLLM`` :58,
``_BaseCausalLM`` :360, ``LlamaLLM`` / ``BloomLLM`` / ``GptneoxLLM`` /
``StarcoderLLM`` :675-690), ``SRC/langchain/embeddings/bigdlllm.py``
(``BigdlNativeEmbeddings`` :58, ``_BaseEmbeddings`` :204, ``LlamaEmbeddings``
... :367-382) and ``SRC/langchain/vllm/vllm.py`` (``VLLM`` :52).

The reference classes are pydantic models of ``langchain.llms.base.LLM``
whose ``client`` is the ggml model; their ``_call`` streams
``client(prompt, stream=True, ...)`` chunks (llama-cpp-python completion
dicts) and concatenates the text, ``get_num_tokens`` tokenizes with the
client, embeddings call ``client.embed``.  Here the client is the native
``Llama`` family wrapper (GGUF / HF / low-bit checkpoints on the MI355X
engine).  When ``langchain_core`` is importable the classes also subclass
its ``LLM`` / ``Embeddings`` interfaces; this image has no LangChain, so the
same methods (``invoke``, ``__call__``, ``stream``, ``generate``,
``embed_documents``, ``embed_query``) are provided standalone.  Parity with
LangChain's own runtime behaviour (callbacks, pydantic validation) is
unpinned here: the package is not installed.
"""
from __future__ import annotations

from typing import Any, Dict, Iterator, List, Optional

try:  # optional dependency
    from langchain_core.language_models.llms import LLM as _LLMBase
    from langchain_core.embeddings import Embeddings as _EmbBase
except ImportError:  # pragma: no cover - not installed in this image
    _LLMBase = object
    _EmbBase = object

# model family -> class of ipex_llm_amd.ggml (reference family_info)
FAMILY_INFO = {
    "llama": "Llama",
    "gptneox": "Gptneox",
    "bloom": "Bloom",
    "starcoder": "Starcoder",
}

_MODEL_PARAMS = ("n_ctx", "seed", "logits_all", "n_batch", "last_n_tokens_size")


def _family_class(family: str):
    from .. import ggml
    fam = family.lower()
    if fam not in FAMILY_INFO:
        raise ValueError(f"Model family '{family}' is not supported. Valid values are {','.join(FAMILY_INFO)}")
    return getattr(ggml, FAMILY_INFO[fam])


class BigdlNativeLLM(_LLMBase):
    """Completion LLM over a native (llama.cpp-style) model of a family."""

    model_family: str = "llama"
    model_path: str = ""
    n_ctx: int = 512
    seed: int = -1
    logits_all: bool = False
    n_batch: int = 512
    last_n_tokens_size: int = 64
    low_bit: str = "sym_int4"
    suffix: Optional[str] = None
    max_tokens: int = 256
    temperature: float = 0.8
    top_p: float = 0.95
    logprobs: Optional[int] = None
    echo: bool = False
    stop: List[str] = []
    repeat_penalty: float = 1.1
    top_k: int = 40
    streaming: bool = True
    client: Any = None

    def __init__(self, model_path: str = "", client: Any = None, **kwargs):
        params = {k: kwargs.pop(k) for k in list(kwargs) if hasattr(type(self), k) and k != "client"}
        if _LLMBase is not object:
            super().__init__(**kwargs)
        self.model_path = model_path
        self.stop = []
        for k, v in params.items():
            setattr(self, k, v)
        if client is None:
            cls = _family_class(self._family())
            client = cls(model_path, low_bit=self.low_bit,
                         **{k: getattr(self, k) for k in _MODEL_PARAMS})
        self.client = client

    def _family(self) -> str:
        return self.model_family

    @property
    def _default_params(self) -> Dict[str, Any]:
        return {"suffix": self.suffix, "max_tokens": self.max_tokens, "temperature": self.temperature,
                "top_p": self.top_p, "logprobs": self.logprobs, "echo": self.echo,
                "stop_sequences": self.stop, "repeat_penalty": self.repeat_penalty, "top_k": self.top_k}

    @property
    def _identifying_params(self) -> Dict[str, Any]:
        return {"model_path": self.model_path, "model_family": self._family(), **self._default_params}

    @property
    def _llm_type(self) -> str:
        return "BigDL"

    def _get_parameters(self, stop: Optional[List[str]] = None) -> Dict[str, Any]:
        if self.stop and stop is not None:
            raise ValueError("`stop` found in both the input and default params.")
        params = self._default_params
        params.pop("stop_sequences")
        params["stop"] = self.stop or stop or []
        return params

    def _call(self, prompt: str, stop: Optional[List[str]] = None, run_manager=None, **kwargs) -> str:
        if self.streaming:
            return "".join(c["choices"][0]["text"] for c in self.stream(prompt, stop=stop, run_manager=run_manager))
        params = self._get_parameters(stop)
        return self.client(prompt=prompt, **params)["choices"][0]["text"]

    def stream(self, prompt: str, stop: Optional[List[str]] = None, run_manager=None, **kwargs) -> Iterator[dict]:
        """llama-cpp-python completion chunks as they are generated"""
        params = self._get_parameters(stop)
        for chunk in self.client(prompt=prompt, stream=True, **params):
            if run_manager is not None:
                run_manager.on_llm_new_token(token=chunk["choices"][0]["text"], verbose=getattr(self, "verbose", False),
                                             log_probs=chunk["choices"][0].get("logprobs"))
            yield chunk

    def get_num_tokens(self, text: str) -> int:
        return len(self.client.tokenize(text.encode("utf-8")))

    if _LLMBase is object:
        def invoke(self, prompt: str, stop: Optional[List[str]] = None, **kwargs) -> str:
            return self._call(prompt, stop, **kwargs)

        def __call__(self, prompt: str, stop: Optional[List[str]] = None, **kwargs) -> str:
            return self._call(prompt, stop, **kwargs)


class _BaseCausalLM(BigdlNativeLLM):
    """Family-bound native LLM (reference ``_BaseCausalLM``): the family comes
    from the subclass.  ``native=False`` serves the same checkpoint through the
    HF-compatible ``TransformersLLM`` path instead."""

    ggml_model: str = "Llama"
    native: bool = True

    def __init__(self, model_path: str = "", client: Any = None, native: bool = True, **kwargs):
        self.native = native
        if not native and client is None:
            from .llms import TransformersLLM
            client = TransformersLLM.from_model_id(model_path, low_bit=kwargs.get("low_bit", "sym_int4"))
        super().__init__(model_path=model_path, client=client, **kwargs)

    def _family(self) -> str:
        return {v: k for k, v in FAMILY_INFO.items()}[self.ggml_model]

    def _call(self, prompt: str, stop: Optional[List[str]] = None, run_manager=None, **kwargs) -> str:
        if not self.native:
            return self.client._call(prompt, stop, **kwargs)
        return super()._call(prompt, stop, run_manager, **kwargs)

    def get_num_tokens(self, text: str) -> int:
        if not self.native:
            return len(self.client.tokenizer.encode(text))
        return super().get_num_tokens(text)


class LlamaLLM(_BaseCausalLM):
    ggml_model = "Llama"


class BloomLLM(_BaseCausalLM):
    ggml_model = "Bloom"


class GptneoxLLM(_BaseCausalLM):
    ggml_model = "Gptneox"


class StarcoderLLM(_BaseCausalLM):
    ggml_model = "Starcoder"


class BigdlNativeEmbeddings(_EmbBase):
    """Embeddings = the native model's ``embed`` (mean-pooled final hidden state)."""

    model_family: str = "llama"

    def __init__(self, model_path: str = "", client: Any = None, model_family: Optional[str] = None,
                 n_ctx: int = 512, seed: int = -1, n_batch: int = 512, low_bit: str = "sym_int4", **kwargs):
        if model_family is not None:
            self.model_family = model_family
        self.model_path = model_path
        if client is None:
            client = _family_class(self._family())(model_path, embedding=True, n_ctx=n_ctx, seed=seed,
                                                   n_batch=n_batch, low_bit=low_bit)
        self.client = client

    def _family(self) -> str:
        return self.model_family

    def embed_documents(self, texts: List[str]) -> List[List[float]]:
        return [list(map(float, self.client.embed(t))) for t in texts]

    def embed_query(self, text: str) -> List[float]:
        return list(map(float, self.client.embed(text)))


class _BaseEmbeddings(BigdlNativeEmbeddings):
    ggml_model: str = "Llama"

    def _family(self) -> str:
        return {v: k for k, v in FAMILY_INFO.items()}[self.ggml_model]


class LlamaEmbeddings(_BaseEmbeddings):
    ggml_model = "Llama"


class BloomEmbeddings(_BaseEmbeddings):
    ggml_model = "Bloom"


class GptneoxEmbeddings(_BaseEmbeddings):
    ggml_model = "Gptneox"


class StarcoderEmbeddings(_BaseEmbeddings):
    ggml_model = "Starcoder"


class VLLM(_LLMBase):
    """Offline batched generation (reference ``langchain/vllm/vllm.py`` ``VLLM``:
    ``IPEXLLMClass`` engine + ``SamplingParams``) on this library's
    continuous-batching engine (``serving.engine.LLMEngine``: paged KV,
    hipGraph decode buckets, C++ scheduler) instead of vLLM."""

    model: str = ""
    n: int = 1
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = -1
    stop: Optional[List[str]] = None
    ignore_eos: bool = False
    max_new_tokens: int = 512
    load_in_low_bit: str = "sym_int4"
    device: str = "cuda"
    max_num_seqs: int = 64
    client: Any = None
    tokenizer: Any = None

    def __init__(self, model: str = "", client: Any = None, tokenizer: Any = None, **kwargs):
        params = {k: kwargs.pop(k) for k in list(kwargs) if hasattr(type(self), k)}
        if _LLMBase is not object:
            super().__init__(**kwargs)
        self.model = model
        for k, v in params.items():
            setattr(self, k, v)
        if client is None:
            from transformers import AutoTokenizer
            from ..serving.engine import LLMEngine
            from ..transformers import AutoModelForCausalLM
            from ..transformers.hf_native import get_native
            hf = AutoModelForCausalLM.from_pretrained(model, load_in_low_bit=self.load_in_low_bit).to(self.device)
            client = LLMEngine(get_native(hf)[0], max_batch=self.max_num_seqs)
            tokenizer = AutoTokenizer.from_pretrained(model)
        self.client, self.tokenizer = client, tokenizer

    @property
    def _default_params(self) -> Dict[str, Any]:
        return {"n": self.n, "max_tokens": self.max_new_tokens, "top_k": self.top_k, "top_p": self.top_p,
                "temperature": self.temperature, "stop": self.stop, "ignore_eos": self.ignore_eos}

    @property
    def _llm_type(self) -> str:
        return "vllm"

    def _sampling(self, **kwargs):
        from ..serving.engine import SamplingParams
        p = {**self._default_params, **kwargs}
        eos = [] if p["ignore_eos"] or self.tokenizer is None or self.tokenizer.eos_token_id is None \
            else [self.tokenizer.eos_token_id]
        greedy = p["temperature"] <= 0 or (p["top_k"] == 1)
        return SamplingParams(max_new_tokens=p["max_tokens"], temperature=max(p["temperature"], 1e-5),
                              top_k=max(0, p["top_k"]), top_p=p["top_p"], do_sample=not greedy,
                              stop_token_ids=eos)

    def generate_texts(self, prompts: List[str], stop: Optional[List[str]] = None, **kwargs) -> List[str]:
        sp = self._sampling(**kwargs)
        ids = [list(self.tokenizer.encode(p)) for p in prompts]
        outs = self.client.generate(ids, sp)
        texts = []
        for o in outs:
            t = self.tokenizer.decode(o, skip_special_tokens=True)
            for s in (stop or self.stop or []):
                i = t.find(s)
                if i >= 0:
                    t = t[:i]
            texts.append(t)
        return texts

    def _generate(self, prompts: List[str], stop: Optional[List[str]] = None, run_manager=None, **kwargs):
        texts = self.generate_texts(prompts, stop, **kwargs)
        try:
            from langchain_core.outputs import Generation, LLMResult
        except ImportError:  # pragma: no cover
            return [[{"text": t}] for t in texts]
        return LLMResult(generations=[[Generation(text=t)] for t in texts])

    def _call(self, prompt: str, stop: Optional[List[str]] = None, run_manager=None, **kwargs) -> str:
        return self.generate_texts([prompt], stop, **kwargs)[0]

    if _LLMBase is object:
        def invoke(self, prompt: str, stop: Optional[List[str]] = None, **kwargs) -> str:
            return self._call(prompt, stop, **kwargs)

        def __call__(self, prompt: str, stop: Optional[List[str]] = None, **kwargs) -> str:
            return self._call(prompt, stop, **kwargs)

        def generate(self, prompts: List[str], stop: Optional[List[str]] = None, **kwargs):
            return self._generate(prompts, stop, **kwargs)
