"""LangChain-style wrappers (reference ``SRC/langchain/*``: TransformersLLM,
TransformersPipelineLLM, TransformersEmbeddings / BgeEmbeddings; the native
``BigdlNativeLLM`` / ``LlamaLLM`` / ... and ``*Embeddings`` over the ggml-style
``Llama`` family, and the vLLM wrapper over the continuous-batching engine).  When
``langchain_core`` is importable the classes subclass its ``LLM`` /
``Embeddings`` interfaces; otherwise they are standalone with the same
methods (``invoke``, ``__call__``, ``stream``, ``embed_documents``,
``embed_query``)."""
from .llms import TransformersLLM, TransformersPipelineLLM  # noqa: F401
from .embeddings import TransformersEmbeddings, TransformersBgeEmbeddings  # noqa: F401
from .native import (BigdlNativeEmbeddings, BigdlNativeLLM, BloomEmbeddings, BloomLLM,  # noqa: F401
                     GptneoxEmbeddings, GptneoxLLM, LlamaEmbeddings, LlamaLLM, StarcoderEmbeddings,
                     StarcoderLLM, VLLM)
