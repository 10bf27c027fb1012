"""LangChain-style wrappers (reference ``SRC/langchain/*``: TransformersLLM,
TransformersPipelineLLM, TransformersEmbeddings / BgeEmbeddings).  When
``langchain_core`` is importable the classes subclass its ``LLM`` /
``Embeddings`` interfaces; otherwise they are standalone with the same
methods (``invoke``, ``__call__``, ``stream``, ``embed_documents``,
``embed_query``)."""
from .llms import TransformersLLM, TransformersPipelineLLM  # noqa: F401
from .embeddings import TransformersEmbeddings, TransformersBgeEmbeddings  # noqa: F401
