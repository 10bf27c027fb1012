"""llama.cpp-python-compatible model API (reference ``SRC/ggml/model``)."""
from .model import AutoModelForCausalLM, Bloom, Gptneox, Llama, LlamaCache, LlamaState, Starcoder  # noqa: F401
