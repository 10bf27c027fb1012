from .api import AutoModelForCausalLM, Bloom, Gptneox, Llama, Starcoder  # noqa: F401
from .llama import LlamaCache, LlamaState  # noqa: F401
