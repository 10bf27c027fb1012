"""vLLM integration (reference ``SRC/vllm``): low-bit parallel linears and the
model-runner load hook for a vLLM install (``model_convert``), and the
reference's engine classes / OpenAI entry point on the native engine
(``engine``, ``entrypoints.openai.api_server``) where vLLM is absent."""
from .engine import (CompletionOutput, EngineArgs, IPEXLLMAsyncLLMEngine, IPEXLLMClass,  # noqa: F401
                     IPEXLLMLLMEngine, RequestOutput, SamplingParams)
from .model_convert import VLLMLowBitLinear, convert_vllm_linears, get_load_function, patch_vllm  # noqa: F401
