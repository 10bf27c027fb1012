"""vLLM integration (reference ``SRC/vllm``): low-bit parallel linears and the
model-runner load hook."""
from .model_convert import VLLMLowBitLinear, convert_vllm_linears, get_load_function, patch_vllm  # noqa: F401
