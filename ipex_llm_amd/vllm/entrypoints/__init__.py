"""vLLM-style entry points (reference ``SRC/vllm/xpu/entrypoints``)."""
