"""ipex_llm_amd.gguf"""
