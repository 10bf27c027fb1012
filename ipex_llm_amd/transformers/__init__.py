"""ipex_llm_amd.transformers"""
