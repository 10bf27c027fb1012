"""ipex_llm_amd.serving"""
