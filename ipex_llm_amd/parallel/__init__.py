"""ipex_llm_amd.parallel"""
