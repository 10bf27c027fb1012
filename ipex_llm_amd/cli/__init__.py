"""ipex_llm_amd.cli"""
