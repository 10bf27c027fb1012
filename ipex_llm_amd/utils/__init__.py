"""ipex_llm_amd.utils"""
