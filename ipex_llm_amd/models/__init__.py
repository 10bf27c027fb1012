"""ipex_llm_amd.models"""
