"""ipex_llm_amd.training"""
