"""ipex_llm_amd.generation"""
