"""ipex_llm_amd.engine"""
