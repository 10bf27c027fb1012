"""Typed settings: from_pretrained kwargs > environment > defaults.

Reference: no config framework -- kwargs of ``from_pretrained``
(``model.py:115-157``) plus environment variables.  The
reference variable names are accepted as aliases so existing launch scripts
keep working; ``IPEX_LLM_AMD_*`` names take precedence.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, fields
from typing import Optional


def _env(*names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v is not None and v != "":
            return v
    return default


def _flag(*names, default=False) -> bool:
    v = _env(*names)
    if v is None:
        return default
    return v.strip().lower() in ("1", "true", "yes", "on")


@dataclass
class Settings:
    quantize_kv_cache: bool = False        # fp8 KV cache
    compress_kv_cache: bool = False        # SnapKV-style compression at prefill
    compress_kv_window: int = 32
    compress_kv_capacity: int = 1024
    compress_kv_pool: int = 7
    performance_mode: bool = False         # auto prompt-lookup for long prompts
    low_mem: bool = False
    last_lm_head: bool = True              # last-token-only lm_head at prefill
    kv_block_size: int = 64
    fastapi_timeout: int = 60
    custom_all_reduce: bool = True         # one-shot xGMI all-reduce for TP
    custom_all_reduce_max_bytes: int = 1 << 20
    allow_torch_fallback: bool = False     # GPU ops without the HIP extension (debug only)
    gemv_force_v1: bool = False
    linear_threshold: int = 512            # CPU: dequant + matmul above this many rows

    @classmethod
    def from_env(cls) -> "Settings":
        s = cls()
        s.quantize_kv_cache = _flag("IPEX_LLM_AMD_QUANTIZE_KV_CACHE", "IPEX_LLM_QUANTIZE_KV_CACHE",
                                    "BIGDL_QUANTIZE_KV_CACHE")
        s.compress_kv_cache = _flag("IPEX_LLM_AMD_COMPRESS_KV_CACHE", "IPEX_LLM_COMPRESS_KV_CACHE")
        s.performance_mode = _flag("IPEX_LLM_AMD_PERFORMANCE_MODE", "IPEX_LLM_PERFORMANCE_MODE")
        s.low_mem = _flag("IPEX_LLM_AMD_LOW_MEM", "IPEX_LLM_LOW_MEM")
        s.last_lm_head = _flag("IPEX_LLM_AMD_LAST_LM_HEAD", "IPEX_LLM_LAST_LM_HEAD", default=True)
        s.kv_block_size = int(_env("IPEX_LLM_AMD_KV_BLOCK_SIZE", default=64))
        s.fastapi_timeout = int(_env("IPEX_LLM_FASTAPI_TIMEOUT", default=60))
        s.custom_all_reduce = _flag("IPEX_LLM_AMD_CUSTOM_AR", default=True)
        s.allow_torch_fallback = _flag("IPEX_LLM_AMD_ALLOW_TORCH_FALLBACK")
        s.gemv_force_v1 = _flag("ILLM_GEMV_V1")
        s.linear_threshold = int(_env("IPEX_LLM_AMD_LINEAR_THRESHOLD", "BIGDL_LLM_LINEAR_THRESHOLD", default=512))
        return s

    def update(self, **kwargs) -> "Settings":
        names = {f.name for f in fields(self)}
        for k, v in kwargs.items():
            if k in names and v is not None:
                setattr(self, k, v)
        return self


_SETTINGS: Optional[Settings] = None


def get_settings(refresh: bool = False) -> Settings:
    global _SETTINGS
    if _SETTINGS is None or refresh:
        _SETTINGS = Settings.from_env()
    return _SETTINGS
