"""Native op layer: loads ``ipex_llm_amd/_C.so`` and exposes typed wrappers.

Every GPU hot op (low-bit GEMV/GEMM, fused norms, RoPE+KV append, decode
attention, MoE routing, quantize-on-device) is a hand-written gfx950 HIP
kernel registered under ``torch.ops.ipex_llm_amd``.  On a GPU box the
extension MUST load: a missing/broken ``_C.so`` raises instead of silently
falling back to eager PyTorch (set ``IPEX_LLM_AMD_ALLOW_TORCH_FALLBACK=1`` to
opt into the reference implementations in :mod:`ipex_llm_amd.ops.reference`,
which exist for CPU-only test runs).
"""
from __future__ import annotations

import os
import threading

import torch

_LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         os.environ.get("IPEX_LLM_AMD_LIB", "_C.so"))
_lock = threading.Lock()
_loaded = False
_load_error: Exception | None = None


def load(build_if_missing: bool = True) -> bool:
    """Load the native library (building it in-tree first if needed)."""
    global _loaded, _load_error
    if _loaded:
        return True
    with _lock:
        if _loaded:
            return True
        try:
            if not os.path.exists(_LIB_PATH) and build_if_missing:
                from .. import _build
                _build.build()
            torch.ops.load_library(_LIB_PATH)
            from . import _meta  # noqa: F401  register fake impls
            _loaded = True
        except Exception as e:  # pragma: no cover - surfaced by require()
            _load_error = e
    return _loaded


def available() -> bool:
    return load()


def require():
    if not load():
        raise RuntimeError(f"ipex_llm_amd native library failed to load from {_LIB_PATH}: {_load_error!r}. "
                           "Run `python -m ipex_llm_amd._build`.")
    return torch.ops.ipex_llm_amd


def allow_fallback() -> bool:
    return os.environ.get("IPEX_LLM_AMD_ALLOW_TORCH_FALLBACK", "0") == "1"


def native_gpu(t: torch.Tensor) -> bool:
    """True if ``t`` lives on a GPU and the HIP kernels must be used."""
    if not t.is_cuda:
        return False
    if load():
        return True
    if allow_fallback():
        return False
    require()
    return False


from .api import *  # noqa: E402,F401,F403
