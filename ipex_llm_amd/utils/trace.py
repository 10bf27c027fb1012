"""Tracing ranges: roctx ranges around engine steps and decoder
layers, visible in ``rocprofv3 --marker-trace`` / torch.profiler timelines.

Reference: BenchmarkWrapper's per-step timing (``SRC/utils/benchmark_util_4_47.py``)
and ``record_function`` in the NPU path (``npu_models/mp_models_base.py:101``).
Off unless ``IPEX_LLM_TRACE=1`` (a disabled range costs one attribute read);
with it on, every range is both a roctx push/pop (``torch.cuda.nvtx`` maps to
roctx on ROCm) and a ``torch.profiler.record_function`` scope.  Ranges are
host-side: inside a hipGraph replay only the outer replay range appears.
"""
from __future__ import annotations

import contextlib
import os

import torch

ENABLED = os.environ.get("IPEX_LLM_TRACE", "0") == "1"


def enable(on: bool = True):
    global ENABLED
    ENABLED = on


@contextlib.contextmanager
def _range(name: str):
    pushed = False
    try:
        if torch.cuda.is_available():
            torch.cuda.nvtx.range_push(name)
            pushed = True
    except Exception:   # pragma: no cover - no roctx in this build
        pushed = False
    with torch.profiler.record_function(name):
        try:
            yield
        finally:
            if pushed:
                torch.cuda.nvtx.range_pop()


def trace_range(name: str):
    """``with trace_range("layer3"): ...`` -- a no-op unless tracing is enabled."""
    return _range(name) if ENABLED else contextlib.nullcontext()
