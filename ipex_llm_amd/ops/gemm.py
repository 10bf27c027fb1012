"""Prefill-size (M > 64) low-bit GEMM dispatch.

M <= 1536: the MFMA kernel with in-register dequant (``csrc/hip/gemm.hip``:
f16 MFMA, weights decoded straight from the tiled blob, never
materialised).  Larger M: dequantize to a transient dense weight + library
GEMM, which is faster there (measured on MI355X, Llama-3-8B shapes, see
profiles/prefill_gemm_r1.jsonl: fused 600-680 TF vs library 1.0-1.2 PF at
M = 4096, parity at M = 1024).  ``ILLM_GEMM_LIB=1`` / ``ILLM_GEMM_FUSED=1``
force either path (A/B measurements).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

_USE_LIB = os.environ.get("ILLM_GEMM_LIB", "0") == "1"
_USE_FUSED = os.environ.get("ILLM_GEMM_FUSED", "0") == "1"
FUSED_MAX_M = 1536


def lowbit_gemm(x, blob, fmt, n, k, bias=None):
    ops = torch.ops.ipex_llm_amd
    M = x.numel() // k
    if not _USE_LIB and (M <= FUSED_MAX_M or _USE_FUSED) and hasattr(ops, "gemm"):
        return ops.gemm(x, blob, fmt, n, k, bias)
    w = ops.dequantize_device(blob, fmt, n, k, x.dtype)
    return F.linear(x, w, bias)


def lowbit_gemm_glu(x, blob, fmt, n, k, act: int = 0):
    """act(x @ Wg^T) * (x @ Wu^T) for a tile-interleaved gate/up weight at
    prefill M: the fused kernel applies the activation in its epilogue (no
    [M, 2I] round trip, no elementwise launches)."""
    ops = torch.ops.ipex_llm_amd
    M = x.numel() // k
    if not _USE_LIB and (M <= FUSED_MAX_M or _USE_FUSED) and hasattr(ops, "gemm_glu"):
        return ops.gemm_glu(x, blob, fmt, n, k, act)
    from ..models.decoder import deinterleave_glu
    g, u = deinterleave_glu(lowbit_gemm(x, blob, fmt, n, k))
    return ((F.silu(g) if act == 0 else F.gelu(g, approximate="tanh")) * u).contiguous()
