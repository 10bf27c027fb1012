"""Prefill-size (M > 64) low-bit GEMM dispatch.

The MFMA kernel with in-LDS dequant (``csrc/hip/lowbit_gemm.hip``) is used
when present; otherwise the weight is dequantized on device into a transient
bf16/f16 tile and multiplied with the library GEMM.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def lowbit_gemm(x, blob, fmt, n, k, bias=None):
    ops = torch.ops.ipex_llm_amd
    if hasattr(ops, "gemm"):
        return ops.gemm(x, blob, fmt, n, k, bias)
    w = ops.dequantize_device(blob, fmt, n, k, x.dtype)
    return F.linear(x, w, bias)
