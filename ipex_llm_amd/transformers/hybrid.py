"""Hybrid CPU/GPU execution for MoE models too large for GPU memory.

Reference: ``SRC/transformers/convert.py:2142-2166`` (``convert_model_hybrid``:
DeepSeek-V3 attention and the first ``first_k_dense_replace`` dense MLPs move
to the GPU in fp16 with forwards that carry activations across the device
boundary; the MoE experts stay in host memory) and
``models/deepseek_v3.py:45-233`` (the hybrid forwards).

Here it applies to any decoder: every attention module and every dense
(non-expert) MLP becomes a *device island* -- its weights live on the GPU
(low-bit layers convert to the MFMA tile layout on the move), inputs are
moved in and outputs moved back -- while everything else, notably the expert
banks, stays on the host (low-bit experts run on the C++ CPU GEMM).  With
288 GB of HBM per MI355X this is only needed for the largest MoE models
(DeepSeek-V3/R1 671B at INT4 is ~350 GB); smaller ones run fully on device.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn


def _move(x, device):
    if isinstance(x, torch.Tensor):
        return x.to(device, non_blocking=True)
    if isinstance(x, tuple):
        return tuple(_move(v, device) for v in x)
    if isinstance(x, list):
        return [_move(v, device) for v in x]
    if isinstance(x, dict):
        return {k: _move(v, device) for k, v in x.items()}
    return x            # caches and other objects pass through


class DeviceIsland(nn.Module):
    """Runs ``inner`` on ``device``; arguments go in, results come back to
    the caller's device (taken from the first tensor argument)."""

    def __init__(self, inner: nn.Module, device, dtype: Optional[torch.dtype] = None):
        super().__init__()
        self.inner = inner.to(device)
        if dtype is not None:
            for p in self.inner.parameters():
                if p.is_floating_point() and p.dtype != dtype:
                    p.data = p.data.to(dtype)
        self.device = torch.device(device)
        self.dtype = dtype

    def _apply(self, fn, recurse=True):
        return self              # the island stays where it was placed when the host model moves

    def forward(self, *args, **kwargs):
        home = next((a.device for a in list(args) + list(kwargs.values()) if isinstance(a, torch.Tensor)), None)
        in_dt = next((a.dtype for a in list(args) + list(kwargs.values())
                      if isinstance(a, torch.Tensor) and a.is_floating_point()), None)
        args, kwargs = _move(args, self.device), _move(kwargs, self.device)
        if self.dtype is not None:
            cast = lambda v: v.to(self.dtype) if isinstance(v, torch.Tensor) and v.is_floating_point() else v
            args = tuple(cast(a) for a in args)
            kwargs = {k: cast(v) for k, v in kwargs.items()}
        out = self.inner(*args, **kwargs)
        if home is None:
            return out
        out = _move(out, home)
        if self.dtype is not None and in_dt is not None:
            fix = lambda v: v.to(in_dt) if isinstance(v, torch.Tensor) and v.is_floating_point() else v
            out = tuple(fix(o) for o in out) if isinstance(out, tuple) else fix(out)
        return out


def _is_attention(name: str, m: nn.Module) -> bool:
    return name in ("self_attn", "attention", "attn") or type(m).__name__.endswith("Attention")


def _is_dense_mlp(name: str, m: nn.Module) -> bool:
    return name in ("mlp", "feed_forward") and not hasattr(m, "experts")


def convert_model_hybrid(model: nn.Module, device=None, dtype: Optional[torch.dtype] = None,
                         dense_mlp_layers: Optional[int] = None) -> nn.Module:
    """Keep ``model`` on the host, move attention + dense MLPs to ``device``.
    ``dense_mlp_layers``: only the first k layers' MLPs (default:
    ``config.first_k_dense_replace`` when present, else every non-MoE MLP)."""
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
    # the native whole-model forward assumes one device: fall back to the HF forward
    for attr in ("forward", "generate"):
        if attr in model.__dict__:
            del model.__dict__[attr]
    model.__dict__.pop("_illm_state", None)
    model._illm_native_attached = False
    from .hf_views import restore_hf_views
    restore_hf_views(model)                 # q/k/v and gate/up views over the merged weights
    cfg = getattr(model, "config", None)
    k = dense_mlp_layers if dense_mlp_layers is not None else getattr(cfg, "first_k_dense_replace", None)
    base = getattr(model, "model", None)
    layers = getattr(base, "layers", None)
    if layers is None:
        raise ValueError("convert_model_hybrid: cannot find the decoder layer list")
    for i, layer in enumerate(layers):
        for name, child in list(layer.named_children()):
            if isinstance(child, DeviceIsland):
                continue
            if _is_attention(name, child) or (_is_dense_mlp(name, child) and (k is None or i < k)):
                setattr(layer, name, DeviceIsland(child, device, dtype))
    model._illm_hybrid = {"device": str(device)}
    return model
