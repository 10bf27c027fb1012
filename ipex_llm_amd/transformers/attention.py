"""Eager attention for the HF-forward families, with the row softmax on the
in-place HIP kernel.

Reference: ``models/common.py:174-181`` (``attention_softmax`` ->
``xe_addons.attn_softmax_inplaced``), called from the eager attention of
aquila, gemma, phi, phi3, minicpmv, mllama, qwen2_vl, baichuan_m1 ... .

Architectures the native decoder does not run keep their HF forward; when
such a model is configured for ``eager`` attention (``output_attentions``,
soft-capping, remote-code models) ``_optimize_post`` switches it to the
``"illm_eager"`` implementation registered here: scores in the activation
dtype, softmax in place on the GPU (f32 math, a fully masked row is zeros),
no extra [B, H, Lq, Lk] f32 copy.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import ops

NAME = "illm_eager"


def _repeat_kv(x: torch.Tensor, n: int) -> torch.Tensor:
    if n == 1:
        return x
    b, h, s, d = x.shape
    return x[:, :, None].expand(b, h, n, s, d).reshape(b, h * n, s, d)


def illm_eager_attention_forward(module: torch.nn.Module, query: torch.Tensor, key: torch.Tensor,
                                 value: torch.Tensor, attention_mask: Optional[torch.Tensor],
                                 scaling: Optional[float] = None, dropout: float = 0.0, **kwargs):
    """HF AttentionInterface signature: q [B, Hq, Lq, D], k/v [B, Hkv, Lk, D]
    -> (out [B, Lq, Hq, D], weights [B, Hq, Lq, Lk])."""
    groups = query.shape[1] // key.shape[1]
    key, value = _repeat_kv(key, groups), _repeat_kv(value, groups)
    if scaling is None:
        scaling = query.shape[-1] ** -0.5
    w = torch.matmul(query, key.transpose(2, 3)) * scaling
    softcap = kwargs.get("softcap", None) or getattr(module, "attn_logit_softcapping", None)
    if softcap:
        w = torch.tanh(w / softcap) * softcap
    if attention_mask is not None:
        w = w + attention_mask[:, :, :, : key.shape[-2]]
    w = ops.attn_softmax_(w.contiguous())
    if dropout and module.training:
        w = torch.nn.functional.dropout(w, p=dropout, training=True)
    out = torch.matmul(w.to(value.dtype), value).transpose(1, 2).contiguous()
    return out, w


_registered = False


def register() -> str:
    global _registered
    if not _registered:
        try:
            from transformers import AttentionInterface
            AttentionInterface.register(NAME, illm_eager_attention_forward)
            try:   # the additive float mask HF builds for "eager"
                from transformers.masking_utils import AttentionMaskInterface, eager_mask
                AttentionMaskInterface.register(NAME, eager_mask)
            except Exception:   # pragma: no cover - older transformers build masks per model
                pass
        except Exception:   # pragma: no cover - transformers without the interface
            return "eager"
        _registered = True
    return NAME


def patch_eager_attention(model: torch.nn.Module) -> bool:
    """Route an eager-configured HF model through ``illm_eager``."""
    cfg = getattr(model, "config", None)
    if cfg is None or getattr(cfg, "_attn_implementation", None) != "eager":
        return False
    name = register()
    if name == "eager":
        return False
    for m in model.modules():
        c = getattr(m, "config", None)
        if c is not None and getattr(c, "_attn_implementation", None) == "eager":
            try:
                c._attn_implementation = name
            except Exception:   # pragma: no cover
                return False
    return True
