"""HIP flash attention (forward + backward) for the HF-forward training path.

Reference: the QLoRA recipe trains through HF's attention (SDPA), which on
ROCm runs AOTriton kernels (``attn_fwd``, ``bwd_kernel_dk_dv``,
``bwd_kernel_dq``).  Here the HF ``AttentionInterface`` entry ``illm_flash``
routes causal self-attention (no padding mask) through the hand-written
gfx950 kernels of ``csrc/hip/train_attn.hip``: a forward that keeps only the
per-row log-sum-exp, and a deterministic two-kernel backward (dK / dV per
key block with the group's query heads swept in registers, dQ per query
block).  Bidirectional self-attention (``is_causal`` False: BERT / ViT /
Whisper-encoder layers) takes the same forward without the causal mask, for
any sequence length at inference (ragged tails masked in the kernel).
Anything else (padding masks, dropout, sliding windows, soft-capping, head
dims other than 64 / 128, cross-attention, T % 64 != 0 with gradients)
falls back to SDPA.
"""
from __future__ import annotations

from typing import Optional

import torch

NAME = "illm_flash"


class _FlashAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale: float, causal: bool):
        out, lse = torch.ops.ipex_llm_amd.train_attn_fwd(q, k, v, scale, causal)
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.scale, ctx.causal = scale, causal
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        dq, dk, dv = torch.ops.ipex_llm_amd.train_attn_bwd(q, k, v, out, lse, dout.contiguous(), ctx.scale,
                                                           ctx.causal)
        return dq, dk, dv, None, None


def flash_attention(q, k, v, scale: Optional[float] = None, causal: bool = True):
    """q [B, Hq, T, D], k / v [B, Hkv, T, D] -> out [B, T, Hq, D]"""
    if scale is None:
        scale = q.shape[-1] ** -0.5
    return _FlashAttn.apply(q, k, v, float(scale), causal)


def supported(q, k, v, attention_mask, dropout, kwargs) -> bool:
    from .. import ops
    if not (q.is_cuda and ops.native_gpu(q)) or q.dtype not in (torch.bfloat16, torch.float16):
        return False
    if dropout or kwargs.get("sliding_window") or kwargs.get("softcap"):
        return False
    if attention_mask is not None:
        return False
    B, Hq, T, D = q.shape
    grad = torch.is_grad_enabled() and (q.requires_grad or k.requires_grad or v.requires_grad)
    # the forward takes ragged T (encoders at inference); the backward needs T % 64 == 0
    return (D in (64, 128) and (T % 64 == 0 or not grad) and k.shape[2] == T and Hq % k.shape[1] == 0
            and q.stride(-1) == 1 and k.stride(-1) == 1 and v.stride(-1) == 1)


def illm_flash_attention_forward(module, query, key, value, attention_mask, scaling: Optional[float] = None,
                                 dropout: float = 0.0, **kwargs):
    """causal decoders (training) and bidirectional encoders (bert / vit /
    whisper-encoder self-attention: ``module.is_causal`` False, no padding)"""
    causal = kwargs.get("is_causal")
    causal = bool(getattr(module, "is_causal", True) if causal is None else causal)
    if supported(query, key, value, attention_mask, dropout if module.training else 0.0, kwargs):
        return flash_attention(query, key, value, scaling, causal=causal), None
    from transformers.integrations.sdpa_attention import sdpa_attention_forward
    return sdpa_attention_forward(module, query, key, value, attention_mask, scaling=scaling, dropout=dropout,
                                  **kwargs)


_registered = False


def register() -> str:
    global _registered
    if not _registered:
        from transformers import AttentionInterface
        AttentionInterface.register(NAME, illm_flash_attention_forward)
        try:  # sdpa's mask convention: None for plain causal batches
            from transformers.masking_utils import AttentionMaskInterface, sdpa_mask
            AttentionMaskInterface.register(NAME, sdpa_mask)
        except Exception:  # pragma: no cover
            pass
        _registered = True
    return NAME


def patch_flash_attention(model) -> bool:
    """switch an HF model's attention implementation to ``illm_flash``"""
    cfg = getattr(model, "config", None)
    if cfg is None:
        return False
    name = register()
    try:
        model.set_attn_implementation(name)
    except Exception:
        cfg._attn_implementation = name
    return True
