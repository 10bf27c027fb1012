"""RWKV-4: the WKV recurrence as a HIP kernel (reference
``xe_linear.rwkv_linear_attention_v4`` / ``rwkv_time_shift``,
``SRC/transformers/models/rwkv4.py:60-171``).

The HF RWKV forward computes WKV through ``modeling_rwkv.rwkv_linear_attention``
(a CUDA extension it cannot build here, else a Python time loop).  ``patch_rwkv``
routes GPU calls to ``ipex_llm_amd::rwkv_wkv4`` (one thread per channel, f32
max-normalised state, every time step in one launch) and leaves CPU calls on
the HF path.  The time shift is a plain pad/cat in the HF module already.
"""
from __future__ import annotations

import torch


def rwkv_linear_attention_native(time_decay, time_first, key, value, state=None, return_state=False):
    B, T, C = key.shape
    if state is None:
        num = torch.zeros(B, C, dtype=torch.float32, device=key.device)
        den = torch.zeros_like(num)
        mx = torch.full_like(num, -1e38)
    else:
        num, den, mx = (s.float().contiguous().clone() for s in state)
    out = torch.ops.ipex_llm_amd.rwkv_wkv4(time_decay, time_first, key, value, num, den, mx)
    new_state = [num, den, mx] if (return_state or state is not None) else None
    return out, new_state


def patch_rwkv():
    """Route HF RWKV's WKV to the HIP kernel for GPU tensors (idempotent)."""
    import transformers.models.rwkv.modeling_rwkv as M
    if getattr(M.rwkv_linear_attention, "_illm", False):
        return
    orig = M.rwkv_linear_attention

    def rwkv_linear_attention(time_decay, time_first, key, value, state=None, return_state=False):
        from .. import ops
        if key.is_cuda and ops.native_gpu(key):
            return rwkv_linear_attention_native(time_decay, time_first, key, value, state, return_state)
        return orig(time_decay, time_first, key, value, state=state, return_state=return_state)

    rwkv_linear_attention._illm = True
    M.rwkv_linear_attention = rwkv_linear_attention


@torch.no_grad()
def prescale_rwkv(model):
    """Apply HF RWKV's inference-time layer rescaling (``_rescale_layers``:
    output / value weights divided by 2 every ``rescale_every`` blocks) to the
    dense weights *before* quantization and mark the model rescaled, so the
    in-place division never touches packed low-bit weights (inference only)."""
    base = getattr(model, "rwkv", None)
    every = getattr(model.config, "rescale_every", 0)
    if base is None or every <= 0 or getattr(base, "layers_are_rescaled", False):
        return model
    for block_id, block in enumerate(base.blocks):
        f = 2 ** int(block_id // every)
        block.attention.output.weight.div_(f)
        block.feed_forward.value.weight.div_(f)
    base.layers_are_rescaled = True
    return model
