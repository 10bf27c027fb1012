"""RWKV-4 / RWKV-5: the WKV recurrences as HIP kernels (reference
``xe_linear.rwkv_linear_attention_v4`` / ``rwkv_linear_attention_v5`` /
``rwkv_time_shift``, ``SRC/transformers/models/rwkv4.py:60-171`` and
``SRC/transformers/models/rwkv5.py:42-216``).

RWKV-5 ("Eagle") has no transformers class: it is remote code
(``model_type == "rwkv5"``).  ``patch_rwkv5(model)`` replaces the forward of
every time-mix module (the ones carrying ``time_faaaa``) with
``rwkv5_attention_forward``: token-shift mixing, the low-bit r/k/v/gate
projections, the WKV-5 kernel over an f32 [B, H, S, S] state per layer,
per-head GroupNorm, gate and output projection.  The remote code's state
layout is kept (``state[0]`` [B, C, L] shift, ``state[1]`` [B, H, S, S, L]
WKV), so its own model forward and generate loop drive the patched modules.

The HF RWKV forward computes WKV through ``modeling_rwkv.rwkv_linear_attention``
(a CUDA extension it cannot build here, else a Python time loop).  ``patch_rwkv``
routes GPU calls to ``ipex_llm_amd::rwkv_wkv4`` (one thread per channel, f32
max-normalised state, every time step in one launch) and leaves CPU calls on
the HF path.  The time shift is a plain pad/cat in the HF module already.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


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


# ---------------------------------------------------------------- RWKV-5
def rwkv5_wkv(w: torch.Tensor, u: torch.Tensor, r: torch.Tensor, k: torch.Tensor, v: torch.Tensor,
              state: torch.Tensor) -> torch.Tensor:
    """WKV-5 over r/k/v [B, T, H, S]; w = exp(-exp(time_decay)) and
    u = time_first, both [H, S]; ``state`` [B, H, S, S] f32 (key dim i, value
    dim j) is updated in place.  Returns f32 [B, T, H, S]."""
    from .. import ops
    if k.is_cuda and ops.native_gpu(k):
        return torch.ops.ipex_llm_amd.rwkv_wkv5(w, u, r, k, v, state)
    return rwkv5_wkv_reference(w, u, r, k, v, state)


def rwkv5_wkv_reference(w, u, r, k, v, state):
    """fp32 reference of the WKV-5 recurrence (time loop; state in place)."""
    B, T, H, S = k.shape
    w = w.float().reshape(H, S, 1)
    u = u.float().reshape(H, S, 1)
    st = state.float()
    out = torch.empty(B, T, H, S, dtype=torch.float32, device=k.device)
    for t in range(T):
        kt, vt, rt = k[:, t].float(), v[:, t].float(), r[:, t].float()       # [B, H, S]
        a = kt.unsqueeze(-1) * vt.unsqueeze(-2)                               # [B, H, S(i), S(j)]
        out[:, t] = (rt.unsqueeze(-2) @ (u * a + st)).squeeze(-2)
        st = a + w * st
    state.copy_(st)
    return out


def rwkv5_attention_forward(self, hidden: torch.Tensor, state=None, use_cache: bool = False, seq_mode: bool = True):
    """Time-mix block of RWKV-5 (remote-code ``RwkvSelfAttention``)."""
    B, T, C = hidden.shape
    H = self.time_decay.shape[0]
    S = C // H
    li = self.layer_id
    # token shift: the previous step's last hidden state comes from the state
    if T == 1 and state is not None:
        shifted = state[0][:, :, li].unsqueeze(1).to(hidden.dtype)
    else:
        shifted = F.pad(hidden, (0, 0, 1, -1))
        if state is not None:
            shifted[:, 0] = state[0][:, :, li].to(hidden.dtype)
    dx = hidden - shifted

    def mix(m):
        return shifted + dx * m.to(hidden.dtype)        # hidden * m + shifted * (1 - m)

    key = self.key(mix(self.time_mix_key))
    value = self.value(mix(self.time_mix_value))
    receptance = self.receptance(mix(self.time_mix_receptance))
    gate = F.silu(self.gate(mix(self.time_mix_gate)))
    if state is not None:
        state[0][:, :, li] = hidden[:, -1].to(state[0].dtype)

    w = torch.exp(-torch.exp(self.time_decay.float())).reshape(H, S)
    u = self.time_faaaa.float().reshape(H, S)
    if state is not None:
        wkv_state = state[1][..., li].float().contiguous()
    else:
        wkv_state = torch.zeros(B, H, S, S, dtype=torch.float32, device=hidden.device)
    out = rwkv5_wkv(w, u, receptance.view(B, T, H, S), key.view(B, T, H, S), value.view(B, T, H, S), wkv_state)
    if state is not None:
        state[1][..., li] = wkv_state.to(state[1].dtype)
    out = F.group_norm(out.reshape(B * T, H * S), num_groups=H, weight=self.ln_x.weight.float(),
                       bias=self.ln_x.bias.float(), eps=getattr(self.ln_x, "eps", 1e-5))
    out = out.reshape(B, T, C).to(hidden.dtype) * gate
    return self.output(out), state


def patch_rwkv5(model: torch.nn.Module) -> int:
    """Bind ``rwkv5_attention_forward`` to every RWKV-5 time-mix module of
    ``model``; returns how many were patched."""
    import types
    n = 0
    for m in model.modules():
        if all(hasattr(m, a) for a in ("time_faaaa", "time_decay", "time_mix_gate", "ln_x", "output", "layer_id")):
            m.forward = types.MethodType(rwkv5_attention_forward, m)
            n += 1
    return n
