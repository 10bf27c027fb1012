"""Fused lm_head + cross-entropy for causal-LM fine-tuning.

Reference: the HF causal-LM loss the QLoRA recipe trains with
(``LlamaForCausalLM.forward`` -> ``logits = lm_head(h)`` -> ``loss_function``
upcasts the [tokens, vocab] logits to f32, softmax, NLL; backward runs the
softmax gradient and a dense ``dlogits @ W`` -- SURVEY §3.5).  With
Llama-3's 128 K vocabulary that is a 2 GB f32 tensor per 4 K-token step and
three full passes over it.

MI355X design: the tokens are processed in chunks; per chunk the logits are
one bf16 GEMM on the dense 8-phase kernel (gemm_8p.hip; ILLM_CE_LIB=1: the
library GEMM), ``ce_fused_``
turns them into the per-row loss and, IN PLACE, the logits gradient
(softmax - onehot) in one read for the row statistics and one read + write
for the gradient, and the hidden-state gradient is the second GEMM
(dlogits @ W) of that chunk -- computed during the forward, since the only
consumer of the loss is a scalar backward.  That second GEMM reduces over
the vocabulary: on the NT 8-phase kernel its operand is W^T, transposed one
vocabulary slice at a time (no resident copy of the head), the slices'
products accumulated in f32 by the kernel epilogue.  Nothing of size [tokens, vocab]
outlives a chunk; backward is one scale of the stored [tokens, hidden]
gradient.  The lm_head weight is frozen here (QLoRA); a trainable head
falls back to the unfused path.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

CHUNK = int(os.environ.get("ILLM_CE_CHUNK", "2048"))
# vocabulary slice of the grad_h GEMM: its W^T operand is transposed per slice
# (VCHUNK x hidden at a time) instead of a resident transposed copy of the
# whole head (1 GB for Llama-3-8B)
VCHUNK = int(os.environ.get("ILLM_CE_VCHUNK", "32768"))
_LIB = os.environ.get("ILLM_CE_LIB", "0") == "1"


def _g8_ok(h, w) -> bool:
    from .. import ops
    return (not _LIB and h.is_cuda and ops.native_gpu(h) and h.dtype == torch.bfloat16 and w.dtype == h.dtype
            and h.shape[1] % 64 == 0 and w.shape[0] % 64 == 0 and hasattr(torch.ops.ipex_llm_amd, "gemm_bf16"))


class _FusedLinearCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, weight, labels, ignore_index: int, denom):
        ops = torch.ops.ipex_llm_amd
        T, H = h.shape
        w = weight if weight.dtype == h.dtype else weight.to(h.dtype)
        V = weight.shape[0]
        loss_rows = torch.empty(T, device=h.device, dtype=torch.float32)
        grad_h = torch.empty_like(h) if h.requires_grad else None
        g8 = _g8_ok(h, w) and V % 64 == 0
        if g8:
            # the 8-phase head GEMMs or the library's, whichever this shape measured faster
            from ..ops.gemm import _pick
            c = min(T, CHUNK)
            g8 = _pick((c, V, H, "ce_head", 0), lambda: ops.gemm_bf16(h[:c], w), lambda: torch.mm(h[:c], w.t())) == "g8d"
        for c0 in range(0, T, CHUNK):
            c1 = min(T, c0 + CHUNK)
            logits = ops.gemm_bf16(h[c0:c1], w) if g8 else torch.mm(h[c0:c1], w.t())
            loss_rows[c0:c1] = ops.ce_fused_(logits, labels[c0:c1], ignore_index, 1.0 if grad_h is not None else 0.0)
            if grad_h is not None:
                if g8:
                    # dlogits @ W, one vocabulary slice at a time, f32 accumulation
                    acc = torch.empty(c1 - c0, H, device=h.device, dtype=torch.float32)
                    for v0 in range(0, V, VCHUNK):
                        v1 = min(V, v0 + VCHUNK)
                        wt = w[v0:v1].t().contiguous()                       # [H, v1 - v0]
                        ops.gemm_bf16(logits[:, v0:v1], wt, None, True, 0, False, 0, -1, acc, v0 > 0)
                        del wt
                    grad_h[c0:c1] = acc
                    del acc
                else:
                    torch.mm(logits, w, out=grad_h[c0:c1])
            del logits
        if denom is None:
            n_valid = (labels != ignore_index).sum().clamp_(min=1).to(torch.float32)
        else:
            # HF ``num_items_in_batch``: the summed loss over the items of the
            # whole (gradient-accumulated) batch, not this micro-batch's mean
            n_valid = torch.as_tensor(denom, device=h.device).to(torch.float32).reshape(())
        ctx.save_for_backward(grad_h, n_valid)
        return loss_rows.sum() / n_valid

    @staticmethod
    def backward(ctx, g):
        grad_h, n_valid = ctx.saved_tensors
        gh = None
        if grad_h is not None and ctx.needs_input_grad[0]:
            gh = grad_h * (g / n_valid).to(grad_h.dtype)
        return gh, None, None, None, None


def fused_linear_cross_entropy(hidden: torch.Tensor, weight: torch.Tensor, labels: torch.Tensor,
                               ignore_index: int = -100, shift: bool = True,
                               num_items_in_batch=None) -> torch.Tensor:
    """CE of ``hidden @ weight^T`` against ``labels`` with HF causal-LM
    semantics: position t predicts label t + 1 when ``shift``; the mean over
    the valid labels, or -- when ``num_items_in_batch`` is given (the HF
    Trainer passes it under gradient accumulation) -- the sum divided by it."""
    H = hidden.shape[-1]
    if shift:
        hidden = hidden[..., :-1, :]
        labels = labels[..., 1:]
    h2 = hidden.reshape(-1, H)
    lab = labels.reshape(-1).to(torch.int64)
    return _FusedLinearCE.apply(h2, weight, lab, ignore_index, num_items_in_batch)


def plain_ce_head(config) -> bool:
    """True when the model's HF loss is plain CE over ``lm_head(h)``: heads that
    soft-cap (Gemma-2 ``final_logit_softcapping``) or scale their logits (Cohere
    ``logit_scale``, Granite ``logits_scaling``) keep the HF forward, which
    applies those terms."""
    if config is None:
        return True
    for name in ("final_logit_softcapping", "output_logit_softcapping"):
        if getattr(config, name, None):
            return False
    for name in ("logit_scale", "logits_scaling", "output_multiplier_scale"):
        v = getattr(config, name, None)
        if v is not None and float(v) != 1.0:
            return False
    return True


def fused_ce_supported(model) -> bool:
    from .. import ops
    head = getattr(model, "lm_head", None)
    w = getattr(head, "weight", None)
    if not plain_ce_head(getattr(model, "config", None)):
        return False
    return (isinstance(head, torch.nn.Linear) and head.bias is None and w is not None and w.is_cuda
            and not w.requires_grad and w.dtype in (torch.bfloat16, torch.float16)
            and w.is_contiguous() and w.shape[1] % 128 == 0 and w.shape[0] % 128 == 0 and ops.native_gpu(w))


def patch_fused_ce(model):
    """Route ``model(input_ids, labels=...)`` of an HF causal LM through the
    fused head + loss while training (logits are not materialised: the
    output's ``logits`` is None).  Inference and unsupported heads keep the
    original forward."""
    if getattr(model, "_illm_fused_ce", False):
        return model
    orig = model.forward

    def forward(*args, labels: Optional[torch.Tensor] = None, **kwargs):
        if (labels is None or not torch.is_grad_enabled() or kwargs.get("return_dict") is False
                or not fused_ce_supported(model)):
            return orig(*args, labels=labels, **kwargs)
        from transformers.modeling_outputs import CausalLMOutputWithPast
        kwargs.pop("logits_to_keep", None)
        n_items = kwargs.pop("num_items_in_batch", None)
        out = model.model(*args, **kwargs)
        loss = fused_linear_cross_entropy(out.last_hidden_state, model.lm_head.weight, labels,
                                          num_items_in_batch=n_items)
        return CausalLMOutputWithPast(loss=loss, logits=None, past_key_values=out.past_key_values,
                                      hidden_states=out.hidden_states, attentions=out.attentions)

    model.forward = forward
    model._illm_fused_ce = True
    return model
