"""Model converter: graph surgery + low-bit module swap + forward swap.

Reference: ``SRC/transformers/convert.py`` -- ``ggml_convert_low_bit``
(1092-1204) = ``_optimize_pre`` (890-1089: merge qkv, split/pad MLP ...) ->
``_replace_with_low_bit_linear`` (472-752) -> ``_optimize_post`` (1275-2139:
per-arch forward replacement).

Here:
  * ``_optimize_pre`` merges q/k/v into ``qkv_proj`` and gate/up into a
    16-row-tile-interleaved ``gate_up_proj`` (the layout the fused GLU GEMV
    epilogue consumes) for every architecture the native decoder runs;
  * ``_replace_with_low_bit_linear`` swaps ``nn.Linear`` for
    :class:`LowBitLinear` (quantized by the C++ host library, or on the GPU
    when the model already lives there);
  * ``_optimize_post`` attaches the native MI355X decoder
    (:mod:`ipex_llm_amd.models`) as the model's forward/generate for the
    supported architectures; everything else keeps its HF forward running on
    low-bit linears + our RMSNorm kernel (like the reference's generic path).
"""
from __future__ import annotations

import logging
import os
import types
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from ..quantize import qtypes as Q
from .low_bit_linear import BF16Linear, DenseLinear, LowBitLinear

logger = logging.getLogger("ipex_llm_amd")

# architectures whose decoder runs on the native engine
NATIVE_ARCHS = {"llama", "mistral", "qwen2", "qwen3", "gemma", "gemma2", "phi3", "internlm2", "yi",
                "aquila", "olmo2", "minicpm", "glm", "glm4", "yuan"}
# granite (embedding/residual/logit multipliers), stablelm (partial rotary + LayerNorm) and
# starcoder2 (biased LayerNorm MLP, no q_proj split) take the HF forward over low-bit linears.
MOE_ARCHS = {"mixtral", "qwen2_moe", "qwen3_moe"}
# encoder / encoder-decoder families whose HF forward runs (reference
# models/bert.py, whisper.py, mllama.py, minicpmv.py): attention on the HIP
# flash kernel where it applies, linears low-bit
ENCODER_FLASH_ARCHS = {"bert", "roberta", "xlm-roberta", "vit", "whisper", "clip", "siglip", "mllama"}


# ----------------------------------------------------------------- pre
def _interleave(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    from ..models.decoder import interleave_glu_rows
    return interleave_glu_rows(gate, up)


def _merge_linears(mods: List[nn.Linear], interleave_glu: bool = False) -> nn.Linear:
    has_bias = mods[0].bias is not None
    dev, dt = mods[0].weight.device, mods[0].weight.dtype
    if interleave_glu:
        w = _interleave(mods[0].weight.data, mods[1].weight.data)
        b = None
    else:
        w = torch.cat([m.weight.data for m in mods], 0)
        b = torch.cat([m.bias.data for m in mods], 0) if has_bias else None
    out = nn.Linear(w.shape[1], w.shape[0], bias=has_bias, device="meta", dtype=dt)
    out.weight = nn.Parameter(w, requires_grad=False)
    if has_bias:
        out.bias = nn.Parameter(b, requires_grad=False)
    return out


def _merge_qkv(attn: nn.Module):
    if hasattr(attn, "qkv_proj") or not all(hasattr(attn, n) for n in ("q_proj", "k_proj", "v_proj")):
        return
    mods = [attn.q_proj, attn.k_proj, attn.v_proj]
    if all(isinstance(m, LowBitLinear) for m in mods):      # pre-quantized (GPTQ/AWQ) checkpoints
        from .low_bit_linear import lowbit_row_concat
        if len({id(m.g_idx_map) if m.g_idx_map is not None else None for m in mods}) > 1 and \
                any(m.g_idx_map is not None for m in mods):
            return                                           # different act-order permutations
        attn.qkv_proj = lowbit_row_concat(mods)
        attn._illm_qkv_split = tuple(m.out_features for m in mods)
        del attn.q_proj, attn.k_proj, attn.v_proj
        return
    from .low_bit_linear import KQuantLinear, kquant_row_concat
    if any(isinstance(m, KQuantLinear) for m in mods) and \
            all(isinstance(m, (KQuantLinear, nn.Linear)) for m in mods):
        # GGUF k-quant checkpoints (kept in their blocks); dense parts are
        # converted later inside the RowConcatLinear
        attn.qkv_proj = kquant_row_concat(mods)
        attn._illm_qkv_split = tuple(m.out_features for m in mods)
        del attn.q_proj, attn.k_proj, attn.v_proj
        return
    if not all(isinstance(m, nn.Linear) for m in mods):
        return
    attn.qkv_proj = _merge_linears([attn.q_proj, attn.k_proj, attn.v_proj])
    attn._illm_qkv_split = tuple(m.out_features for m in mods)
    del attn.q_proj, attn.k_proj, attn.v_proj


def _merge_gate_up(mlp: nn.Module):
    if hasattr(mlp, "gate_up_proj") and not getattr(mlp, "_illm_interleaved", False) and \
            isinstance(mlp.gate_up_proj, nn.Linear):
        # phi3-style fused [gate; up] -> tile-interleaved
        w = mlp.gate_up_proj.weight.data
        I = w.shape[0] // 2
        mlp.gate_up_proj.weight = nn.Parameter(_interleave(w[:I], w[I:]), requires_grad=False)
        mlp._illm_interleaved = True
        return
    if not all(hasattr(mlp, n) for n in ("gate_proj", "up_proj")):
        return
    if mlp.gate_proj.bias is not None:
        return
    if isinstance(mlp.gate_proj, LowBitLinear) and isinstance(mlp.up_proj, LowBitLinear):
        if mlp.gate_proj.g_idx_map is not None or mlp.up_proj.g_idx_map is not None:
            if mlp.gate_proj.g_idx_map is not mlp.up_proj.g_idx_map:
                return
        from .low_bit_linear import lowbit_row_concat
        mlp.gate_up_proj = lowbit_row_concat([mlp.gate_proj, mlp.up_proj], interleave_glu=True)
    elif type(mlp.gate_proj).__name__ == "KQuantLinear" or type(mlp.up_proj).__name__ == "KQuantLinear":
        from .low_bit_linear import kquant_row_concat
        mlp.gate_up_proj = kquant_row_concat([mlp.gate_proj, mlp.up_proj], interleave_glu=True)
    elif isinstance(mlp.gate_proj, nn.Linear) and isinstance(mlp.up_proj, nn.Linear):
        mlp.gate_up_proj = _merge_linears([mlp.gate_proj, mlp.up_proj], interleave_glu=True)
    else:
        return
    mlp._illm_interleaved = True
    del mlp.gate_proj, mlp.up_proj


def _phi3_split_qkv(attn):
    # phi3 ships qkv_proj already fused in [q; k; v] order: nothing to do
    return


def _optimize_pre(model: nn.Module, qtype: int):
    """Per-arch weight rewrites before quantization (reference convert.py:890-1089)."""
    mt = getattr(getattr(model, "config", None), "model_type", None)
    if mt == "rwkv":
        from ..models.rwkv import prescale_rwkv
        prescale_rwkv(model)
        return model
    from ..models.generic import GENERIC_ARCHS, generic_pre
    if mt in GENERIC_ARCHS:
        if generic_pre(model):
            model._illm_pre = True
        return model
    from ..models.mla import MLA_ARCHS
    if mt in MLA_ARCHS:
        model._illm_pre = True          # MLA: weights used as converted (kv_b absorbed at attach)
        return model
    from ..models.vl import VL_ARCHS, vl_pre
    if mt in VL_ARCHS:
        vl_pre(model)
        model._illm_pre = True
        return model
    if mt not in NATIVE_ARCHS and mt not in MOE_ARCHS:
        return model
    base = getattr(model, "model", None)
    layers = getattr(base, "layers", None)
    if layers is None:
        return model
    for layer in layers:
        attn = getattr(layer, "self_attn", None) or getattr(layer, "attention", None)
        if attn is not None and mt == "yuan":
            # LFA: q / k read the filtered stream, v the plain one -> [q; k] only
            if not hasattr(attn, "qk_proj") and isinstance(getattr(attn, "q_proj", None), nn.Linear):
                attn.qk_proj = _merge_linears([attn.q_proj, attn.k_proj])
                del attn.q_proj, attn.k_proj
        elif attn is not None:
            _merge_qkv(attn)
        mlp = getattr(layer, "mlp", None) or getattr(layer, "feed_forward", None)
        if mlp is not None and hasattr(mlp, "experts"):
            mlp = getattr(mlp, "shared_expert", None)     # MoE block: only the shared expert is dense
        if mlp is not None:
            I = getattr(getattr(mlp, "gate_proj", None), "out_features", None) or \
                (getattr(getattr(mlp, "gate_up_proj", None), "out_features", 0) // 2)
            if I and I % 16 == 0 and (isinstance(getattr(mlp, "gate_up_proj", getattr(mlp, "gate_proj", None)),
                                                 (nn.Linear, LowBitLinear)) or
                                      type(getattr(mlp, "gate_proj", None)).__name__ == "KQuantLinear"):
                _merge_gate_up(mlp)
    model._illm_pre = True
    return model


# ----------------------------------------------------------------- module swap
def _is_linear(m: nn.Module) -> bool:
    return isinstance(m, nn.Linear) and not isinstance(m, (LowBitLinear, DenseLinear))


def _is_expert_bank(m: nn.Module) -> bool:
    """HF fused experts (3-D gate_up_proj / down_proj parameters)"""
    gu, dn = getattr(m, "gate_up_proj", None), getattr(m, "down_proj", None)
    return isinstance(gu, nn.Parameter) and isinstance(dn, nn.Parameter) and gu.dim() == 3


def _convert_experts(m: nn.Module, qtype: int, device, convert_shape_only: bool):
    from ..models.moe import HFLowBitExperts, LowBitExperts
    if Q.is_dense(qtype) or Q.get_format(qtype) is None:
        return None
    E, I2, H = m.gate_up_proj.shape
    if H % Q.get_format(qtype).k_align or (I2 // 2) % Q.get_format(qtype).k_align or I2 % 32:
        return None
    if convert_shape_only or m.gate_up_proj.device.type == "meta":
        return HFLowBitExperts(LowBitExperts(E, I2, H, qtype, "meta"), LowBitExperts(E, H, I2 // 2, qtype, "meta"))
    return HFLowBitExperts.from_hf(m, qtype, device)


def _convert_one(module: nn.Linear, qtype: int, device, imatrix=None, mp_group=None, lm_head=False,
                 enable_scale_search=False, convert_shape_only=False):
    if Q.is_dense(qtype):
        dt = torch.bfloat16 if qtype == Q.BF16 else torch.float16
        return DenseLinear.from_linear(module, dt, device, mp_group)
    if qtype in (Q.TORCH_FP8E4, Q.TORCH_FP8E5):
        from .low_bit_linear import TorchFp8Linear
        if convert_shape_only or module.weight.device.type == "meta":
            return TorchFp8Linear(module.in_features, module.out_features, qtype, module.bias is not None,
                                  device="meta", mp_group=mp_group, optimize_lm_head=lm_head)
        return TorchFp8Linear.from_linear(module, qtype, device=device, mp_group=mp_group, optimize_lm_head=lm_head)
    fmt = Q.get_format(qtype)
    if fmt.kquant and module.in_features % fmt.k_align:
        # reference check_hidden_size: the nearest 64-block format instead
        qtype = Q.KQ_FALLBACK[fmt.qtype]
        fmt = Q.get_format(qtype)
    if module.in_features % fmt.k_align:
        return None
    if fmt.kquant:
        from .low_bit_linear import KQuantLinear
        if convert_shape_only or module.weight.device.type == "meta":
            return KQuantLinear(module.in_features, module.out_features, fmt.qtype, module.bias is not None,
                                device="meta", mp_group=mp_group, optimize_lm_head=lm_head)
        return KQuantLinear.from_linear(module, fmt.qtype, device=device, imatrix=imatrix, mp_group=mp_group,
                                        optimize_lm_head=lm_head)
    if convert_shape_only or module.weight.device.type == "meta":
        m = LowBitLinear(module.in_features, module.out_features, qtype, module.bias is not None,
                         device="meta", mp_group=mp_group, optimize_lm_head=lm_head)
        return m
    return LowBitLinear.from_linear(module, qtype, device=device, imatrix=imatrix, mp_group=mp_group,
                                    optimize_lm_head=lm_head, enable_scale_search=enable_scale_search)


_ROOT_CFG = [None]
_MIXED_PLAN = [None]      # {module name: qtype name} of a saved mixed_fp4 / mixed_fp8 model


def model_root_cfg():
    return _ROOT_CFG[0]


def _num_layers(cfg):
    return getattr(cfg, "num_hidden_layers", None) if cfg is not None else None


def _replace_with_low_bit_linear(model: nn.Module, qtype: int, modules_to_not_convert=None, prefix="",
                                 device=None, imatrix_data: Optional[Dict] = None, mixed_precision=False,
                                 convert_shape_only=False, enable_scale_search=False):
    """Recursively replace nn.Linear (reference convert.py:472-752)."""
    skip = set(modules_to_not_convert or [])
    n_conv = 0
    if isinstance(model, nn.MultiheadAttention):
        # torch MHA reads out_proj.weight directly (F.multi_head_attention_forward):
        # its projections stay dense (e.g. the Gemma-3 / SigLIP multimodal pooler)
        return 0
    for name, child in list(model.named_children()):
        full = f"{prefix}.{name}" if prefix else name
        if name in skip or full in skip:
            continue
        if _is_expert_bank(child):
            new = _convert_experts(child, qtype, device, convert_shape_only)
            if new is not None:
                setattr(model, name, new)
                n_conv += 1
            continue
        if _is_linear(child) and (name == "shared_expert_gate" or child.out_features < 16) and \
                not (name == "lm_head" or full.endswith("lm_head")):
            continue                                  # tiny gates stay dense
        if _is_linear(child):
            q = Q.mixed_kquant_qtype(qtype, full, _num_layers(model_root_cfg()))
            if q in (Q.MOFQ4, Q.MOFQ8):
                # per tensor; shape-only rebuilds (load_low_bit) follow the saved plan
                plan = _MIXED_PLAN[0] or {}
                if full in plan:
                    q = Q.resolve_qtype(plan[full])
                elif convert_shape_only or child.weight.device.type == "meta":
                    q = Q.SYM_INT4 if q == Q.MOFQ4 else Q.SYM_INT8
                else:
                    q = _pick_tensor_format(child.weight, q)
            is_head = name == "lm_head" or full.endswith("lm_head")
            if is_head and mixed_precision and qtype in (Q.SYM_INT4, Q.ASYM_INT4, Q.WOQ_INT4, Q.NF4, Q.FP4):
                q = Q.SYM_INT8
            im = imatrix_data.get(full) if imatrix_data else None
            new = _convert_one(child, q, device, im, getattr(child, "mp_group", None), is_head,
                               enable_scale_search, convert_shape_only)
            if new is not None:
                setattr(model, name, new)
                n_conv += 1
                del child
        else:
            n_conv += _replace_with_low_bit_linear(child, qtype, modules_to_not_convert, full, device, imatrix_data,
                                                   mixed_precision, convert_shape_only, enable_scale_search)
    return n_conv


# ----------------------------------------------------------------- post
class _RMSNormFn(torch.autograd.Function):
    """HIP RMSNorm forward + HIP backward for x (frozen weight, the QLoRA
    case): one kernel each way instead of the ~6 f32 cast / pow / mean /
    rsqrt / mul kernels per direction of the HF module (reference
    xe_addons.rms_norm, SRC/transformers/models/common.py:184-200)"""

    @staticmethod
    def forward(ctx, x, w, eps):
        from .. import ops
        ctx.save_for_backward(x, w)
        ctx.eps = eps
        return ops.rms_norm(x, w, eps)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        return torch.ops.ipex_llm_amd.rms_norm_bwd(x, g.contiguous(), w, ctx.eps, False), None, None


def _rmsnorm_forward(self, hidden_states):
    from .. import ops
    w = self.weight
    eps = getattr(self, "variance_epsilon", None) or getattr(self, "eps", 1e-6)
    if hidden_states.is_cuda and hidden_states.dtype == w.dtype and hidden_states.shape[-1] % 8 == 0:
        if torch.is_grad_enabled() and (hidden_states.requires_grad or w.requires_grad):
            if not w.requires_grad and ops.native_gpu(hidden_states):
                return _RMSNormFn.apply(hidden_states.contiguous(), w, eps)
            from ..ops import reference as R
            return R.rms_norm(hidden_states, w, eps)          # differentiable torch graph
        return ops.rms_norm(hidden_states.contiguous(), w, eps)
    from ..ops import reference as R
    return R.rms_norm(hidden_states, w.to(hidden_states.dtype), eps)


def _ds_router_forward(self, hidden_states):
    """DeepSeek-V3 router on the group-limited top-k kernel (reference
    deepseek.py:274-290 -> xe_addons.moe_group_topk)."""
    from .. import ops
    import torch.nn.functional as F
    h = hidden_states.view(-1, self.hidden_dim)
    logits = F.linear(h.float(), self.weight.float())
    w, idx = ops.moe_group_topk(logits, self.e_score_correction_bias, self.top_k, self.num_group, self.topk_group,
                                bool(self.norm_topk_prob), float(self.routed_scaling_factor))
    return logits, w, idx.long()


def _patch_routers(model: nn.Module):
    for m in model.modules():
        if m.__class__.__name__.endswith("TopkRouter") and all(
                hasattr(m, a) for a in ("num_group", "topk_group", "e_score_correction_bias", "routed_scaling_factor")):
            m.forward = types.MethodType(_ds_router_forward, m)


class _RopeHalfFn(torch.autograd.Function):
    """rotate-half RoPE of the HF forward as one HIP kernel each way (the
    transposed rotation for the gradient) instead of mul / slice / neg / cat
    / mul / add per tensor and direction"""

    @staticmethod
    def forward(ctx, x, cos, sin):
        ctx.save_for_backward(cos, sin)
        return torch.ops.ipex_llm_amd.rope_half(x, cos, sin, False)

    @staticmethod
    def backward(ctx, g):
        cos, sin = ctx.saved_tensors
        return torch.ops.ipex_llm_amd.rope_half(g, cos, sin, True), None, None


_ROPE_ORIG = {}


def _rope_fusable(q, cos, unsqueeze_dim):
    from .. import ops
    return (isinstance(unsqueeze_dim, int) and unsqueeze_dim == 1 and q.dim() == 4 and cos.dim() == 3 and q.is_cuda and ops.native_gpu(q)
            and q.stride(-1) == 1 and q.shape[-1] % 8 == 0 and cos.shape[-1] == q.shape[-1]
            and cos.shape[1] == q.shape[2] and cos.dtype == q.dtype and q.dtype in (torch.bfloat16, torch.float16)
            and cos.shape[0] in (1, q.shape[0]) and all(st % 4 == 0 for st in q.stride()[:3]))


def _make_rope(orig):
    def apply_rotary_pos_emb(q, k, cos, sin, unsqueeze_dim=1, **kw):
        if not kw and _rope_fusable(q, cos, unsqueeze_dim) and _rope_fusable(k, cos, unsqueeze_dim):
            cos, sin = cos.contiguous(), sin.contiguous()
            return _RopeHalfFn.apply(q, cos, sin), _RopeHalfFn.apply(k, cos, sin)
        return orig(q, k, cos, sin, unsqueeze_dim, **kw)
    apply_rotary_pos_emb.__wrapped__ = orig
    return apply_rotary_pos_emb


def _patch_rope(model: nn.Module):
    """the HF modeling module's ``apply_rotary_pos_emb`` (rotate-half form:
    llama / mistral / qwen2 / qwen3 ...) -> the HIP kernel on GPU tensors,
    the original elsewhere (model-module global, as the reference's
    per-arch forward patches)"""
    import sys
    mods = {type(m).__module__ for m in model.modules() if type(m).__name__.endswith("Attention")}
    for name in mods:
        mod = sys.modules.get(name)
        f = getattr(mod, "apply_rotary_pos_emb", None)
        if f is None or getattr(f, "__wrapped__", None) is not None or name in _ROPE_ORIG:
            continue
        rh = getattr(mod, "rotate_half", None)
        if rh is None:
            continue
        try:                            # interleaved forms (GLM, ...) keep their own function
            t = torch.arange(8.0)
            if not torch.equal(rh(t), torch.cat([-t[4:], t[:4]])):
                continue
        except Exception:
            continue
        _ROPE_ORIG[name] = f
        mod.apply_rotary_pos_emb = _make_rope(f)


class _ActMulFn(torch.autograd.Function):
    """act(gate) * up of the HF MLP as one HIP kernel each way (HF rounding)"""

    @staticmethod
    def forward(ctx, g, u, act):
        ctx.save_for_backward(g, u)
        ctx.act = act
        return torch.ops.ipex_llm_amd.act_mul(g, u, None, act)[0]

    @staticmethod
    def backward(ctx, dy):
        g, u = ctx.saved_tensors
        dg, du = torch.ops.ipex_llm_amd.act_mul(g, u, dy.contiguous(), ctx.act)
        return dg, du, None


def _mlp_act_code(act_fn):
    name = type(act_fn).__name__
    if isinstance(act_fn, nn.SiLU) or name == "SiLUActivation":
        return 0
    if name in ("GELUTanh", "PytorchGELUTanh", "NewGELUActivation", "GELUPytorchTanh"):
        return 1
    return None


def _mlp_forward(self, x):
    from .. import ops
    g = self.gate_proj(x)
    u = self.up_proj(x)
    if (g.is_cuda and ops.native_gpu(g) and g.dtype in (torch.bfloat16, torch.float16) and g.dtype == u.dtype
            and g.shape == u.shape and g.numel() % 8 == 0):
        h = _ActMulFn.apply(g.contiguous(), u.contiguous(), self._illm_act)
    else:
        h = self.act_fn(g) * u
    return self.down_proj(h)


def _patch_mlp(model: nn.Module):
    """gated MLPs (gate_proj / up_proj / down_proj, silu or gelu-tanh) of
    the HF forward -> the fused act * up kernel and its gradient"""
    for m in model.modules():
        if not type(m).__name__.endswith("MLP") or getattr(m, "_illm_act", None) is not None:
            continue
        if not all(hasattr(m, a) for a in ("gate_proj", "up_proj", "down_proj", "act_fn")):
            continue
        code = _mlp_act_code(m.act_fn)
        if code is None:
            continue
        m._illm_act = code
        m.forward = types.MethodType(_mlp_forward, m)


def _patch_norms(model: nn.Module):
    for m in model.modules():
        cls = m.__class__.__name__
        if cls.endswith("RMSNorm") and hasattr(m, "weight") and "Gemma" not in cls:
            m.forward = types.MethodType(_rmsnorm_forward, m)


def _optimize_post(model: nn.Module):
    """Swap in the native MI355X decoder for supported architectures."""
    mt = getattr(getattr(model, "config", None), "model_type", None)
    _patch_norms(model)
    _patch_rope(model)
    _patch_mlp(model)
    _patch_routers(model)
    from .attention import patch_eager_attention
    patch_eager_attention(model)
    if mt in ENCODER_FLASH_ARCHS and getattr(model.config, "_attn_implementation", None) in (None, "sdpa"):
        # bidirectional encoder self-attention on the HIP flash kernel
        # (training/flash_attn.py; padded batches / cross-attention keep SDPA)
        from ..training.flash_attn import patch_flash_attention
        patch_flash_attention(model)
    if mt == "rwkv":
        from ..models.rwkv import patch_rwkv
        patch_rwkv()
    if mt == "rwkv5":
        from ..models.rwkv import patch_rwkv5
        patch_rwkv5(model)
    from ..models.generic import GENERIC_ARCHS
    from ..models.mla import MLA_ARCHS
    from ..models.vl import VL_ARCHS, attach_vl
    if mt in VL_ARCHS and getattr(model, "_illm_pre", False):
        return attach_vl(model)
    if (mt in NATIVE_ARCHS or mt in MOE_ARCHS or mt in GENERIC_ARCHS or mt in MLA_ARCHS) and \
            getattr(model, "_illm_pre", False):
        from .hf_native import attach_native
        attach_native(model)
        if not getattr(model, "_illm_native_attached", False):
            # variant the native decoder cannot run: HF forward over the merged weights
            if mt in GENERIC_ARCHS:
                from ..models.generic import restore_generic_views
                restore_generic_views(model)
            elif mt not in MLA_ARCHS:
                from .hf_views import restore_hf_views
                restore_hf_views(model)
    return model


# ----------------------------------------------------------------- entry
def ggml_convert_low_bit(model: nn.Module, qtype="sym_int4", optimize_model: bool = True, device=None,
                         modules_to_not_convert=None, convert_shape_only: bool = False,
                         imatrix_data=None, embedding_qtype=None, mixed_precision: bool = False,
                         cpu_embedding: bool = False, disk_embedding: bool = False,
                         enable_scale_search: bool = False, torch_dtype=None):
    """Quantize ``model`` in place and install optimized forwards."""
    qtype = Q.resolve_qtype(qtype)
    if qtype in (Q.SYM_INT4, Q.WOQ_INT4):
        qtype = Q.SYM_INT4 if qtype == Q.SYM_INT4 else Q.WOQ_INT4
    modules_to_not_convert = list(modules_to_not_convert or [])
    if optimize_model:
        _optimize_pre(model, qtype)
    _ROOT_CFG[0] = getattr(model, "config", None)     # layer count for the gguf_q4k_s/m policies
    try:
        n = _replace_with_low_bit_linear(model, qtype, modules_to_not_convert, "", device, imatrix_data,
                                         mixed_precision, convert_shape_only, enable_scale_search)
    finally:
        _ROOT_CFG[0] = None
    if n == 0:
        logger.warning("ggml_convert_low_bit: no linear layer converted")
    if embedding_qtype is not None or cpu_embedding or disk_embedding:
        from .embedding import replace_embeddings
        replace_embeddings(model, embedding_qtype, cpu_embedding, disk_embedding)
    if torch_dtype is not None and torch_dtype != "auto" and not convert_shape_only:
        _cast_non_linear(model, torch_dtype)
    if optimize_model:
        _optimize_post(model)
    model._illm_qtype = qtype
    if hasattr(model, "config"):
        model.config.bigdl_transformers_low_bit = Q.qtype_name(qtype)
    return model


def _cast_non_linear(model, dtype):
    for m in model.modules():
        if isinstance(m, (LowBitLinear,)):
            continue
        for pn, p in list(m.named_parameters(recurse=False)):
            if p.is_floating_point() and p.dtype != dtype:
                p.data = p.data.to(dtype)


def _pick_tensor_format(w: torch.Tensor, qtype):
    """mixed_fp4 / mixed_fp8: the lower-MSE of (sym_int4, fp4) or (sym_int8,
    fp8_e4m3) for THIS tensor (reference low_bit_linear.py:370-408,
    FP4Params.quantize)"""
    from .. import ops
    cands = (Q.SYM_INT4, Q.FP4) if qtype == Q.MOFQ4 else (Q.SYM_INT8, Q.FP8E4)
    wf = w.detach().float().cpu()
    if wf.dim() != 2 or wf.shape[1] % 64:
        return cands[0]
    best, best_err = cands[0], None
    for c in cands:
        f = Q.get_format(c).fmt
        err = (ops.dequantize(ops.quantize(wf, f), f, wf.shape[0], wf.shape[1]) - wf).pow(2).mean().item()
        if best_err is None or err < best_err:
            best, best_err = c, err
    return best
