"""LoRA / QLoRA / QA-LoRA on low-bit base weights (a self-contained,
peft-compatible API; ``peft`` is not a dependency).

Reference: ``SRC/transformers/qlora.py`` -- ``LoraLowBitLinear`` (66-143:
frozen low-bit base + LoRA A/B, QA-LoRA average-pools the input by the
quantization group size), ``LoraBF16Linear`` (146-211), ``get_peft_model``
(282-301), ``prepare_model_for_kbit_training`` (304-352), ``LoraConfig``
with ``training_mode`` (254-267), ``cast_lora_weight`` (377-391).

MI355X design: the base ``LowBitLinear`` runs the low-bit GEMM forward
(decode-class GEMV for small M, dequant+GEMM for training batches) and its
backward through ``MatMulLowBit`` (grad_x = grad_y @ dequant(W), no weight
gradient); the adapters are plain bf16 parameters updated by the fused
multi-tensor AdamW kernel (``training/optim.py``).  Checkpoints are
``adapter_model.safetensors`` + ``adapter_config.json`` (peft's file names,
so adapters interoperate).
"""
from __future__ import annotations

import contextlib
import json
import math
import os
import re
import weakref
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional, Union

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..quantize import qtypes as Q
from ..transformers.low_bit_linear import DenseLinear, LowBitLinear

TRAINING_MODES = ("qlora", "lora", "qalora", "relora")


@dataclass
class LoraConfig:
    r: int = 8
    lora_alpha: int = 16
    lora_dropout: float = 0.0
    target_modules: Optional[Union[List[str], str]] = None
    bias: str = "none"
    task_type: Optional[str] = "CAUSAL_LM"
    training_mode: str = "qlora"
    use_rslora: bool = False
    modules_to_save: Optional[List[str]] = None
    init_lora_weights: bool = True
    peft_type: str = "LORA"

    def __post_init__(self):
        if self.training_mode not in TRAINING_MODES:
            raise ValueError(f"training_mode must be one of {TRAINING_MODES}")

    @property
    def scaling(self) -> float:
        return self.lora_alpha / (math.sqrt(self.r) if self.use_rslora else self.r)

    def to_dict(self):
        return asdict(self)

    def save_pretrained(self, path):
        os.makedirs(path, exist_ok=True)
        with open(os.path.join(path, "adapter_config.json"), "w") as f:
            json.dump(self.to_dict(), f, indent=2)

    @classmethod
    def from_pretrained(cls, path):
        with open(os.path.join(path, "adapter_config.json")) as f:
            d = json.load(f)
        keys = cls.__dataclass_fields__.keys()
        return cls(**{k: v for k, v in d.items() if k in keys})


DEFAULT_TARGETS = ["q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj",
                   "qkv_proj", "gate_up_proj", "query_key_value", "dense", "W_pack"]


_FUSED = os.environ.get("ILLM_LORA_FUSED", "1") == "1"
# sibling adapters over one input (q/k/v, gate/up) as one autograd node
_GROUP = os.environ.get("ILLM_LORA_GROUP", "1") == "1"
_GROUPS = (("q_proj", "k_proj", "v_proj"), ("gate_proj", "up_proj"))


def _rank_update_(C: torch.Tensor, A: torch.Tensor, B: torch.Tensor, alpha: float = 1.0) -> torch.Tensor:
    """C += alpha * A @ B^T in place (A [M, r], B [N, r]): the LoRA rank-r term
    on the HIP rank-update kernel (csrc/hip/lora_update.hip: a read-modify-
    write of C at memory speed) where it applies, the library addmm otherwise"""
    from .. import ops
    r = A.shape[1]
    if (_RANK_KERNEL and C.is_cuda and ops.native_gpu(C) and C.dtype in (torch.bfloat16, torch.float16)
            and A.dtype == C.dtype and B.dtype == C.dtype and r % 8 == 0 and r <= 64 and C.shape[1] % 8 == 0
            and C.stride(1) == 1 and C.stride(0) % 8 == 0 and C.data_ptr() % 16 == 0 and A.stride(1) == 1
            and A.stride(0) % 8 == 0 and A.data_ptr() % 16 == 0):
        if B.stride(1) != 1 or B.stride(0) % 8 or B.data_ptr() % 16:
            B = B.contiguous()
        return torch.ops.ipex_llm_amd.lora_update_(C, A, B, float(alpha))
    return C.addmm_(A, B.t(), alpha=alpha)


# ILLM_LORA_RANK_KERNEL=0: the LoRA adds on the library addmm (A/B)
_RANK_KERNEL = os.environ.get("ILLM_LORA_RANK_KERNEL", "1") == "1"


def _tn_ok(a: torch.Tensor, b: torch.Tensor) -> bool:
    from .. import ops
    r, N = a.shape[1], b.shape[1]
    return (_TN_KERNEL and a.is_cuda and ops.native_gpu(a) and a.dtype in (torch.bfloat16, torch.float16)
            and b.dtype == a.dtype and r % 8 == 0 and r <= 64 and N % 8 == 0
            and all(t.stride(1) == 1 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0 for t in (a, b)))


def _tn_many(jobs, dtype):
    """[(a, b, alpha, trans)] -> [alpha a^T b] ([r, N], or [N, r] with trans)
    in ``dtype``.  On the HIP reduction all of one node's weight gradients
    accumulate into ONE zeroed f32 slab (the B gradients written transposed
    by the kernel) and leave through ONE cast: one fill + one cast launch per
    autograd node instead of a fill, a cast and a transpose copy per gradient"""
    if not jobs:
        return []
    if all(_tn_ok(a, b) for a, b, _, _ in jobs):
        shapes = [((b.shape[1], a.shape[1]) if tr else (a.shape[1], b.shape[1])) for a, b, _, tr in jobs]
        slab = torch.zeros(sum(x * y for x, y in shapes), dtype=torch.float32, device=jobs[0][0].device)
        outs, off = [], 0
        for (a, b, alpha, tr), (x, y) in zip(jobs, shapes):
            v = slab[off:off + x * y].view(x, y)
            torch.ops.ipex_llm_amd.lora_tn_acc_(v, a, b, float(alpha), tr)
            outs.append((off, x, y))
            off += x * y
        cast = slab.to(dtype)
        return [cast[o:o + x * y].view(x, y) for o, x, y in outs]
    return [(_tn(a, b, alpha).t().contiguous() if tr else _tn(a, b, alpha)) for a, b, alpha, tr in jobs]


def _tn(a: torch.Tensor, b: torch.Tensor, alpha: float = 1.0) -> torch.Tensor:
    """alpha * a^T b over the token axis (a [M, r], b [M, N]) -> [r, N] in
    a's dtype: the LoRA weight gradients.  On the HIP token-axis reduction
    (csrc/hip/lora_update.hip lora_tn: both operands through transposed LDS
    reads, f32 atomics over row slices) where it applies -- the library
    runs these K = tokens, M = r shapes on a 256 x 128 macro-tile at a
    fraction of HBM speed -- the library GEMM otherwise"""
    if _tn_ok(a, b):
        return torch.ops.ipex_llm_amd.lora_tn(a, b, float(alpha)).to(a.dtype)
    if alpha == 1.0:
        return torch.mm(a.t(), b)
    return torch.addmm(a.new_empty(()), a.t(), b, beta=0, alpha=alpha)


# ILLM_LORA_GXA_SLICES=0: grouped s g B as separate outputs + concatenation (A/B)
_GXA_SLICES = os.environ.get("ILLM_LORA_GXA_SLICES", "1") == "1"
# ILLM_LORA_TN_KERNEL=0: dA / dB on the library GEMM (A/B)
_TN_KERNEL = os.environ.get("ILLM_LORA_TN_KERNEL", "1") == "1"


def _skinny(x2: torch.Tensor, W: torch.Tensor, alpha: float = 1.0) -> torch.Tensor:
    """alpha * x2 @ W^T for a rank-r factor W [r, K] (x2 [M, K] -> [M, r]):
    the LoRA down-projections x A^T and g B.  On the streaming skinny GEMM
    (csrc/hip/dense_gemv.hip, <= 16 rows per launch) with the roles swapped
    -- the r factor rows are the "activations", the M token rows the
    "weight" streamed once -- instead of a library GEMM on a 16 x 16 macro
    tile; the library GEMM elsewhere"""
    from .. import ops
    r, K = W.shape
    # the factor is pre-scaled in its 16-bit dtype: exact only for a power-of-two
    # alpha (alpha / r = 16 / 8 ...); any other scale (16 / 12, rsLoRA) keeps the
    # library GEMM, which applies alpha to the f32 sums
    if (_SKINNY and x2.is_cuda and ops.native_gpu(x2) and x2.dtype in (torch.bfloat16, torch.float16)
            and W.dtype == x2.dtype and x2.is_contiguous() and K % 64 == 0 and r <= 64
            and x2.shape[0] >= 64 and _pow2(alpha)):
        Wc = (W * alpha if alpha != 1.0 else W).contiguous()
        dlt = torch.ops.ipex_llm_amd.dense_linear_t            # [tokens, rows] straight from the kernel
        if r <= 16:
            return dlt(Wc, x2)
        return torch.cat([dlt(Wc[c0:c0 + 16].contiguous(), x2) for c0 in range(0, r, 16)], 1)
    if alpha == 1.0:
        return torch.mm(x2, W.t())
    return torch.addmm(x2.new_empty(()), x2, W.t(), beta=0, alpha=alpha)


def _pow2(a: float) -> bool:
    """a is +-2^e (multiplying by it is exact in any float format, barring range)"""
    m, _ = math.frexp(abs(float(a)))
    return a != 0 and m == 0.5


# ILLM_LORA_SKINNY=0: the rank-r down-projections on the library GEMM (A/B)
_SKINNY = os.environ.get("ILLM_LORA_SKINNY", "1") == "1"


def _g8_bwd_ok(g2: torch.Tensor, base) -> bool:
    """grad_x = g W on the dense 8-phase GEMM over W^T dequantized straight
    from the blob (no resident shadow budget: the shadow paths below own it)"""
    from .. import ops
    from ..ops.gemm import _DENSE_BUDGET, use_g8d
    N = base.out_features
    return (_DENSE_BUDGET <= 0 and base.weight.is_cuda and ops.native_gpu(base.weight)
            and getattr(base, "g_idx_map", None) is None and N % 64 == 0
            and use_g8d(g2, g2.shape[0], base.in_features, N))


def _g8_grad_x(g2: torch.Tensor, base, acc: Optional[torch.Tensor] = None) -> torch.Tensor:
    """g W (+ acc: sibling adapters' grad_x) over a transient dequantized W,
    whichever form the shape measured faster (ops/gemm.py _pick, the
    dequantization included): the 8-phase kernel over W^T dequantized
    transposed (acc added in its epilogue), the library GEMM over W as stored
    (no transposed dequant, whose 32-B row pieces make it the slower one), or
    the library over the transposed dequant"""
    from ..ops.gemm import _pick
    ops = torch.ops.ipex_llm_amd
    N, K = base.out_features, base.in_features

    def wt():
        return ops.dequantize_device(base.weight, base.fmt, N, K, g2.dtype, True)      # W^T [K, N]

    def w():
        return ops.dequantize_device(base.weight, base.fmt, N, K, g2.dtype, False)     # W [N, K]
    key = (g2.shape[0], K, N, "grad_x", 0)
    c = _pick(key, lambda: ops.gemm_bf16(g2, wt()), lambda: torch.mm(g2, w()), lambda: torch.mm(g2, wt().t()))
    if c == "lib":
        return torch.mm(g2, w()) if acc is None else acc.addmm_(g2, w())
    if c == "lib1":          # the library over the transposed dequant (its other operand layout)
        return torch.mm(g2, wt().t()) if acc is None else acc.addmm_(g2, wt().t())
    if acc is None:
        return ops.gemm_bf16(g2, wt())
    return ops.gemm_bf16(g2, wt(), None, False, 0, False, 0, -1, acc, True)


def _base_dense_weight(base, dt):
    """the frozen base weight as the backward GEMM operand: the resident dense
    shadow / a transient dequant on the GPU (as MatMulLowBit), dequant on CPU"""
    from .. import ops
    if base.weight.is_cuda and ops.native_gpu(base.weight):
        from ..ops.gemm import _dense_weight
        return _dense_weight(base.weight, base.fmt, base.out_features, base.in_features, dt)
    return ops.dequantize(base.weight, base.fmt, base.out_features, base.in_features, dtype=dt)


class _LoraLowBitFn(torch.autograd.Function):
    """y = x W^T (+ bias) + s (x A^T) B^T over a frozen low-bit W as one
    autograd node.  The LoRA term accumulates into the base GEMM's output
    (addmm, beta = 1, alpha = s) and, backward, into grad_x = g W + (s g B) A
    (one accumulating rank-r GEMM): the scale, the two adds over [M, N] /
    [M, K] and the cast that the module-by-module graph launches per adapter
    disappear (reference LoraLowBitLinear.forward, SRC/transformers/qlora.py:114-143)."""

    @staticmethod
    def forward(ctx, x, A, B, base, s):
        from .. import ops
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        bias = base.bias
        if bias is not None and bias.dtype != x2.dtype:
            bias = bias.to(x2.dtype)
        with torch.no_grad():
            y = ops.lowbit_matmul(x2, base.weight, base.fmt, base.out_features, base.in_features, bias)
            xa = _skinny(x2, A)
            _rank_update_(y, xa, B, s)
        ctx.save_for_backward(x2, xa, A, B)
        ctx.base, ctx.s, ctx.shp = base, s, shp
        return y.view(*shp[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, g):
        x2, xa, A, B = ctx.saved_tensors
        g2 = g.reshape(-1, g.shape[-1]).to(x2.dtype)
        s = ctx.s
        # the LoRA scale rides on the GEMMs' alpha (beta = 0: the 1-element
        # input is never read) instead of separate [M, r] / [N, r] scale launches
        gxa = _skinny(g2, B.t(), s)                       # s g B [M, r]
        jobs = ([(gxa, x2, 1.0, False)] if ctx.needs_input_grad[1] else []) + \
            ([(xa, g2, s, True)] if ctx.needs_input_grad[2] else [])
        res = _tn_many(jobs, A.dtype)
        gA = res.pop(0) if ctx.needs_input_grad[1] else None
        gB = res.pop(0) if ctx.needs_input_grad[2] else None
        gx = None
        if ctx.needs_input_grad[0]:
            base = ctx.base
            if _g8_bwd_ok(g2, base):
                gx = _g8_grad_x(g2, base)
            elif _kcat_rows_ok(base, g2, A):
                # gx = [g | s g B] [W ; A]: the adapter term as r extra K rows of
                # the grad_x GEMM (row-augmented shadow) instead of a rank-update
                # pass over the [M, K] output (the 14336-wide down projection)
                N, r = base.out_features, A.shape[0]
                Rp = -(-(N + r) // _KCAT_PAD) * _KCAT_PAD - N
                w = _aug_rows_weight(base, Rp, x2.dtype, A)
                parts = [g2, gxa] + ([g2.new_zeros(g2.shape[0], Rp - r)] if Rp > r else [])
                gx = torch.mm(torch.cat(parts, 1), w).view(ctx.shp)
                return gx, gA, gB, None, None
            else:
                w = _base_dense_weight(base, x2.dtype)
                gx = torch.mm(g2, w)
            _rank_update_(gx, gxa, A.t())
            gx = gx.view(ctx.shp)
        return gx, gA, gB, None, None


# K-concatenated LoRA for wide siblings (gate / up): y_i = [x | s x A_all^T]
# [W_i | B_i-block]^T -- the adapter rides as R extra K columns of the base
# GEMM (R = sum of ranks, <= 0.6 % more MACs) on a resident augmented shadow
# [N, K + R] whose tail holds B_i in its sibling's column block, instead of a
# rank-update pass that reads and writes the [M, N] output (235 MB per
# 14336-wide projection at 4096 tokens).  The backward's g W reads the same
# shadow through a [:, :K] view.  ILLM_LORA_KCAT=auto (default: siblings with
# N >= 2 K, dense shadow budget > 0) / 1 (every group) / 0 (off).  Same-box
# A/B on MI355X, Llama-3-8B QLoRA (profiles/qlora_ab_*kcat*_r4.json): 137.7 vs
# 140.1 ms/step for the rank-update pass with the extended K padded to 4160;
# unpadded (K = 4112) it was slower, 142.3 vs 139.9.
_KCAT = os.environ.get("ILLM_LORA_KCAT", "auto")
_KCAT_PAD = int(os.environ.get("ILLM_LORA_KCAT_PAD", "64"))
_KCAT_ROWS = os.environ.get("ILLM_LORA_KCAT_ROWS", "1") == "1"   # the down projection's grad_x form
from ..ops.gemm import ChargedCache as _ChargedCache  # noqa: E402

# (blob ptr, version, R, off, dtype) -> (weakref to blob, [N, K + R] shadow, bytes): charged to the
# same resident-shadow budget as ops/gemm.py's prefill shadows (ILLM_TRAIN_DENSE_GB / ILLM_PREFILL_DENSE_GB)
_aug_cache = _ChargedCache()


def _aug_fits(key, nbytes: int) -> bool:
    from ..ops.gemm import dense_fits
    return key in _aug_cache or dense_fits(nbytes)


def _kcat_ok(bases, x2, As) -> bool:
    from .. import ops
    from ..ops.gemm import _DENSE_BUDGET
    if _KCAT == "0" or not (x2.is_cuda and ops.native_gpu(x2) and _DENSE_BUDGET > 0):
        return False
    if x2.dtype not in (torch.bfloat16, torch.float16) or x2.shape[0] <= ops.GEMV_MAX_M:
        return False
    K, R = x2.shape[1], sum(A.shape[0] for A in As)
    if (K + R) % 8 or any(b.in_features != K for b in bases):
        return False
    if not (_KCAT == "1" or min(b.out_features for b in bases) >= 2 * K):
        return False
    # every augmented shadow is resident or still fits the budget (else the rank-update path)
    need, off = 0, 0
    for b, A in zip(bases, As):
        key = (b.weight.data_ptr(), b.weight._version, R, off, x2.dtype)
        if key not in _aug_cache:
            need += b.out_features * (K + R) * x2.element_size()
        off += A.shape[0]
    from ..ops.gemm import dense_fits
    return need == 0 or dense_fits(need)


def _aug_weight(base, R: int, off: int, dtype, B=None):
    """the augmented shadow of ``base`` ([N, K + R], made on first use from the
    dequantized blob); ``B`` ([N, r], the adapter's current value) is written
    into columns K + off .. K + off + r"""
    blob = base.weight
    key = (blob.data_ptr(), blob._version, R, off, dtype)
    ent = _aug_cache.get(key)
    if ent is None or ent[0]() is not blob:
        N, K = base.out_features, base.in_features
        w = torch.zeros(N, K + R, dtype=dtype, device=blob.device)
        w[:, :K].copy_(torch.ops.ipex_llm_amd.dequantize_device(blob, base.fmt, N, K, dtype))
        _aug_cache.put(key, blob, w, w.numel() * w.element_size())
        ent = _aug_cache[key]
    w = ent[1]
    if B is not None:
        K = base.in_features
        w[:, K + off:K + off + B.shape[1]].copy_(B)
    return w


def _kcat_rows_ok(base, g2, A) -> bool:
    """row-augmented grad_x for a single adapter whose input is much wider
    than its output (down projection: K >= 2 N), same switches as _kcat_ok"""
    from .. import ops
    from ..ops.gemm import _DENSE_BUDGET
    if _KCAT == "0" or not _KCAT_ROWS or not (g2.is_cuda and ops.native_gpu(g2) and _DENSE_BUDGET > 0):
        return False
    if g2.dtype not in (torch.bfloat16, torch.float16) or g2.shape[0] <= ops.GEMV_MAX_M or A.dtype != g2.dtype:
        return False
    if not (_KCAT == "1" or base.in_features >= 2 * base.out_features):
        return False
    N, K = base.out_features, base.in_features
    Rp = -(-(N + A.shape[0]) // _KCAT_PAD) * _KCAT_PAD - N        # as in _LoraLowBitFn.backward
    key = ("rows", base.weight.data_ptr(), base.weight._version, Rp, g2.dtype)
    # the W rows are shared with the prefill / forward shadow (below): only the
    # adapter rows are new when that shadow is already resident
    from ..ops.gemm import _dense_cache
    dkey = (base.weight.data_ptr(), base.weight._version, N, K, g2.dtype)
    need = (N + Rp) * K * g2.element_size() - (_dense_cache[dkey][2] if dkey in _dense_cache else 0)
    return _aug_fits(key, need)


def _aug_rows_weight(base, Rp: int, dtype, A=None):
    """[N + Rp, K] shadow of ``base``: W on top, ``A`` ([r, K], current value)
    written into rows N .. N + r, zeros below"""
    blob = base.weight
    key = ("rows", blob.data_ptr(), blob._version, Rp, dtype)
    ent = _aug_cache.get(key)
    if ent is None or ent[0]() is not blob:
        from ..ops.gemm import _dense_cache
        N, K = base.out_features, base.in_features
        w = torch.zeros(N + Rp, K, dtype=dtype, device=blob.device)
        w[:N].copy_(torch.ops.ipex_llm_amd.dequantize_device(blob, base.fmt, N, K, dtype))
        # one copy of W: the forward's shadow (lowbit_matmul -> _dense_weight) becomes a
        # view of these rows; its bytes move into this entry
        dkey = (blob.data_ptr(), blob._version, N, K, dtype)
        _dense_cache.pop(dkey)
        _aug_cache.put(key, blob, w, w.numel() * w.element_size())
        _dense_cache.put(dkey, blob, w[:N], 0)
        _aug_cache.link(key, _dense_cache, dkey)      # the 0-charged view leaves with its storage
        ent = _aug_cache[key]
    w = ent[1]
    if A is not None:
        N = base.out_features
        w[N:N + A.shape[0]].copy_(A)
    return w


class _LoraGroupFn(torch.autograd.Function):
    """q / k / v (or gate / up) adapters over ONE shared input as one
    autograd node: x A_all^T for all siblings in one pass over x (A_all =
    [A_q; A_k; A_v]), each base GEMM + its rank-r add as in _LoraLowBitFn;
    backward reads x once more for every dA (gxa_all^T x), accumulates
    grad_x = sum_i g_i W_i + gxa_all A_all into one buffer (beta = 1 GEMMs)
    instead of per-sibling outputs summed by autograd.  Same math as the
    per-module path, fewer passes over the [tokens, hidden] activations."""

    @staticmethod
    def forward(ctx, x, s, bases, *AB):
        from .. import ops
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        As, Bs = AB[0::2], AB[1::2]
        kcat = _kcat_ok(bases, x2, As)
        with torch.no_grad():
            if kcat:
                K, R = x2.shape[1], sum(A.shape[0] for A in As)
                xa_all = torch.addmm(x2.new_empty(()), x2, torch.cat(As, 0).t(), beta=0, alpha=s)   # s x A^T
                # the extended K padded to a multiple of _KCAT_PAD (zero columns):
                # the library GEMM at K = 4112 picked a slow tile
                Rp = -(-(K + R) // _KCAT_PAD) * _KCAT_PAD - K
                parts = [x2, xa_all] + ([x2.new_zeros(x2.shape[0], Rp - R)] if Rp > R else [])
                x_ext = torch.cat(parts, 1)
                R = Rp
                ys, off = [], 0
                for base, A, B in zip(bases, As, Bs):
                    w = _aug_weight(base, R, off, x2.dtype, B)
                    y = torch.mm(x_ext, w.t())
                    if base.bias is not None:
                        y.add_(base.bias.to(y.dtype))
                    ys.append(y.view(*shp[:-1], y.shape[-1]))
                    off += A.shape[0]
                del x_ext
                ctx.save_for_backward(x2, xa_all, *AB)
                ctx.s, ctx.shp, ctx.bases, ctx.kcat = s, shp, bases, (R, x2.dtype)
                return tuple(ys)
            xa_all = _skinny(x2, torch.cat(As, 0))              # [M, sum r]
            ys, off = [], 0
            for base, A, B in zip(bases, As, Bs):
                r = A.shape[0]
                bias = base.bias
                if bias is not None and bias.dtype != x2.dtype:
                    bias = bias.to(x2.dtype)
                y = ops.lowbit_matmul(x2, base.weight, base.fmt, base.out_features, base.in_features, bias)
                _rank_update_(y, xa_all[:, off:off + r], B, s)
                ys.append(y.view(*shp[:-1], y.shape[-1]))
                off += r
        ctx.save_for_backward(x2, xa_all, *AB)
        ctx.s, ctx.shp, ctx.bases, ctx.kcat = s, shp, bases, None
        return tuple(ys)

    @staticmethod
    def backward(ctx, *gs):
        x2, xa_all, *AB = ctx.saved_tensors
        As, Bs = AB[0::2], AB[1::2]
        s = ctx.s
        jobs, gx, off = [], None, 0
        # every sibling's s g B lands in its column slice of one [M, sum r]
        # buffer (strided GEMM output: no concatenation pass)
        gxa_all = (x2.new_empty if all(g is not None for g in gs) else x2.new_zeros)(xa_all.shape)
        gxas = []
        for base, A, B, g in zip(ctx.bases, As, Bs, gs):
            r = A.shape[0]
            if g is None:
                gxas.append(gxa_all[:, off:off + r])
                off += r
                continue
            g2 = g.reshape(-1, g.shape[-1]).to(x2.dtype)
            if _GXA_SLICES:
                gxa_all[:, off:off + r] = _skinny(g2, B.t(), s)
            else:
                gxas.append(_skinny(g2, B.t(), s))
            # dB [N, r] (the K-concat forward saved s x A^T: alpha 1)
            jobs.append((xa_all[:, off:off + r], g2, 1.0 if ctx.kcat else s, True))
            if ctx.needs_input_grad[0]:
                if not ctx.kcat and _g8_bwd_ok(g2, base):
                    gx = _g8_grad_x(g2, base, acc=gx)          # siblings accumulate in the GEMM epilogue
                else:
                    w = (_aug_weight(base, ctx.kcat[0], off, ctx.kcat[1])[:, :base.in_features] if ctx.kcat
                         else _base_dense_weight(base, x2.dtype))
                    gx = torch.mm(g2, w) if gx is None else gx.addmm_(g2, w)
            off += r
        if not _GXA_SLICES:
            gxa_all = torch.cat(gxas, 1)
        # [sum r, K] (one pass over x) + every dB: one slab, one cast
        *gBs, gA_all = _tn_many(jobs + [(gxa_all, x2, 1.0, False)], As[0].dtype)
        grads = [(None, gBs.pop(0) if g is not None else torch.zeros_like(B)) for B, g in zip(Bs, gs)]
        if gx is not None:
            _rank_update_(gx, gxa_all, torch.cat(As, 0).t())
            gx = gx.view(ctx.shp)
        out, off = [], 0
        for (A, (_, gB)) in zip(As, grads):
            r = A.shape[0]
            out += [gA_all[off:off + r], gB]
            off += r
        return (gx, None, None, *out)


class LoraLinear(nn.Module):
    """base(x) + B(A(dropout(pool(x)))) * scaling over a frozen base layer
    (LowBitLinear -> QLoRA/QA-LoRA, DenseLinear/nn.Linear -> LoRA)."""

    def __init__(self, base: nn.Module, r: int, alpha: int, dropout: float = 0.0, qa_lora: bool = False,
                 use_rslora: bool = False, dtype=torch.bfloat16):
        super().__init__()
        self.base_layer = base
        for p in base.parameters():
            p.requires_grad_(False)
        self.in_features, self.out_features = base.in_features, base.out_features
        self.r, self.lora_alpha = r, alpha
        self.scaling = alpha / (math.sqrt(r) if use_rslora else r)
        self.qa_group = 0
        if qa_lora:
            if not isinstance(base, LowBitLinear):
                raise ValueError("QA-LoRA needs a low-bit base layer")
            self.qa_group = Q.get_format(base.qtype).block
        in_a = self.in_features // self.qa_group if self.qa_group else self.in_features
        dev = base.weight.device if base.weight.device.type != "meta" else "cpu"
        self.lora_A = nn.Linear(in_a, r, bias=False, device=dev, dtype=dtype)
        self.lora_B = nn.Linear(r, self.out_features, bias=False, device=dev, dtype=dtype)
        self.lora_dropout = nn.Dropout(dropout) if dropout > 0 else nn.Identity()
        self.reset_lora_parameters()
        self.merged = False
        self.disable_adapters = False

    def reset_lora_parameters(self):
        nn.init.kaiming_uniform_(self.lora_A.weight, a=math.sqrt(5))
        nn.init.zeros_(self.lora_B.weight)

    def _pool(self, x):
        if not self.qa_group:
            return x
        return x.reshape(*x.shape[:-1], self.in_features // self.qa_group, self.qa_group).mean(-1)

    def _fused_ok(self, x) -> bool:
        b = self.base_layer
        return (_FUSED and isinstance(b, LowBitLinear) and not self.qa_group and torch.is_grad_enabled()
                and isinstance(self.lora_dropout, nn.Identity) and b.g_idx_map is None and b.mp_group is None
                and x.dtype == self.lora_A.weight.dtype and x.dtype in (torch.bfloat16, torch.float16)
                and x.device == b.weight.device and (x.requires_grad or self.lora_A.weight.requires_grad))

    def _group_forward(self, x):
        """sibling adapters sharing this input (get_peft_model links q/k/v and
        gate/up): the first one computes every sibling's output in one
        _LoraGroupFn node, the others pick theirs up (same input tensor)"""
        grp = self.__dict__.get("_lora_group")
        if not grp or not _GROUP:
            return None
        key = (id(x), x._version, x.data_ptr())
        cache = grp["cache"]
        if cache is not None and cache[0] == key and self in cache[1]:
            out = cache[1].pop(self)
            if not cache[1]:
                grp["cache"] = None
            return out
        mods = grp["mods"]
        if self is not mods[0] or not all(m._fused_ok(x) and not (m.disable_adapters or m.merged) for m in mods) \
                or len({m.scaling for m in mods}) != 1:
            return None
        ab = []
        for m in mods:
            ab += [m.lora_A.weight, m.lora_B.weight]
        ys = _LoraGroupFn.apply(x, self.scaling, [m.base_layer for m in mods], *ab)
        grp["cache"] = (key, {m: y for m, y in zip(mods[1:], ys[1:])})
        return ys[0]

    def forward(self, x):
        if not (self.disable_adapters or self.merged) and self._fused_ok(x):
            y = self._group_forward(x)
            if y is not None:
                return y
            return _LoraLowBitFn.apply(x, self.lora_A.weight, self.lora_B.weight, self.base_layer, self.scaling)
        result = self.base_layer(x)
        if self.disable_adapters or self.merged:
            return result
        a = self.lora_A.weight
        h = self._pool(self.lora_dropout(x)).to(a.dtype)
        return result + (self.lora_B(self.lora_A(h)) * self.scaling).to(result.dtype)

    def delta_weight(self) -> torch.Tensor:
        """dense [out, in] update B @ A * scaling (QA-LoRA expanded per group)"""
        d = (self.lora_B.weight.float() @ self.lora_A.weight.float()) * self.scaling
        if self.qa_group:
            d = d.repeat_interleave(self.qa_group, dim=1) / self.qa_group
        return d

    @torch.no_grad()
    def merge(self):
        """fold the adapter into the base weight (re-quantized for low-bit)"""
        base = self.base_layer
        d = self.delta_weight()
        if isinstance(base, LowBitLinear):
            w = base.dequantize(torch.float32) + d.to(base.weight.device)
            base.load_dense(w, device=base.weight.device)
        else:
            base.weight.data += d.to(base.weight.device, base.weight.dtype)
        self.merged = True


def _match(name: str, targets) -> bool:
    if targets is None:
        targets = DEFAULT_TARGETS
    if isinstance(targets, str):
        return re.fullmatch(targets, name) is not None
    leaf = name.split(".")[-1]
    return leaf in targets or any(name.endswith("." + t) for t in targets)


class PeftModel(nn.Module):
    """Wrapper returned by :func:`get_peft_model` (peft.PeftModel-like)."""

    def __init__(self, model: nn.Module, config: LoraConfig):
        super().__init__()
        self.base_model = model
        self.peft_config = {"default": config}

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self.base_model, name)

    def forward(self, *args, **kwargs):
        return self.base_model(*args, **kwargs)

    def generate(self, *args, **kwargs):
        return self.base_model.generate(*args, **kwargs)

    def lora_modules(self) -> Dict[str, LoraLinear]:
        return {n: m for n, m in self.base_model.named_modules() if isinstance(m, LoraLinear)}

    def adapter_state_dict(self) -> Dict[str, torch.Tensor]:
        sd = {}
        for n, m in self.lora_modules().items():
            sd[f"{n}.lora_A.weight"] = m.lora_A.weight.detach().cpu().contiguous()
            sd[f"{n}.lora_B.weight"] = m.lora_B.weight.detach().cpu().contiguous()
        cfg = self.peft_config["default"]
        for n, p in self.base_model.named_parameters():
            if cfg.modules_to_save and any(s in n for s in cfg.modules_to_save) and p.requires_grad:
                sd[n] = p.detach().cpu().contiguous()
        return sd

    def save_pretrained(self, path: str, **_):
        from safetensors.torch import save_file
        os.makedirs(path, exist_ok=True)
        save_file(self.adapter_state_dict(), os.path.join(path, "adapter_model.safetensors"))
        self.peft_config["default"].save_pretrained(path)

    @torch.no_grad()
    def load_adapter(self, path: str):
        from safetensors.torch import load_file
        sd = load_file(os.path.join(path, "adapter_model.safetensors"))
        mods = self.lora_modules()
        params = dict(self.base_model.named_parameters())
        for k, v in sd.items():
            if ".lora_A." in k or ".lora_B." in k:
                mname, which = k.rsplit(".lora_", 1)
                lin = getattr(mods[mname], "lora_" + which.split(".")[0])
                lin.weight.copy_(v.to(lin.weight.device, lin.weight.dtype))
            elif k in params:
                params[k].copy_(v.to(params[k].device, params[k].dtype))
        return self

    @classmethod
    def from_pretrained(cls, model: nn.Module, path: str, is_trainable: bool = False, **_):
        cfg = LoraConfig.from_pretrained(path)
        pm = get_peft_model(model, cfg)
        pm.load_adapter(path)
        if not is_trainable:
            for p in pm.parameters():
                p.requires_grad_(False)
        return pm

    @contextlib.contextmanager
    def disable_adapter(self):
        mods = list(self.lora_modules().values())
        for m in mods:
            m.disable_adapters = True
        try:
            yield
        finally:
            for m in mods:
                m.disable_adapters = False

    def merge_and_unload(self) -> nn.Module:
        for name, m in list(self.lora_modules().items()):
            m.merge()
            parent = self.base_model.get_submodule(name.rsplit(".", 1)[0]) if "." in name else self.base_model
            setattr(parent, name.rsplit(".", 1)[-1], m.base_layer)
        return self.base_model

    def get_nb_trainable_parameters(self):
        tr = sum(p.numel() for p in self.parameters() if p.requires_grad)
        tot = sum(p.numel() for p in self.parameters())
        return tr, tot

    def print_trainable_parameters(self):
        tr, tot = self.get_nb_trainable_parameters()
        print(f"trainable params: {tr:,d} || all params: {tot:,d} || trainable%: {100 * tr / max(tot, 1):.4f}")


def get_peft_model(model: nn.Module, config: LoraConfig, adapter_name: str = "default") -> PeftModel:
    """Wrap every targeted linear of ``model`` with a LoRA adapter."""
    for p in model.parameters():
        p.requires_grad_(False)
    qa = config.training_mode == "qalora"
    n = 0
    for name, mod in list(model.named_modules()):
        for cname, child in list(mod.named_children()):
            full = f"{name}.{cname}" if name else cname
            if not isinstance(child, (LowBitLinear, DenseLinear, nn.Linear)) or isinstance(child, LoraLinear):
                continue
            if not _match(full, config.target_modules):
                continue
            setattr(mod, cname, LoraLinear(child, config.r, config.lora_alpha, config.lora_dropout,
                                           qa_lora=qa and isinstance(child, LowBitLinear),
                                           use_rslora=config.use_rslora))
            n += 1
    if n == 0:
        raise ValueError(f"no module matched target_modules={config.target_modules}")
    link_lora_groups(model)
    if config.modules_to_save:
        for pn, p in model.named_parameters():
            if any(s in pn for s in config.modules_to_save) and p.is_floating_point():
                p.requires_grad_(True)
    return PeftModel(model, config)


def _cross_attention(name: str, mod: nn.Module) -> bool:
    """cross-attention blocks (mllama cross-attention layers, Whisper / T5
    encoder_attn / EncDecAttention): their k / v project another input than q"""
    leaf = name.rsplit(".", 1)[-1].lower()
    if getattr(mod, "is_cross_attention", False) or "cross" in leaf or "encoder_attn" in leaf \
            or "encdec" in leaf:
        return True
    return "crossattention" in type(mod).__name__.lower()


def link_lora_groups(model: nn.Module) -> int:
    """link sibling LoraLinear modules that read the same input (a parent's
    q/k/v, gate/up) for the grouped forward; returns the number of groups"""
    n = 0
    for mname, mod in model.named_modules():
        if _cross_attention(mname, mod):
            continue                  # k / v read the encoder states, not q's input
        for names in _GROUPS:
            mods = [getattr(mod, c, None) for c in names]
            if all(isinstance(m, LoraLinear) for m in mods) and \
                    len({m.in_features for m in mods}) == 1:
                grp = {"mods": mods, "cache": None}
                for m in mods:
                    m.__dict__["_lora_group"] = grp
                n += 1
    return n


def prepare_model_for_kbit_training(model: nn.Module, use_gradient_checkpointing: bool = True) -> nn.Module:
    """Freeze the base, keep norms in fp32, make inputs require grad (so
    checkpointed blocks backprop into the adapters) and enable gradient
    checkpointing (reference qlora.py:304-352)."""
    for p in model.parameters():
        p.requires_grad_(False)
    for m in model.modules():
        if not list(m.children()) and not isinstance(m, (LowBitLinear, DenseLinear, nn.Linear, nn.Embedding)):
            for p in m.parameters():
                if p.dtype in (torch.float16, torch.bfloat16):
                    p.data = p.data.float()
    if use_gradient_checkpointing:
        if hasattr(model, "enable_input_require_grads"):
            model.enable_input_require_grads()
        else:
            model.get_input_embeddings().register_forward_hook(lambda m, i, o: o.requires_grad_(True))
        if hasattr(model, "gradient_checkpointing_enable"):
            model.gradient_checkpointing_enable(gradient_checkpointing_kwargs={"use_reentrant": False})
    enable_training_kernels(model)
    return model


def enable_training_kernels(model: nn.Module) -> nn.Module:
    """On an MI355X: the fused lm_head + cross-entropy (training/fused_ce.py)
    and the HIP flash attention forward / backward (training/flash_attn.py)
    for the HF forward.  ILLM_TRAIN_CE=0 / ILLM_TRAIN_ATTN=0 keep HF's."""
    from .. import ops
    w = next((p for p in model.parameters()), None)
    if w is None or not w.is_cuda or not ops.native_gpu(w):
        return model
    if os.environ.get("ILLM_TRAIN_CE", "1") == "1" and hasattr(model, "lm_head"):
        from .fused_ce import patch_fused_ce
        patch_fused_ce(model)
    if os.environ.get("ILLM_TRAIN_ATTN", "1") == "1":
        from .flash_attn import patch_flash_attention
        patch_flash_attention(model)
    if os.environ.get("ILLM_TRAIN_ROPE", "1") == "1":
        _patch_rotary(model)
    # Default: the pure low-bit footprint -- each base GEMM dequantizes its
    # weight (forward) or W^T (grad_x) into a transient buffer for the dense
    # 8-phase kernel.  ILLM_TRAIN_DENSE_GB=<GiB> (or "auto": min(48, HBM / 4)
    # on >= 128 GiB devices) keeps the dequantized base resident instead -- on
    # a 288 GB MI355X a Llama-3-8B base costs 15 GB and saves the per-step
    # dequant passes -- and enables the K-concatenated adapter GEMMs.
    gb = os.environ.get("ILLM_TRAIN_DENSE_GB", "0")
    if gb == "auto":
        total = torch.cuda.get_device_properties(w.device).total_memory / 2 ** 30
        gb = min(48.0, 0.25 * total) if total >= 128 else 0.0
    gb = float(gb)
    if gb > 0:
        from ..ops.gemm import _DENSE_BUDGET, set_dense_budget
        if _DENSE_BUDGET < gb * 2 ** 30:
            set_dense_budget(gb)
    model._illm_train_dense_gb = gb
    return model


def _patch_rotary(model: nn.Module) -> int:
    """HF rotary-embedding modules (default rope: ``inv_freq``,
    ``attention_scaling``) compute cos / sin with a batched f32 matmul of the
    [D/2, 1] frequencies by the [1, T] positions -- a K = 1 library GEMM per
    forward.  The same products as one broadcast multiply (exact: each entry
    is a single f32 product either way).

    Only the standard 2-D form ([bs, seq] positions) is replaced: a rotary
    whose forward takes other positions (Qwen2-VL / Qwen2.5-Omni M-RoPE with
    [3, bs, seq]) keeps its own forward, and any call whose positions are not
    2-D falls back to the original forward."""
    n = 0
    for name, m in model.named_modules():
        if not name.endswith("rotary_emb") or not hasattr(m, "inv_freq") or not hasattr(m, "attention_scaling"):
            continue
        if getattr(m, "rope_type", "default") != "default" or getattr(m, "_illm_rope", False):
            continue
        if "VL" in type(m).__name__ or "Omni" in type(m).__name__ or hasattr(m, "mrope_section"):
            continue                    # multimodal (3-D M-RoPE) rotaries
        orig = m.forward

        def fwd(x, position_ids, *args, _m=m, _orig=orig, **kw):
            if position_ids.dim() != 2 or args or kw:
                return _orig(x, position_ids, *args, **kw)
            freqs = position_ids[:, :, None].float() * _m.inv_freq.float()[None, None, :]
            emb = torch.cat((freqs, freqs), dim=-1)
            return (emb.cos() * _m.attention_scaling).to(x.dtype), (emb.sin() * _m.attention_scaling).to(x.dtype)
        m.forward = fwd
        m._illm_rope = True
        n += 1
    return n


def cast_lora_weight(model: nn.Module, dtype=torch.bfloat16):
    """adapters and bf16 layers in ``dtype``, norms in fp32 (qlora.py:377-391)"""
    for name, m in model.named_modules():
        if isinstance(m, LowBitLinear):
            m.compute_dtype = dtype
        if isinstance(m, LoraLinear):
            m.lora_A.to(dtype)
            m.lora_B.to(dtype)
        if "norm" in name and not list(m.children()):
            m.to(torch.float32)
    return model
