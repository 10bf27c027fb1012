"""Typed entry points over ``torch.ops.ipex_llm_amd`` with device dispatch.

GPU tensors always go to the HIP kernels (see ``ops.native_gpu``); CPU
tensors use the C++ host library where one exists (quantizers, low-bit GEMM)
and the torch references otherwise.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from . import reference as R

__all__ = [
    "quantize", "dequantize", "kq_quantize", "kq_dequantize", "kq_linear", "fp8_linear", "fp8_act_quant",
    "fp8_quantize_weight", "dense_linear", "check_kernel_errors", "KernelError", "repack_to_device", "repack_from_device", "lowbit_matmul",
    "gemv_partials", "gemv_glu", "add_rms_norm", "rms_norm", "layer_norm", "rope_kv",
    "attn_decode", "glu", "attn_softmax_", "moe_topk", "reduce_partials", "to_fp8_bytes", "GEMV_MAX_M", "gather_kv",
    "moe_align", "moe_gemm", "moe_gemv_glu", "moe_gemv_partials", "moe_combine", "moe_route", "moe_gemv_accum", "rope_kv_fused", "gemv_glu_in", "gemv_accum", "gemv_accum_norm", "gemv_glu_ss",
    "attn_decode_split", "gemv_attn", "gemv_norm_in", "attn_decode_rope", "attn_decode_rope_split", "attn_prefill", "moe_group_topk",
]


def _ops():
    from . import require
    return require()


def _native(t: torch.Tensor) -> bool:
    from . import native_gpu
    return native_gpu(t)


# ------------------------------------------------------------ quantization
def quantize(w: torch.Tensor, fmt: int, imatrix: Optional[torch.Tensor] = None,
             scale_search: bool = False) -> torch.Tensor:
    """Dense [n, k] -> packed blob.  GPU input -> MI355X tiled layout
    (quantized on device); CPU input -> canonical planar layout (C++)."""
    if _native(w) and imatrix is None:
        return _ops().quantize_device(w, fmt, scale_search)
    if w.is_cuda:
        return _ops().repack_to_device(_ops().quantize_cpu(w.cpu(), fmt, imatrix, scale_search),
                                       fmt, w.shape[0], w.shape[1]).to(w.device)
    return _ops().quantize_cpu(w, fmt, imatrix, scale_search)


def dequantize(blob: torch.Tensor, fmt: int, n: int, k: int, dtype=torch.float32,
               device_layout: Optional[bool] = None) -> torch.Tensor:
    device_layout = blob.is_cuda if device_layout is None else device_layout
    if device_layout:
        if _native(blob) and dtype in (torch.bfloat16, torch.float16):
            return _ops().dequantize_device(blob, fmt, n, k, dtype)
        return R.dequantize_device_blob(blob, fmt, n, k).to(dtype)
    if blob.is_cuda:
        return R.dequantize_canonical(blob, fmt, n, k).to(dtype)
    return _ops().dequantize_cpu(blob, fmt, n, k).to(dtype)


def repack_to_device(canon: torch.Tensor, fmt: int, n: int, k: int) -> torch.Tensor:
    return _ops().repack_to_device(canon.cpu(), fmt, n, k)


def repack_from_device(dev: torch.Tensor, fmt: int, n: int, k: int) -> torch.Tensor:
    return _ops().repack_from_device(dev.cpu(), fmt, n, k)


def to_fp8_bytes(x: torch.Tensor, e5m2: bool) -> torch.Tensor:
    return _ops().to_fp8_bytes(x.cpu(), e5m2)


# ------------------------------------------------------------ k-quants
def kq_quantize(w: torch.Tensor, fmt: int, imatrix: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dense [n, k] -> GGUF k-quant super-blocks (C++ host quantizer)"""
    return _ops().kq_quantize(w.float().cpu().contiguous(), fmt, imatrix)


def kq_dequantize(blob: torch.Tensor, fmt: int, n: int, k: int, dtype=torch.float32) -> torch.Tensor:
    if blob.is_cuda and not _native(blob):
        return _ops().kq_dequantize(blob.cpu(), fmt, n, k, torch.float32).to(blob.device, dtype)
    return _ops().kq_dequantize(blob, fmt, n, k, dtype)


def kq_linear(x: torch.Tensor, blob: torch.Tensor, fmt: int, n: int, k: int) -> torch.Tensor:
    """x @ W^T for a k-quant W (HIP GEMV / dequant + BLAS on the GPU, C++ on the host)"""
    if x.is_cuda and not _native(x):
        return F.linear(x, kq_dequantize(blob, fmt, n, k, torch.float32).to(x.dtype))
    return _ops().kq_linear(x, blob, fmt, n, k)


# ------------------------------------------------------------ kernel error word
class KernelError(RuntimeError):
    pass


_KERR_NAMES = {1: "block-table entry outside the KV cache", 2: "cache slot outside the KV cache",
               4: "expert id out of range", 8: "sequence length out of range (block-table row / split grid)",
               16: "token id outside the vocabulary", 32: "launch geometry does not cover the output (debug build)",
               64: "a peer rank did not answer in time (collective / expert all-to-all timed out)"}


def check_kernel_errors(device=None, reset: bool = True):
    """Raise KernelError if a HIP kernel skipped an out-of-range index since
    the last check (device-side bounds checks).  Synchronises.
    ILLM_CHECK_KERNELS=1 makes the engines call this after every step."""
    if device is None:
        if not torch.cuda.is_available():
            return 0
        device = torch.device("cuda", torch.cuda.current_device())
    like = torch.empty(0, device=device)
    if like.is_cuda and not _native(like):
        return 0
    code = int(_ops().kernel_errors(like, reset)[0])
    if code:
        what = [v for k, v in _KERR_NAMES.items() if code & k]
        raise KernelError(f"HIP kernel bounds check failed (code {code}): {', '.join(what)}")
    return 0


CHECK_KERNELS = __import__("os").environ.get("ILLM_CHECK_KERNELS", "0") == "1"


# ------------------------------------------------------------ dense skinny GEMM
def dense_linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x @ w^T (+ bias) for dense bf16/fp16 weights: the streaming skinny
    kernel for <= 16 rows on the GPU, the library GEMM otherwise"""
    if x.is_cuda and _native(x) and x.numel() // x.shape[-1] <= 16:
        return _ops().dense_linear(x, w, bias)
    return F.linear(x, w, bias)


# ------------------------------------------------------------ torch_fp8
FP8_MAX = {False: 448.0, True: 57344.0}


def fp8_quantize_weight(w: torch.Tensor, e5m2: bool = False, per_channel: bool = False):
    """dense [n, k] -> (uint8 fp8 codes [n, k], f32 scale [1] or [n]): the
    reference's dynamic_scaled_fp8_quant of a weight (per-tensor amax)"""
    wf = w.float()
    amax = wf.abs().amax(dim=1, keepdim=True) if per_channel else wf.abs().amax().reshape(1, 1)
    s = torch.where(amax > 0, amax / FP8_MAX[e5m2], torch.ones_like(amax))
    q = (wf / s).clamp(-FP8_MAX[e5m2], FP8_MAX[e5m2]).to(torch.float8_e5m2 if e5m2 else torch.float8_e4m3fn)
    return q.view(torch.uint8), s.reshape(-1).float()


def fp8_act_quant(x: torch.Tensor):
    """per-token e4m3 quantization -> (codes uint8 [M, K], scales f32 [M])"""
    return _ops().fp8_act_quant(x)


def fp8_linear(x: torch.Tensor, w: torch.Tensor, w_scale: torch.Tensor, bias: Optional[torch.Tensor] = None,
               e5m2: bool = False) -> torch.Tensor:
    """y = x @ (w * w_scale)^T (+ bias): GEMV for <= 16 rows, else per-token
    fp8 activations on the block-scaled f8f6f4 MFMA GEMM (run_linear_fp8)"""
    if x.is_cuda and not _native(x):
        wd = w.view(torch.float8_e5m2 if e5m2 else torch.float8_e4m3fn).float() * w_scale.float().view(-1, 1)
        y = F.linear(x.float(), wd, None if bias is None else bias.float())
        return y.to(x.dtype)
    M = x.numel() // x.shape[-1]
    if x.is_cuda and M >= FP8_LIB_MIN_M and _FP8_LIB[0] is not False:
        y = _fp8_linear_lib(x, w, w_scale, bias, e5m2)
        if y is not None:
            return y
    return _ops().fp8_linear(x, w, w_scale, bias, e5m2)


# prefill-size fp8 GEMMs: per-token e4m3 activations (our quant kernel) on the
# hipBLASLt fp8 GEMM, row / column scales applied by its rowwise-scaled
# epilogue.  Measured on MI355X (Llama-3-8B projections, M = 1024-8192,
# profiles/fp8_gemm_sweep_r3.jsonl): 2.4-3.0 PFLOP/s vs 0.47-0.68 for the
# hand-written 128 x 128 f8f6f4 kernel, which stays the path for
# 16 < M < FP8_LIB_MIN_M and wherever the library call is unavailable.
FP8_LIB_MIN_M = int(__import__("os").environ.get("ILLM_FP8_LIB_MIN_M", "128"))
_FP8_LIB = [None]      # None: untested, True / False: rowwise-scaled _scaled_mm works


def _fp8_linear_lib(x, w, w_scale, bias, e5m2):
    if not hasattr(torch, "_scaled_mm"):
        _FP8_LIB[0] = False
        return None
    K, N = x.shape[-1], w.shape[0]
    if K % 16 or N % 16 or e5m2:          # (rowwise-scaled e4m3 x e5m2 is not a library combination)
        return None
    x2 = x.reshape(-1, K)
    try:
        xq, sx = _ops().fp8_act_quant(x2)
        wt = w.view(torch.float8_e5m2 if e5m2 else torch.float8_e4m3fn).t()
        sw = w_scale.float().reshape(1, -1).expand(1, N).contiguous()
        y = torch._scaled_mm(xq.view(torch.float8_e4m3fn), wt, scale_a=sx.view(-1, 1), scale_b=sw,
                             bias=None, out_dtype=x.dtype)
        _FP8_LIB[0] = True
    except (RuntimeError, TypeError, ValueError):
        _FP8_LIB[0] = False
        return None
    if bias is not None:
        y = y + bias.to(y.dtype)
    return y.view(*x.shape[:-1], N)


# ------------------------------------------------------------ low-bit GEMM
GEMV_MAX_M = 64


def lowbit_matmul(x: torch.Tensor, blob: torch.Tensor, fmt: int, n: int, k: int,
                  bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x @ W^T (+ bias) for a packed weight W[n, k]."""
    if x.is_cuda:
        if _native(x):
            M = x.numel() // k
            if M <= GEMV_MAX_M:
                return _ops().gemv(x, blob, fmt, n, k, bias, 0, 0, 0)
            from .gemm import lowbit_gemm
            return lowbit_gemm(x, blob, fmt, n, k, bias)
        w = R.dequantize_device_blob(blob, fmt, n, k).to(x.dtype)
        return F.linear(x, w, bias)
    y = _ops().linear_cpu(x, blob, fmt, n, k)
    if bias is not None:
        y = y + bias.float()
    return y.to(x.dtype)


def gemv_partials(x, blob, fmt, n, k, ksplit: int) -> torch.Tensor:
    """f32 split-K partial slabs [ksplit, M, n] (summed by add_rms_norm)."""
    return _ops().gemv(x, blob, fmt, n, k, None, 1, ksplit, 0)


def gemv_accum(x, blob, fmt, n, k, acc: torch.Tensor, ksplit: int = 0,
               zero: Optional[torch.Tensor] = None, rope=None) -> torch.Tensor:
    """acc [M, n] f32 (zero on entry) += x @ W^T via split-K f32 atomics; the
    consumer (add_rms_norm / rope_kv_fused with zero_*=True) re-zeroes it, or
    a later launch does through ``zero`` (a buffer whose readers are done).
    ``rope`` = (cos_sin [max_pos, D/2, 2], pos [M], rotated columns, D): NeoX
    RoPE applied to each split's partial before its atomic add (rotation is
    linear), so ``acc`` ends up holding rotated q / k."""
    if _native(x):
        rc, rp, rn, rd = rope if rope is not None else (None, None, 0, 0)
        _ops().gemv_accum(x, blob, fmt, n, k, acc, ksplit, zero, rc, rp, rn, rd)
        return acc
    if zero is not None:
        zero.zero_()
    acc += _rope_cols(lowbit_matmul(x, blob, fmt, n, k).float(), rope, x.dtype).view_as(acc)
    return acc


def gemv_accum_norm(x, blob, fmt, n, k, acc: torch.Tensor, ctr: torch.Tensor, residual: torch.Tensor,
                    res_out: torch.Tensor, norm_w: torch.Tensor, unit_offset: bool, xo: torch.Tensor,
                    ss: torch.Tensor, zero: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``gemv_accum`` whose last split-K workgroup per column block also does
    the residual add and stages the deferred RMSNorm input of the next GEMV
    (decode o_proj -> gate/up without a norm launch): res_out = rnd(rnd(x W^T)
    + residual), xo = rnd(w * res_out), ss[m] += sum(res_out[m]^2); ``acc``
    (zero on entry) is left zeroed, ``ctr`` int32 tickets (zero on the first
    call) reset themselves.  The consumer is ``gemv_glu_ss``."""
    if _native(x):
        _ops().gemv_accum_norm(x, blob, fmt, n, k, acc, ctr, residual, res_out, norm_w, unit_offset, xo, ss, zero)
        return xo
    if zero is not None:
        zero.zero_()
    y = lowbit_matmul(x, blob, fmt, n, k).float().view_as(acc) + acc
    h = (y.to(residual.dtype).float() + residual.float()).to(residual.dtype)
    res_out.copy_(h.view_as(res_out))
    w = norm_w.float() + 1.0 if unit_offset else norm_w.float()
    xo.copy_((w.to(residual.dtype).float() * h.float()).to(residual.dtype).view_as(xo))
    ss[:h.shape[0]] += h.float().pow(2).sum(-1)
    acc.zero_()
    return xo


def gemv_glu_ss(x, blob, fmt, n, k, act: int, ss: torch.Tensor, ss_n: int, eps: float) -> torch.Tensor:
    """act(s x Wg^T) * (s x Wu^T) with s = rsqrt(ss / ss_n + eps) per row: the
    gate/up GEMV over ``gemv_accum_norm``'s deferred-norm input."""
    if _native(x):
        return _ops().gemv_glu_ss(x, blob, fmt, n, k, act, ss, ss_n, eps)
    from ..models.decoder import deinterleave_glu
    M = x.numel() // k
    inv = torch.rsqrt(ss[:M].float() / ss_n + eps)[:, None]
    g, u = deinterleave_glu(lowbit_matmul(x, blob, fmt, n, k).float())
    g, u = g * inv, u * inv
    return ((F.silu(g) if act == 0 else F.gelu(g, approximate="tanh")) * u).to(x.dtype).contiguous()


def _rope_cols(y: torch.Tensor, rope, dtype) -> torch.Tensor:
    """fallback of the GEMV RoPE epilogue: rotate_half RoPE of the first
    ``cols`` columns of y [M, n] (heads of D dims) at positions ``pos``"""
    if rope is None:
        return y
    cs, pos, cols, D = rope
    half = D // 2
    tab = cs[pos.long()].to(dtype).float()                    # [M, half, 2], cos/sin rounded like HF
    c = torch.cat([tab[..., 0], tab[..., 0]], -1)[:, None, :]
    sn = torch.cat([tab[..., 1], tab[..., 1]], -1)[:, None, :]
    h = y[:, :cols].reshape(y.shape[0], cols // D, D)
    rot = torch.cat([-h[..., half:], h[..., :half]], -1)
    y = y.clone()
    y[:, :cols] = (h * c + rot * sn).reshape(y.shape[0], cols)
    return y


def gemv_norm_in(acc_in: torch.Tensor, residual: torch.Tensor, res_out: torch.Tensor, norm_w: torch.Tensor,
                 eps: float, unit_offset: bool, blob, fmt, n, k, glu: bool, act: int = 0,
                 acc_out: Optional[torch.Tensor] = None, zero: Optional[torch.Tensor] = None,
                 ss: Optional[torch.Tensor] = None, rope=None) -> torch.Tensor:
    """Decode projection of rms_norm(residual + acc_in) * norm_w with the
    residual add and the norm done in the GEMV prologue (no norm launch):
    res_out = residual + acc_in; returns act(gate)*up (``glu``) or acc_out
    += x @ W^T (atomics).  acc_in is only read; ``zero`` is zeroed first.

    ``ss`` (f32 [M], zero on entry): deferred norm -- the atomic output is
    W (w * h) without the 1/rms row scale, ss receives the per-row sum of
    squares of h and the consumer (rope_kv_fused / attn_decode_rope /
    gemv_glu_in with pss/xss) applies rsqrt(ss / k + eps); a GLU launch
    applies it itself before the activation."""
    if _native(residual):
        rc, rp, rn, rd = rope if rope is not None else (None, None, 0, 0)
        return _ops().gemv_norm_in(acc_in, residual, res_out, norm_w, eps, unit_offset, blob, fmt, n, k,
                                   2 if glu else 3, act, acc_out, zero, ss, rc, rp, rn, rd)
    if zero is not None:
        zero.zero_()
    x = acc_in.to(residual.dtype).view_as(residual)
    if ss is not None:
        h = (x + residual).to(residual.dtype)
        res_out.copy_(h)
        w = norm_w.float() + 1.0 if unit_offset else norm_w.float()
        xp = (w.to(residual.dtype).float() * h.float()).to(residual.dtype)
        sq = h.float().pow(2).sum(-1)
        if glu:
            from ..models.decoder import deinterleave_glu
            inv = torch.rsqrt(sq / k + eps)[:, None]
            g, u = deinterleave_glu(lowbit_matmul(xp, blob, fmt, n, k).float())
            g, u = g * inv, u * inv
            return ((F.silu(g) if act == 0 else F.gelu(g, approximate="tanh")) * u).to(residual.dtype).contiguous()
        ss[:sq.numel()] += sq
        acc_out += _rope_cols(lowbit_matmul(xp, blob, fmt, n, k).float(), rope, residual.dtype).view_as(acc_out)
        return acc_out
    normed, new_res = R.add_rms_norm(x, residual, norm_w, eps, unit_offset)
    res_out.copy_(new_res)
    if glu:
        from ..models.decoder import deinterleave_glu
        g, u = deinterleave_glu(lowbit_matmul(normed, blob, fmt, n, k))
        return ((F.silu(g) if act == 0 else F.gelu(g, approximate="tanh")) * u).contiguous()
    acc_out += _rope_cols(lowbit_matmul(normed, blob, fmt, n, k).float(), rope, residual.dtype).view_as(acc_out)
    return acc_out


def gemv_glu(x, blob, fmt, n, k, act: int = 0) -> torch.Tensor:
    """act(x @ Wg^T) * (x @ Wu^T) for a tile-interleaved gate/up weight."""
    return _ops().gemv(x, blob, fmt, n, k, None, 2, 1, act)


def gemv_glu_in(part, blob, fmt, n, k, act: int = 0, ksplit: int = 0, dtype=torch.bfloat16,
                acc: Optional[torch.Tensor] = None, zero: Optional[torch.Tensor] = None,
                xss: Optional[torch.Tensor] = None, xss_n: int = 0, xss_eps: float = 0.0) -> torch.Tensor:
    """down-projection over act(gate)*up taken straight from the gate/up
    GEMV's split-K slabs (or atomic accumulator) ``part`` [ns, M, 2k];
    returns f32 slabs [ks, M, n], or ``acc`` [M, n] += the product (atomics).
    ``zero`` (a buffer whose readers are done) is zeroed by the launch.
    ``xss``: deferred-norm sums of squares of the gate/up input (rows scaled by
    rsqrt(xss / xss_n + xss_eps) before the activation)."""
    if _native(part):
        return _ops().gemv_glu_in(part, blob, fmt, n, k, act, ksplit, dtype, acc, zero, xss, xss_n, xss_eps)
    from ..models.decoder import deinterleave_glu
    ps = part.sum(0)
    if xss is not None:
        ps = ps * torch.rsqrt(xss[:ps.shape[0]] / xss_n + xss_eps)[:, None]
    g, u = deinterleave_glu(ps)
    a = ((F.silu(g) if act == 0 else F.gelu(g, approximate="tanh")) * u).to(dtype)
    if zero is not None:
        zero.zero_()
    y = lowbit_matmul(a, blob, fmt, n, k).float()
    if acc is not None:
        acc += y.view_as(acc)
        return acc
    return y.unsqueeze(0)


def reduce_partials(ws, bias=None, dtype=torch.bfloat16):
    return _ops().reduce_partials(ws, bias, dtype)


# ------------------------------------------------------------ norms / act
def add_rms_norm(x: Optional[torch.Tensor], residual: Optional[torch.Tensor], w: torch.Tensor,
                 eps: float, partials: Optional[torch.Tensor] = None,
                 unit_offset: bool = False, zero_partials: bool = False) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """residual += x (or the sum of GEMV partials); returns (rms_norm(residual), residual).
    On GPU the residual is updated in place.  zero_partials re-zeroes the
    partial slab after reading it (atomic accumulators, gemv_accum)."""
    if _native(w):
        out = _ops().add_rms_norm(x, partials, residual, w, eps, unit_offset, True, zero_partials)
        return out, residual
    if partials is not None:
        x = partials.sum(0).to(w.dtype).view_as(residual) if residual is not None else partials.sum(0).to(w.dtype)
        if zero_partials:
            partials.zero_()
    normed, new_res = R.add_rms_norm(x, residual, w, eps, unit_offset)
    if residual is not None:
        residual.copy_(new_res)
    return normed, residual


def rms_norm(x, w, eps, unit_offset=False):
    if _native(x):
        return _ops().add_rms_norm(x.contiguous(), None, None, w, eps, unit_offset, False)
    return R.rms_norm(x, w, eps, unit_offset)


def layer_norm(x, w, b, eps):
    if _native(x) and x.shape[-1] % 8 == 0:
        return _ops().layer_norm(x, w, b, eps)
    return R.layer_norm(x, w, b, eps)


def glu(gu, act=0, tile=0):
    """act(gate) * up; gate / up are the two halves of the last dim, or
    (tile > 0) interleaved in groups of ``tile`` columns (the fused gate_up
    weight layout)."""
    I = gu.shape[-1] // 2
    if _native(gu) and I % 8 == 0 and (tile == 0 or (tile % 8 == 0 and I % tile == 0)):
        return _ops().glu(gu, act, tile)
    if tile:
        x = gu.reshape(*gu.shape[:-1], I // tile, 2, tile)
        gu = torch.cat([x[..., 0, :].reshape(*gu.shape[:-1], I), x[..., 1, :].reshape(*gu.shape[:-1], I)], -1)
    return R.glu(gu, act)


def attn_softmax_(x: torch.Tensor) -> torch.Tensor:
    """In-place softmax over the last dim (reference xe_addons.attn_softmax_inplaced,
    models/common.py:174-181).  f32 math, result in x's dtype.  A fully
    masked row (every score -inf) comes out as zeros on both paths."""
    if _native(x) and x.is_contiguous() and x.dtype in (torch.bfloat16, torch.float16):
        _ops().attn_softmax_(x)
        return x
    xf = x.float()
    y = torch.softmax(xf, -1)
    y = torch.where(torch.isneginf(xf.amax(-1, keepdim=True)), torch.zeros_like(y), y)
    return x.copy_(y.to(x.dtype))


def moe_topk(logits, k, renorm=True, scoring=0):
    if _native(logits) and logits.shape[-1] <= 512:
        return _ops().moe_topk(logits, k, renorm, scoring)
    return R.moe_topk(logits, k, renorm, scoring)


def moe_group_topk(logits, bias, k: int, n_group: int, topk_group: int, renorm: bool = True, scale: float = 1.0):
    """DeepSeek-V3 group-limited routing (sigmoid + correction bias, top
    groups by their top-2 sum, top-k, renormalise, routed scaling):
    logits [T, E] -> (weights f32 [T, k], ids int32 [T, k])."""
    if _native(logits) and logits.shape[-1] <= 512 and n_group <= 64:
        return _ops().moe_group_topk(logits, bias, k, n_group, topk_group, renorm, scale)
    return R.moe_group_topk(logits, bias, k, n_group, topk_group, renorm, scale)


def moe_align(ids, e0: int, num_local: int):
    """top-k ids [T, k] -> (off [El+1], rows [T*k]): pair ids grouped by local
    expert (experts outside [e0, e0+El) are skipped, for expert parallel)."""
    if _native(ids):
        return _ops().moe_align(ids, e0, num_local)
    return R.moe_align(ids, e0, num_local)


def moe_gemv_glu(x, blob, fmt, n, k, off, rows, topk: int, act: int = 0):
    """Grouped GLU GEMV over experts: x [T, k] -> [T*topk, n/2] (pair rows)."""
    P = x.shape[0] * topk
    return _ops().moe_gemv(x, blob, fmt, n, k, off, rows, topk, P, 2, 1, act)


def moe_gemv_partials(x, blob, fmt, n, k, off, rows, ksplit: int = 0):
    """Grouped GEMV over experts on pair rows: x [P, k] -> f32 [ks, P, n]."""
    return _ops().moe_gemv(x, blob, fmt, n, k, off, rows, 1, x.shape[0], 1, ksplit, 0)


def moe_gemv_accum(x, blob, fmt, n, k, off, rows, acc, w, topk: int, ksplit: int = 0):
    """Grouped down projection with the routing-weighted combine in the
    epilogue: acc[p // topk] += w[p] * x[p] @ W_e^T (f32 atomics; acc [T, n]
    zero on entry, re-zeroed by its consumer)."""
    _ops().moe_gemv_accum(x, blob, fmt, n, k, off, rows, acc, w.contiguous(), topk, ksplit)
    return acc


def moe_route(x, router, k: int, renorm: bool, scoring: int, e0: int, num_local: int,
              counter: Optional[torch.Tensor] = None):
    """Decode router (<= 16 tokens) in one launch: logits = x router^T (f32),
    softmax (scoring 0) / sigmoid (1) top-k (+renormalise) and the per-local-
    expert pair lists -> (w f32 [T, k], ids int32 [T, k], off [El+1], rows [T*k]).
    ``counter``: int32 device scalar, zero on entry and left zero."""
    if _native(x) and x.shape[0] <= 16 and router.shape[0] <= 512 and k <= 16 and num_local <= 512:
        if counter is None:
            counter = torch.zeros(1, dtype=torch.int32, device=x.device)
        return _ops().moe_route(x, router.to(x.dtype), k, renorm, scoring, e0, num_local, counter)
    logits = (x.float() @ router.float().t())
    w, ids = R.moe_topk(logits, k, renorm, scoring)
    off, rows = R.moe_align(ids, e0, num_local)
    return w, ids, off, rows


def moe_gemm(x, blob, fmt, n, k, off, rows, xdiv: int, x_sorted: bool, out_sorted: bool, glu: bool,
             act: int = 0, out_f32: bool = False):
    """Grouped low-bit GEMM over (token, expert) pairs sorted by expert
    (``moe_align``), one launch for every local expert.  blob: uint8 [E, bytes].
    Rows of the result: sorted position (``out_sorted``) or pair id."""
    if _native(x):
        return _ops().moe_gemm(x, blob, fmt, n, k, off, rows, xdiv, x_sorted, out_sorted, glu, act, out_f32)
    return R.moe_gemm(x, blob, fmt, n, k, off, rows, xdiv, x_sorted, out_sorted, glu, act, out_f32)


def moe_combine(part, w, ids, e0: int, num_local: int, dtype=torch.bfloat16):
    """y[t] = sum_j w[t, j] * sum_s part[s, t*k+j] over local experts."""
    if _native(part):
        return _ops().moe_combine(part, w, ids, e0, num_local, dtype)
    return R.moe_combine(part, w, ids, e0, num_local, dtype)


# ------------------------------------------------------------ attention
def rope_kv(qkv, q_out, k_cache, v_cache, slots, pos, inv_freq, Hq, Hkv, D, rot_dim=None,
            interleaved=False, q_norm=None, k_norm=None, norm_eps=1e-6, q_scale=1.0,
            kv_fp8=0, k_scale=1.0, v_scale=1.0):
    """Rotate q/k of a fused QKV projection, write q to q_out [T, Hq, D] and
    k/v into the paged cache [nblocks, Hkv, bs, D] at ``slots``."""
    rot_dim = rot_dim or D
    if _native(qkv):
        _ops().rope_kv(qkv, q_out, k_cache, v_cache, slots, pos, inv_freq, q_norm, k_norm, norm_eps,
                       q_scale, Hq, Hkv, D, rot_dim, interleaved, kv_fp8, k_scale, v_scale)
        return q_out
    T = qkv.numel() // qkv.shape[-1]
    x = qkv.reshape(T, Hq + 2 * Hkv, D)
    q, k, v = x[:, :Hq], x[:, Hq:Hq + Hkv], x[:, Hq + Hkv:]
    if q_norm is not None:
        q = R.rms_norm(q, q_norm, norm_eps)
    if k_norm is not None:
        k = R.rms_norm(k, k_norm, norm_eps)
    if inv_freq.dim() == 3:  # precomputed [P, rot/2, 2] table
        cs = inv_freq[pos.long()]
        cos = torch.cat([cs[..., 0]] * 2, -1).to(qkv.dtype)
        sin = torch.cat([cs[..., 1]] * 2, -1).to(qkv.dtype)
    else:
        cos, sin = R.rope_cos_sin(pos, inv_freq[: rot_dim // 2], qkv.dtype)
    if interleaved:
        cos = torch.cat([cos[:, : rot_dim // 2]] * 2, -1)
        sin = torch.cat([sin[:, : rot_dim // 2]] * 2, -1)
    q = R.apply_rope(q, cos, sin, interleaved, rot_dim)
    k = R.apply_rope(k, cos, sin, interleaved, rot_dim)
    q_out.view(T, Hq, D).copy_(q * q_scale if q_scale != 1.0 else q)
    bs = k_cache.shape[2]
    ok = slots >= 0
    s = slots[ok]
    blk, off = s // bs, s % bs
    if kv_fp8:
        k_cache[blk, :, off] = to_fp8_bytes((k[ok] / k_scale).float(), kv_fp8 == 1).to(k_cache.device)
        v_cache[blk, :, off] = to_fp8_bytes((v[ok] / v_scale).float(), kv_fp8 == 1).to(v_cache.device)
    else:
        k_cache[blk, :, off] = k[ok].to(k_cache.dtype)
        v_cache[blk, :, off] = v[ok].to(v_cache.dtype)
    return q_out


def rope_kv_fused(part, bias, q_out, k_cache, v_cache, pos, block_tables, tq, inv_freq, Hq, Hkv, D, rot_dim=None,
                  interleaved=False, q_norm=None, k_norm=None, norm_eps=1e-6, q_scale=1.0, kv_fp8=0,
                  k_scale=1.0, v_scale=1.0, pos_offset=None, zero_part=False, pss=None, pss_n=0, pss_eps=0.0):
    """rope_kv over the split-K partials of the QKV GEMV ([ks, T, N] f32,
    summed + bias in the kernel) with device-side slots from the block table.
    ``pss``: deferred-norm sums of squares of the qkv input (row t scaled by
    rsqrt(pss[t] / pss_n + pss_eps) before the bias)."""
    rot_dim = rot_dim or D
    if _native(part):
        _ops().rope_kv_fused(part, bias, q_out, k_cache, v_cache, pos, block_tables, tq, inv_freq, q_norm, k_norm,
                             norm_eps, q_scale, Hq, Hkv, D, rot_dim, interleaved, kv_fp8, k_scale, v_scale,
                             pos_offset, zero_part, pss, pss_n, pss_eps)
        return q_out
    qkv = part.sum(0)
    if pss is not None:
        qkv = qkv * torch.rsqrt(pss[:qkv.shape[0]] / pss_n + pss_eps)[:, None]
    if zero_part:
        part.zero_()
    if bias is not None:
        qkv = qkv + bias.float()
    qkv = qkv.to(q_out.dtype)
    bs = k_cache.shape[2]
    seq = torch.arange(pos.numel(), device=pos.device) // tq
    ci = pos - (pos_offset[seq] if pos_offset is not None else 0)
    slots = block_tables.long()[seq, ci // bs] * bs + ci % bs
    return rope_kv(qkv, q_out, k_cache, v_cache, slots, pos, inv_freq, Hq, Hkv, D, rot_dim, interleaved, q_norm,
                   k_norm, norm_eps, q_scale, kv_fp8, k_scale, v_scale)


def gather_kv(cache, block_tables, b, L, kv_fp8=0, scale=1.0, dtype=torch.bfloat16):
    """[L, Hkv, D] view of sequence b's cached keys/values (reference path)."""
    bs = cache.shape[2]
    nblk = (L + bs - 1) // bs
    blks = block_tables[b, :nblk].long()
    x = cache[blks].permute(0, 2, 1, 3).reshape(nblk * bs, cache.shape[1], cache.shape[3])[:L]
    if kv_fp8:
        tab = R.code_table(6 if kv_fp8 == 1 else 5).to(x.device)
        x = (tab[x.long()] * scale).to(dtype)
    return x


def attn_decode(q, k_cache, v_cache, block_tables, seq_lens, nsplit, scale, softcap=0.0, window=0,
                kv_fp8=0, k_scale=1.0, v_scale=1.0, alibi=None, seq_lens_host=None):
    """q [B, Tq, Hq, D] against the paged cache -> [B, Tq, Hq, D]."""
    if _native(q):
        return _ops().attn_decode(q.contiguous(), k_cache, v_cache, block_tables, seq_lens, nsplit, scale,
                                  softcap, window, kv_fp8, k_scale, v_scale, alibi)
    B = q.shape[0]
    lens = seq_lens_host if seq_lens_host is not None else seq_lens.tolist()
    outs = []
    for b in range(B):
        L = int(lens[b])
        kk = gather_kv(k_cache, block_tables, b, L, kv_fp8, k_scale, q.dtype)
        vv = gather_kv(v_cache, block_tables, b, L, kv_fp8, v_scale, q.dtype)
        outs.append(R.attention(q[b:b + 1], kk[None], vv[None], True, scale, softcap, window, None, alibi))
    return torch.cat(outs, 0)


def attn_prefill(q, k_cache, v_cache, block_tables, seq_lens, Tq: int, scale: float, softcap: float = 0.0,
                 window: int = 0, kv_fp8: int = 0, k_scale: float = 1.0, v_scale: float = 1.0,
                 seq_lens_host=None):
    """Causal attention of q [B*Tq, Hq, D] (query t of sequence b at position
    seq_lens[b] - Tq + t) against the paged cache -> [B*Tq, Hq, D].  GPU:
    the flash-attention HIP kernel reading K/V straight from the cache
    blocks (D in {64, 128}); otherwise the fp32 reference per sequence."""
    D = q.shape[-1]
    if _native(q) and D in (64, 128) and k_cache.shape[2] % 64 == 0:
        return _ops().attn_prefill(q.contiguous(), k_cache, v_cache, block_tables, seq_lens, Tq, scale, softcap,
                                   window, kv_fp8, k_scale, v_scale)
    B = block_tables.shape[0]
    lens = seq_lens_host if seq_lens_host is not None else seq_lens.tolist()
    qv = q.view(B, Tq, q.shape[1], D)
    outs = []
    for b in range(B):
        L = int(lens[b])
        kk = gather_kv(k_cache, block_tables, b, L, kv_fp8, k_scale, q.dtype)
        vv = gather_kv(v_cache, block_tables, b, L, kv_fp8, v_scale, q.dtype)
        outs.append(R.attention(qv[b:b + 1], kk[None], vv[None], True, scale, softcap, window))
    return torch.cat(outs, 0).reshape(B * Tq, q.shape[1], D).to(q.dtype)


def attn_decode_rope(part, bias, cos_sin, pos, k_cache, v_cache, block_tables, seq_lens, nsplit, scale,
                     softcap, window, Hq: int, rot_dim: int, interleaved: bool, q_scale: float = 1.0,
                     dtype=torch.bfloat16, pss=None, pss_n: int = 0, pss_eps: float = 0.0, prerot: bool = False):
    """Decode attention (one new token per sequence) with the RoPE of q/k and
    the KV append fused in, reading q/k/v from the qkv GEMV's f32
    accumulator ``part`` [B, (Hq + 2 Hkv) * D].  Returns [B, 1, Hq, D].
    ``pss``: deferred-norm row sums of squares (see gemv_norm_in)."""
    return _ops().attn_decode_rope(part, bias, cos_sin, pos, k_cache, v_cache, block_tables, seq_lens, nsplit,
                                   scale, softcap, window, Hq, rot_dim, interleaved, q_scale, dtype, pss, pss_n,
                                   pss_eps, prerot)


def attn_decode_split(q, k_cache, v_cache, block_tables, seq_lens, nsplit, scale, softcap=0.0, window=0,
                      kv_fp8=0, k_scale=1.0, v_scale=1.0, alibi=None):
    """flash-decoding split kernel only: (o, m, l) partials [B, Hq, Tq, nsplit, D] / [..., 2]
    for a consumer that merges them itself (gemv_attn)."""
    return _ops().attn_decode_split(q.contiguous(), k_cache, v_cache, block_tables, seq_lens, nsplit, scale,
                                    softcap, window, kv_fp8, k_scale, v_scale, alibi)


def gemv_attn(po, pml, seq_lens, blob, fmt, n, k, acc=None, ksplit: int = 0, dtype=torch.bfloat16, zero=None,
              nw: int = 0):
    """o_proj over the attention partials (combined in the GEMV prologue):
    atomics into ``acc`` [T, n] when given, else f32 split-K slabs [ks, T, n].
    ``zero``: an f32 buffer zeroed first (a consumed accumulator); ``nw``:
    waves per workgroup (8 halves the re-reads of each head's partials)."""
    return _ops().gemv_attn(po, pml, seq_lens, blob, fmt, n, k, acc, ksplit, dtype, zero, nw)


def attn_decode_rope_split(part, bias, cos_sin, pos, k_cache, v_cache, block_tables, seq_lens, nsplit, scale,
                           softcap, window, Hq: int, rot_dim: int, interleaved: bool, q_scale: float = 1.0,
                           dtype=torch.bfloat16, pss=None, pss_n: int = 0, pss_eps: float = 0.0,
                           prerot: bool = False):
    """:func:`attn_decode_rope` without the combine: returns the (o, m, l)
    partials for :func:`gemv_attn`; ``part`` is left for the caller to zero."""
    return _ops().attn_decode_rope_split(part, bias, cos_sin, pos, k_cache, v_cache, block_tables, seq_lens,
                                         nsplit, scale, softcap, window, Hq, rot_dim, interleaved, q_scale, dtype,
                                         pss, pss_n, pss_eps, prerot)
