"""Low-bit linear layers (the FP4Params / LowBitLinear equivalents).

Reference: ``SRC/transformers/low_bit_linear.py`` -- ``FP4Params`` (332-491),
``MatMulLowBit`` (532-602), ``LowBitLinear`` (605-755), ``FP16Linear`` /
``BF16Linear`` (758-948).

MI355X design:
  * the packed weight is ONE uint8 blob per layer (codes | fp16 scales |
    fp16 mins).  On the host it is kept in the canonical planar layout (what
    checkpoints store); on the GPU in the MFMA-fragment tiled layout of
    ``csrc/common/formats.h``.  ``Module._apply`` converts between the two
    when the module changes device, so ``model.to("cuda")`` just works;
  * quantization is lazy: a dense weight placed with ``LowBitLinear.from_linear``
    is quantized on the device it lands on (C++ on the host, a HIP kernel on
    the GPU, so loading an 8B model quantizes in well under a second);
  * forward dispatches to the HIP skinny-GEMM (M <= 64) / GEMM kernels or to
    the C++ CPU GEMM;
  * training: ``MatMulLowBit`` gives ``grad_x`` through an on-device dequant
    (the base weight is frozen, as in QLoRA).
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..quantize import qtypes as Q


def _dev_total(fmt, n, k):
    from ..ops.reference import dev_total
    return dev_total(fmt, n, k)


def _canon_total(fmt, n, k):
    from ..ops.reference import canon_sizes
    c, s = canon_sizes(fmt, n, k)
    return c + 2 * s * (2 if fmt in (Q.FMT_ASYM_INT4, Q.FMT_ASYM_INT5) else 1)


class MatMulLowBit(torch.autograd.Function):
    """y = x W^T with a frozen low-bit W; backward gives grad_x only
    (reference: low_bit_linear.py:532-602)."""

    @staticmethod
    def forward(ctx, x, blob, fmt, n, k, layer):
        ctx.fmt, ctx.n, ctx.k = fmt, n, k
        ctx.save_for_backward(blob)
        ctx.xdtype = x.dtype
        return ops.lowbit_matmul(x, blob, fmt, n, k)

    @staticmethod
    def backward(ctx, grad_y):
        (blob,) = ctx.saved_tensors
        grad_x = None
        if ctx.needs_input_grad[0]:
            dt = grad_y.dtype if grad_y.dtype in (torch.bfloat16, torch.float16) else torch.bfloat16
            if blob.is_cuda and ops.native_gpu(blob):
                # same dense weight as the forward's library GEMM: the resident
                # shadow when ILLM_PREFILL_DENSE_GB allows it, else a transient dequant
                from ..ops.gemm import _dense_weight
                w = _dense_weight(blob, ctx.fmt, ctx.n, ctx.k, dt)
            else:
                w = ops.dequantize(blob, ctx.fmt, ctx.n, ctx.k, dtype=dt)
            grad_x = torch.matmul(grad_y.to(w.dtype), w).to(ctx.xdtype)
        return grad_x, None, None, None, None, None


class LowBitLinear(nn.Module):
    """nn.Linear replacement holding a packed low-bit weight."""

    def __init__(self, in_features: int, out_features: int, qtype="sym_int4", bias: bool = True,
                 device=None, dtype=None, mp_group=None, enable_xetla=False, optimize_lm_head=False,
                 act_order=False, enable_scale_search=False):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.qtype = Q.resolve_qtype(qtype)
        fmt = Q.get_format(self.qtype)
        if fmt is None:
            raise ValueError(f"{Q.qtype_name(self.qtype)} is a dense type; use FP16Linear/BF16Linear")
        self.fmt = fmt.fmt
        if in_features % fmt.k_align:
            raise ValueError(f"in_features={in_features} must be a multiple of {fmt.k_align}")
        device = torch.device(device) if device is not None else torch.device("cpu")
        nbytes = _dev_total(self.fmt, out_features, in_features) if device.type == "cuda" else \
            _canon_total(self.fmt, out_features, in_features)
        self.weight = nn.Parameter(torch.zeros(nbytes, dtype=torch.uint8, device=device), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(out_features, dtype=dtype or torch.float32, device=device)) \
            if bias else None
        self.mp_group = mp_group          # row-parallel TP group: all-reduce after the GEMM
        self.optimize_lm_head = optimize_lm_head
        self.act_order = act_order
        self.g_idx_map = None             # GPTQ act-order input permutation
        self.enable_scale_search = enable_scale_search
        self.compute_dtype = None

    # ------------------------------------------------------------ construction
    @classmethod
    @torch.no_grad()
    def from_linear(cls, linear: nn.Module, qtype="sym_int4", device=None, imatrix=None,
                    enable_scale_search=False, mp_group=None, optimize_lm_head=False):
        w = linear.weight.data
        n, k = w.shape
        dev = torch.device(device) if device is not None else w.device
        m = cls(k, n, qtype, bias=getattr(linear, "bias", None) is not None, device="meta",
                mp_group=mp_group, optimize_lm_head=optimize_lm_head, enable_scale_search=enable_scale_search)
        m.load_dense(w, device=dev, imatrix=imatrix)
        if linear.bias is not None:
            m.bias = nn.Parameter(linear.bias.data.detach().to(dev).clone(), requires_grad=False)
        return m

    @torch.no_grad()
    def load_dense(self, w: torch.Tensor, device=None, imatrix=None):
        """Quantize a dense [out, in] weight into this module (on ``device``)."""
        dev = torch.device(device) if device is not None else w.device
        if dev.type == "cuda":
            wq = w.to(dev)
            if wq.dtype not in (torch.bfloat16, torch.float16, torch.float32):
                wq = wq.float()
            blob = ops.quantize(wq, self.fmt, imatrix, self.enable_scale_search)
        else:
            blob = ops.quantize(w.float().cpu(), self.fmt, imatrix, self.enable_scale_search)
        self.weight = nn.Parameter(blob, requires_grad=False)

    @property
    def device_layout(self) -> bool:
        return self.weight.is_cuda

    def dequantize(self, dtype=torch.float32) -> torch.Tensor:
        return ops.dequantize(self.weight, self.fmt, self.out_features, self.in_features, dtype)

    def canonical_blob(self) -> torch.Tensor:
        if self.weight.is_cuda:
            return ops.repack_from_device(self.weight, self.fmt, self.out_features, self.in_features)
        return self.weight.data

    # ------------------------------------------------------------ device moves
    def _apply(self, fn, recurse=True):
        w = self.weight
        if w is not None and w.device.type != "meta":
            probe = fn(torch.empty(0, dtype=torch.uint8, device=w.device))
            tgt = probe.device
            if tgt.type != w.device.type:
                n, k = self.out_features, self.in_features
                if tgt.type == "cuda":
                    new = ops.repack_to_device(w.data.cpu(), self.fmt, n, k).to(tgt)
                else:
                    new = ops.repack_from_device(w.data, self.fmt, n, k)
                self.weight = nn.Parameter(new, requires_grad=False)
                if self.bias is not None:
                    self.bias = nn.Parameter(fn(self.bias.data), requires_grad=self.bias.requires_grad)
                return self
        return super()._apply(fn, recurse)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        # checkpoints always hold the portable canonical layout
        destination[prefix + "weight"] = self.canonical_blob().cpu() if not keep_vars else self.weight
        if self.bias is not None:
            destination[prefix + "bias"] = self.bias if keep_vars else self.bias.detach()

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        key = prefix + "weight"
        if key in state_dict:
            blob = state_dict[key]
            n, k = self.out_features, self.in_features
            if blob.dtype != torch.uint8:
                # a dense checkpoint tensor: quantize it now
                self.load_dense(blob.view(n, k), device=self.weight.device if self.weight.device.type != "meta" else "cpu")
            else:
                blob = blob.reshape(-1)
                tgt = self.weight.device
                if blob.numel() != _canon_total(self.fmt, n, k):
                    error_msgs.append(f"{key}: blob has {blob.numel()} bytes, expected "
                                      f"{_canon_total(self.fmt, n, k)} for {Q.qtype_name(self.qtype)} [{n}, {k}]")
                    return
                if tgt.type == "cuda":
                    new = ops.repack_to_device(blob, self.fmt, n, k).to(tgt)
                else:
                    new = blob.clone()
                self.weight = nn.Parameter(new, requires_grad=False)
        elif strict:
            missing_keys.append(key)
        bkey = prefix + "bias"
        if self.bias is not None:
            if bkey in state_dict:
                b = state_dict[bkey]
                dev = self.bias.device if self.bias.device.type != "meta" else self.weight.device
                self.bias = nn.Parameter(b.detach().to(dev).clone(), requires_grad=False)
            elif strict:
                missing_keys.append(bkey)

    # ------------------------------------------------------------ forward
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.optimize_lm_head and x.dim() == 3 and x.shape[1] > 10 and not self.training:
            # last-token-only lm_head (reference: reshape_lm_head_input, :282-289)
            x = x[:, -1:, :]
        if self.g_idx_map is not None:
            x = x.index_select(-1, self.g_idx_map)
        in_dtype = x.dtype
        if x.is_cuda and x.dtype not in (torch.bfloat16, torch.float16):
            x = x.to(self.compute_dtype or torch.float16)
        bias = self.bias
        if bias is not None and bias.dtype != x.dtype:
            bias = bias.to(x.dtype)
        if self.training and torch.is_grad_enabled() and x.requires_grad:
            y = MatMulLowBit.apply(x, self.weight, self.fmt, self.out_features, self.in_features, self)
            if bias is not None:
                y = y + bias
        else:
            y = ops.lowbit_matmul(x, self.weight, self.fmt, self.out_features, self.in_features,
                                  None if self.mp_group is not None else bias)
        if self.mp_group is not None:
            from ..parallel.comm import all_reduce_inplace
            y = all_reduce_inplace(y, self.mp_group)
            if bias is not None:
                y = y + bias
        return y.to(in_dtype) if y.dtype != in_dtype else y

    def extra_repr(self):
        return (f"in_features={self.in_features}, out_features={self.out_features}, "
                f"qtype={Q.qtype_name(self.qtype)}, bias={self.bias is not None}")


class DenseLinear(nn.Module):
    """fp16/bf16 linear (FP16Linear / BF16Linear equivalent) with optional
    row-parallel all-reduce (reference: low_bit_linear.py:758-948)."""

    def __init__(self, in_features, out_features, bias=True, dtype=torch.float16, device=None, mp_group=None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features, dtype=dtype, device=device),
                                   requires_grad=False)
        self.bias = nn.Parameter(torch.empty(out_features, dtype=dtype, device=device), requires_grad=False) \
            if bias else None
        self.mp_group = mp_group
        self.qtype = Q.BF16 if dtype == torch.bfloat16 else Q.FP16

    @classmethod
    def from_linear(cls, linear, dtype=torch.float16, device=None, mp_group=None):
        m = cls(linear.in_features, linear.out_features, linear.bias is not None, dtype, "meta", mp_group)
        dev = device or linear.weight.device
        m.weight = nn.Parameter(linear.weight.data.to(dev, dtype), requires_grad=False)
        if linear.bias is not None:
            m.bias = nn.Parameter(linear.bias.data.to(dev, dtype), requires_grad=False)
        return m

    def forward(self, x):
        xx = x.to(self.weight.dtype)
        b = None if self.mp_group else self.bias
        if xx.is_cuda and xx.numel() // xx.shape[-1] <= 16 and \
                not (torch.is_grad_enabled() and (xx.requires_grad or self.weight.requires_grad)):
            y = ops.dense_linear(xx, self.weight, b)          # decode: streaming skinny kernel
        else:
            y = F.linear(xx, self.weight, b)
        if self.mp_group is not None:
            from ..parallel.comm import all_reduce_inplace
            y = all_reduce_inplace(y, self.mp_group)
            if self.bias is not None:
                y = y + self.bias
        return y.to(x.dtype)


FP16Linear = DenseLinear


class BF16Linear(DenseLinear):
    def __init__(self, in_features, out_features, bias=True, dtype=torch.bfloat16, device=None, mp_group=None):
        super().__init__(in_features, out_features, bias, torch.bfloat16, device, mp_group)


# ---------------------------------------------------------------- canonical blob surgery
def canon_planes(blob: torch.Tensor, fmt: int, n: int, k: int):
    """split a canonical blob into (codes [n, k*bits/8] u8, scales [n, k/64] f16, mins or None)"""
    from ..ops.reference import canon_sizes, fmt_bits, HAS_MIN
    cb, se = canon_sizes(fmt, n, k)
    b = blob.reshape(-1)
    codes = b[:cb].view(n, k * fmt_bits(fmt) // 8)
    scales = b[cb:cb + 2 * se].view(torch.float16).view(n, k // 64)
    mins = b[cb + 2 * se:cb + 4 * se].view(torch.float16).view(n, k // 64) if fmt in HAS_MIN else None
    return codes, scales, mins


def canon_join(codes, scales, mins=None) -> torch.Tensor:
    parts = [codes.reshape(-1), scales.contiguous().view(torch.uint8).reshape(-1)]
    if mins is not None:
        parts.append(mins.contiguous().view(torch.uint8).reshape(-1))
    return torch.cat(parts)


def lowbit_row_concat(mods, interleave_glu: bool = False) -> "LowBitLinear":
    """Stack the output rows of low-bit linears sharing qtype / in_features
    (merge q/k/v; gate/up with 16-row tile interleave) without re-quantizing."""
    m0 = mods[0]
    k, fmt = m0.in_features, m0.fmt
    assert all(isinstance(m, LowBitLinear) and m.fmt == fmt and m.in_features == k for m in mods)
    planes = [canon_planes(m.canonical_blob().cpu(), fmt, m.out_features, k) for m in mods]
    if interleave_glu:
        from ..models.decoder import interleave_glu_rows
        cat = lambda i: None if planes[0][i] is None else interleave_glu_rows(planes[0][i], planes[1][i])  # noqa: E731
    else:
        cat = lambda i: None if planes[0][i] is None else torch.cat([p[i] for p in planes], 0)  # noqa: E731
    n = sum(m.out_features for m in mods)
    new = LowBitLinear(k, n, m0.qtype, bias=False, device="meta")
    blob = canon_join(cat(0), cat(1), cat(2))
    dev = m0.weight.device
    if dev.type == "cuda":
        blob = ops.repack_to_device(blob, fmt, n, k).to(dev)
    new.weight = nn.Parameter(blob, requires_grad=False)
    if any(m.bias is not None for m in mods) and not interleave_glu:
        new.bias = nn.Parameter(torch.cat([m.bias.data if m.bias is not None else
                                           torch.zeros(m.out_features, device=dev) for m in mods]),
                                requires_grad=False)
    if m0.g_idx_map is not None:
        new.g_idx_map = m0.g_idx_map
    return new


# ---------------------------------------------------------------- k-quants
class _KQMatMul(torch.autograd.Function):
    """y = x W^T with a frozen k-quant W (QLoRA-style base weight): grad_x only"""

    @staticmethod
    def forward(ctx, x, blob, fmt, n, k):
        ctx.fmt, ctx.n, ctx.k = fmt, n, k
        ctx.save_for_backward(blob)
        ctx.xdtype = x.dtype
        return ops.kq_linear(x, blob, fmt, n, k)

    @staticmethod
    def backward(ctx, grad_y):
        (blob,) = ctx.saved_tensors
        gx = None
        if ctx.needs_input_grad[0]:
            dt = grad_y.dtype if grad_y.dtype in (torch.bfloat16, torch.float16) else torch.float32
            w = ops.kq_dequantize(blob, ctx.fmt, ctx.n, ctx.k, dt)
            gx = torch.matmul(grad_y.to(w.dtype), w).to(ctx.xdtype)
        return gx, None, None, None, None


class KQuantLinear(nn.Module):
    """Linear over a GGUF k-quant weight (q4_k / q5_k / q6_k / q2_k).

    Reference: the k-quant qtypes of ``SRC/ggml/quantize.py:28-60`` held by
    ``FP4Params`` / ``LowBitLinear`` (``low_bit_linear.py:106-190``) and the
    gguf_q4k_s/m mixed policies (``transformers/utils.py:286-401``).  The
    GGUF super-block bytes are the storage on the host, on the device and in
    checkpoints (``csrc/common/kquant.h``), so GGUF k-quant tensors are used
    without re-quantization and the bits per weight are the reference's
    (4.5 / 5.5 / 6.5625 / 2.625).  Decode GEMV and dequantize are HIP kernels
    (``csrc/hip/kquant.hip``); the CPU path is the C++ kernel library."""

    def __init__(self, in_features: int, out_features: int, qtype="q4_k", bias: bool = True, device=None,
                 dtype=None, mp_group=None, optimize_lm_head=False):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.qtype = Q.resolve_qtype(qtype)
        f = Q.get_format(self.qtype)
        if f is None or not f.kquant:
            raise ValueError(f"{Q.qtype_name(self.qtype)} is not a k-quant format")
        if in_features % 256:
            raise ValueError(f"k-quant formats need in_features % 256 == 0, got {in_features}")
        self.kq_fmt = f.fmt
        device = torch.device(device) if device is not None else torch.device("cpu")
        self.weight = nn.Parameter(torch.zeros(Q.storage_bytes(self.qtype, out_features, in_features),
                                               dtype=torch.uint8, device=device), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(out_features, dtype=dtype or torch.float32, device=device)) \
            if bias else None
        self.mp_group = mp_group
        self.optimize_lm_head = optimize_lm_head

    @classmethod
    @torch.no_grad()
    def from_linear(cls, linear: nn.Module, qtype="q4_k", device=None, imatrix=None, mp_group=None,
                    optimize_lm_head=False):
        w = linear.weight.data
        dev = torch.device(device) if device is not None else w.device
        m = cls(w.shape[1], w.shape[0], qtype, bias=getattr(linear, "bias", None) is not None, device="meta",
                mp_group=mp_group, optimize_lm_head=optimize_lm_head)
        m.load_dense(w, dev, imatrix)
        if linear.bias is not None:
            m.bias = nn.Parameter(linear.bias.data.detach().to(dev).clone(), requires_grad=False)
        return m

    @torch.no_grad()
    def load_dense(self, w: torch.Tensor, device=None, imatrix=None):
        """quantize a dense [out, in] weight (C++ host quantizer, imatrix-aware)"""
        dev = torch.device(device) if device is not None else w.device
        blob = ops.kq_quantize(w.float().cpu(), self.kq_fmt, imatrix)
        self.weight = nn.Parameter(blob.to(dev), requires_grad=False)

    @classmethod
    def from_blocks(cls, blob: torch.Tensor, qtype, n: int, k: int, device=None, bias=None):
        """wrap GGUF super-block bytes of an [n, k] weight as they are"""
        m = cls(k, n, qtype, bias=bias is not None, device="meta")
        if blob.numel() != Q.storage_bytes(m.qtype, n, k):
            raise ValueError(f"k-quant blob has {blob.numel()} bytes, expected {Q.storage_bytes(m.qtype, n, k)}")
        m.weight = nn.Parameter(blob.reshape(-1).to(torch.uint8).to(device or blob.device), requires_grad=False)
        if bias is not None:
            m.bias = nn.Parameter(bias.detach().to(m.weight.device), requires_grad=False)
        return m

    def dequantize(self, dtype=torch.float32) -> torch.Tensor:
        return ops.kq_dequantize(self.weight, self.kq_fmt, self.out_features, self.in_features, dtype)

    def canonical_blob(self) -> torch.Tensor:
        return self.weight.data

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        key = prefix + "weight"
        if key in state_dict:
            blob = state_dict[key]
            n, k = self.out_features, self.in_features
            dev = self.weight.device if self.weight.device.type != "meta" else torch.device("cpu")
            if blob.dtype != torch.uint8:
                self.load_dense(blob.view(n, k), dev)
            elif blob.numel() != Q.storage_bytes(self.qtype, n, k):
                error_msgs.append(f"{key}: k-quant blob has {blob.numel()} bytes, expected "
                                  f"{Q.storage_bytes(self.qtype, n, k)}")
                return
            else:
                self.weight = nn.Parameter(blob.reshape(-1).to(dev).clone(), requires_grad=False)
        elif strict:
            missing_keys.append(key)
        bkey = prefix + "bias"
        if self.bias is not None:
            if bkey in state_dict:
                dev = self.bias.device if self.bias.device.type != "meta" else self.weight.device
                self.bias = nn.Parameter(state_dict[bkey].detach().to(dev).clone(), requires_grad=False)
            elif strict:
                missing_keys.append(bkey)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.optimize_lm_head and x.dim() == 3 and x.shape[1] > 10 and not self.training:
            x = x[:, -1:, :]
        in_dtype = x.dtype
        if x.is_cuda and x.dtype not in (torch.bfloat16, torch.float16):
            x = x.to(torch.float16)
        if self.training and torch.is_grad_enabled() and x.requires_grad:
            y = _KQMatMul.apply(x, self.weight, self.kq_fmt, self.out_features, self.in_features)
        else:
            y = ops.kq_linear(x, self.weight, self.kq_fmt, self.out_features, self.in_features)
        if self.mp_group is not None:
            from ..parallel.comm import all_reduce_inplace
            y = all_reduce_inplace(y, self.mp_group)
        if self.bias is not None:
            y = y + self.bias.to(y.dtype)
        return y.to(in_dtype) if y.dtype != in_dtype else y

    def extra_repr(self):
        return (f"in_features={self.in_features}, out_features={self.out_features}, "
                f"qtype={Q.qtype_name(self.qtype)}, bias={self.bias is not None}")


class RowConcatLinear(nn.Module):
    """Output rows of several linears (e.g. a merged qkv / gate_up whose
    parts keep different GGUF k-quant types); ``interleave_glu``: 16-row
    tile interleave of (gate, up) -- the layout of a merged gate_up_proj."""

    def __init__(self, parts, interleave_glu: bool = False):
        super().__init__()
        self.parts = nn.ModuleList(parts)
        self.interleave_glu = interleave_glu
        self.in_features = parts[0].in_features
        self.out_features = sum(p.out_features for p in parts)
        self.bias = None
        self.mp_group = None

    def forward(self, x):
        ys = [p(x) for p in self.parts]
        if self.interleave_glu:
            g, u = ys
            I = g.shape[-1]
            return torch.stack([g.reshape(*g.shape[:-1], I // 16, 16), u.reshape(*u.shape[:-1], I // 16, 16)],
                               -2).reshape(*g.shape[:-1], 2 * I)
        return torch.cat(ys, -1)


def kquant_row_concat(mods, interleave_glu: bool = False) -> nn.Module:
    """Merge q/k/v (or gate/up with the 16-row tile interleave) whose parts
    are GGUF k-quant linears: one KQuantLinear over the concatenated block
    rows when the parts share a type (rows are independent block runs), else
    a RowConcatLinear keeping each part's type (gguf_q4k_m: v in q6_k)."""
    if all(isinstance(m, KQuantLinear) for m in mods) and len({m.qtype for m in mods}) == 1 and \
            len({m.in_features for m in mods}) == 1:
        k = mods[0].in_features
        rows = [m.weight.data.view(m.out_features, -1) for m in mods]
        if interleave_glu:
            from ..models.decoder import interleave_glu_rows
            blob = interleave_glu_rows(rows[0], rows[1])
        else:
            blob = torch.cat(rows, 0)
        bias = None
        if any(m.bias is not None for m in mods) and not interleave_glu:
            bias = torch.cat([m.bias.data if m.bias is not None else
                              torch.zeros(m.out_features, dtype=torch.float32) for m in mods])
        return KQuantLinear.from_blocks(blob.reshape(-1), mods[0].qtype, sum(m.out_features for m in mods), k,
                                        bias=bias)
    return RowConcatLinear(mods, interleave_glu)


class TorchFp8Linear(nn.Module):
    """torch_fp8_e4m3 / torch_fp8_e5m2 linear (reference FP8 path:
    ``ggml_convert_qtype`` -> fp8 weight + f32 scale, forward
    ``xe_linear.run_linear_fp8``; SRC/transformers/low_bit_linear.py:110-113,
    168-178, 692-696).  Weight: fp8 codes [out, in] (uint8) + a per-tensor
    scale (``per_channel``: one per output row); forward on the GPU is the
    fp8 GEMV (decode) or per-token e4m3 activations on the block-scaled
    f8f6f4 MFMA GEMM (ops.fp8_linear)."""

    def __init__(self, in_features: int, out_features: int, qtype="torch_fp8_e4m3", bias: bool = True, device=None,
                 mp_group=None, optimize_lm_head: bool = False, per_channel: bool = False):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.qtype = Q.resolve_qtype(qtype)
        self.e5m2 = self.qtype == Q.TORCH_FP8E5
        self.weight = nn.Parameter(torch.empty(out_features, in_features, dtype=torch.uint8, device=device),
                                   requires_grad=False)
        self.w_scale = nn.Parameter(torch.ones(out_features if per_channel else 1, dtype=torch.float32,
                                               device=device), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(out_features, dtype=torch.float32, device=device), requires_grad=False) \
            if bias else None
        self.mp_group = mp_group
        self.optimize_lm_head = optimize_lm_head

    @classmethod
    def from_linear(cls, linear, qtype, device=None, mp_group=None, optimize_lm_head=False, per_channel=False):
        w = linear.weight.data
        m = cls(w.shape[1], w.shape[0], qtype, bias=getattr(linear, "bias", None) is not None, device="meta",
                mp_group=mp_group, optimize_lm_head=optimize_lm_head, per_channel=per_channel)
        dev = device or w.device
        q, s = ops.fp8_quantize_weight(w, m.e5m2, per_channel)
        m.weight = nn.Parameter(q.to(dev), requires_grad=False)
        m.w_scale = nn.Parameter(s.to(dev), requires_grad=False)
        if linear.bias is not None:
            m.bias = nn.Parameter(linear.bias.data.detach().to(dev).clone(), requires_grad=False)
        return m

    def dequantize(self, dtype=torch.float32) -> torch.Tensor:
        f8 = torch.float8_e5m2 if self.e5m2 else torch.float8_e4m3fn
        return (self.weight.view(f8).float() * self.w_scale.float().view(-1, 1)).to(dtype)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.optimize_lm_head and x.dim() == 3 and x.shape[1] > 10 and not self.training:
            x = x[:, -1:, :]
        in_dtype = x.dtype
        if x.is_cuda and x.dtype not in (torch.bfloat16, torch.float16):
            x = x.to(torch.bfloat16)
        if self.training and torch.is_grad_enabled() and x.requires_grad:
            y = F.linear(x, self.dequantize(x.dtype))             # (reference: fp8 training unsupported)
        else:
            bias = self.bias if self.mp_group is None else None
            y = ops.fp8_linear(x, self.weight, self.w_scale, None if bias is None else bias.to(x.dtype), self.e5m2)
        if self.mp_group is not None:
            from ..parallel.comm import all_reduce_inplace
            y = all_reduce_inplace(y, self.mp_group)
            if self.bias is not None:
                y = y + self.bias.to(y.dtype)
        return y.to(in_dtype) if y.dtype != in_dtype else y

    def extra_repr(self):
        return (f"in_features={self.in_features}, out_features={self.out_features}, "
                f"qtype={Q.qtype_name(self.qtype)}, bias={self.bias is not None}")
