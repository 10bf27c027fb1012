"""Load GPTQ / AWQ 4-bit checkpoints straight into asym_int4 low-bit layers.

Reference: ``SRC/transformers/convert.py:301-456`` (``convert_gptq`` /
``convert_vllm_awq_or_gptq``: unpack ``qweight``/``qzeros``/``scales``, sort
by ``g_idx`` for act-order, emit ggml q4_1 blocks with d = scale,
m = -zero * scale) and ``model.py`` (GPTQ/AWQ checkpoints load as
asym_int4).  ``optimum`` / ``auto-gptq`` / ``autoawq`` are not needed: the
safetensors are read directly.

Exactness: for group sizes that are multiples of 64 the conversion is exact
up to the fp16 rounding of m = -z*s (our asym block is 64 wide; a 128-group
maps to two blocks with equal scale/min).  Smaller groups are dequantized
and re-quantized.
"""
from __future__ import annotations

import glob
import json
import os
from typing import Dict, Optional

import torch
import torch.nn as nn

from . import ops
from .quantize import qtypes as Q
from .transformers.low_bit_linear import LowBitLinear, canon_join

AWQ_ORDER = [0, 2, 4, 6, 1, 3, 5, 7]


def _unpack_cols(x: torch.Tensor, order=None) -> torch.Tensor:
    """int32 [R, C/8] packed along columns -> int [R, C]"""
    shifts = torch.arange(8, dtype=torch.int32) * 4
    v = (x.unsqueeze(-1) >> shifts) & 0xF                       # [R, C/8, 8] nibble i
    if order is not None:
        inv = [0] * 8
        for i, col in enumerate(order):
            inv[col] = i                                        # column j lives in nibble inv[j]
        v = v[..., inv]
    return v.reshape(x.shape[0], -1)


def _unpack_rows(x: torch.Tensor) -> torch.Tensor:
    """int32 [K/8, N] packed along rows (GPTQ qweight) -> int [K, N]"""
    shifts = torch.arange(8, dtype=torch.int32) * 4
    v = (x.unsqueeze(1) >> shifts[None, :, None]) & 0xF          # [K/8, 8, N]
    return v.reshape(-1, x.shape[1])


def gptq_to_dense_parts(qweight, qzeros, scales, g_idx=None, method: str = "gptq", zero_offset: int = 1):
    """-> (q [N, K] int codes, zeros [N, G], scales [N, G] f32, g_idx [K] or None)"""
    if method == "awq":
        q = _unpack_cols(qweight.int(), AWQ_ORDER).t().contiguous()        # [K, N] -> [N, K]
        z = _unpack_cols(qzeros.int(), AWQ_ORDER).t().contiguous()         # [N, G]
        zero_offset = 0
    else:
        q = _unpack_rows(qweight.int()).t().contiguous()                   # [N, K]
        z = _unpack_cols(qzeros.int()).t().contiguous() + zero_offset      # GPTQ v1 stores zero - 1
    s = scales.float().t().contiguous()                                     # [N, G]
    return q, z, s, g_idx


def gptq_to_lowbit(qweight, qzeros, scales, g_idx=None, bias=None, method: str = "gptq", group_size: int = 128,
                   device=None, zero_offset: int = 1) -> LowBitLinear:
    q, z, s, g_idx = gptq_to_dense_parts(qweight, qzeros, scales, g_idx, method, zero_offset)
    N, K = q.shape
    perm = None
    if g_idx is not None:
        g_idx = g_idx.long()
        default = torch.arange(K) // group_size
        if not torch.equal(g_idx, default):
            perm = torch.argsort(g_idx, stable=True)                       # act-order: sort input channels
            q = q[:, perm]
        gcol = g_idx[perm] if perm is not None else g_idx
    else:
        gcol = torch.arange(K) // group_size
    fmt = Q.get_format(Q.ASYM_INT4).fmt
    blocks = torch.arange(0, K, 64)
    # every 64-block must sit inside one group for an exact conversion
    exact = K % 64 == 0 and bool((gcol[blocks] == gcol[blocks + 63]).all())
    m = LowBitLinear(K, N, Q.ASYM_INT4, bias=bias is not None, device="meta")
    if exact:
        gb = gcol[blocks]                                                   # group of each 64-block
        d = s[:, gb]                                                        # [N, K/64]
        mn = -(z[:, gb].float() * d)
        codes = q.to(torch.uint8).view(N, K // 64, 2, 32)
        packed = (codes[:, :, 0, :] | (codes[:, :, 1, :] << 4)).reshape(N, K // 2)
        blob = canon_join(packed.contiguous(), d.to(torch.float16), mn.to(torch.float16))
    else:
        w = (q.float() - z[:, gcol].float()) * s[:, gcol]
        blob = ops.quantize(w, fmt)
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if dev.type == "cuda":
        blob = ops.repack_to_device(blob, fmt, N, K).to(dev)
    m.weight = nn.Parameter(blob, requires_grad=False)
    if bias is not None:
        m.bias = nn.Parameter(bias.detach().to(dev), requires_grad=False)
    if perm is not None:
        m.g_idx_map = perm.to(dev)
        m.act_order = True
    return m


def _read_state_dict(path: str) -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file
    files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
    if files:
        sd = {}
        for f in files:
            sd.update(load_file(f))
        return sd
    bins = sorted(glob.glob(os.path.join(path, "pytorch_model*.bin")))
    sd = {}
    for f in bins:
        sd.update(torch.load(f, map_location="cpu", weights_only=True))
    return sd


def load_gptq_model(hf_cls, path: str, prequant, torch_dtype="auto", **kwargs):
    """Build ``hf_cls`` from ``path`` with every GPTQ/AWQ-packed linear
    converted to an asym_int4 :class:`LowBitLinear` (reference model.py +
    convert.py:382-456)."""
    from accelerate import init_empty_weights
    from transformers import AutoConfig
    method, qcfg = prequant
    bits = int(qcfg.get("bits", qcfg.get("w_bit", 4)))
    if bits != 4:
        raise ValueError(f"{method} with {bits} bits is not supported (4-bit only, like the reference)")
    group = int(qcfg.get("group_size", qcfg.get("q_group_size", 128)))
    config = AutoConfig.from_pretrained(path, trust_remote_code=kwargs.get("trust_remote_code", False))
    if hasattr(config, "quantization_config"):
        delattr(config, "quantization_config")
    dt = torch.float16 if torch_dtype in (None, "auto") else torch_dtype
    with init_empty_weights():
        model = hf_cls.from_config(config, torch_dtype=dt)
    sd = _read_state_dict(path)
    prefixes = sorted({k[:-len(".qweight")] for k in sd if k.endswith(".qweight")})
    for pre in prefixes:
        parent_name, child = pre.rsplit(".", 1)
        parent = model.get_submodule(parent_name)
        lin = gptq_to_lowbit(sd.pop(pre + ".qweight"), sd.pop(pre + ".qzeros"), sd.pop(pre + ".scales"),
                             sd.pop(pre + ".g_idx", None), sd.pop(pre + ".bias", None), method, group)
        setattr(parent, child, lin)
    missing = [k for k in model.state_dict() if k not in sd and not any(k.startswith(p + ".") for p in prefixes)]
    model.load_state_dict({k: v.to(dt) if v.is_floating_point() else v for k, v in sd.items()}, strict=False,
                          assign=True)
    if getattr(config, "tie_word_embeddings", False) and hasattr(model, "tie_weights"):
        model.tie_weights()
    from .transformers.model import _reinit_meta_buffers
    _reinit_meta_buffers(model, config)
    still_meta = [n for n, p in model.named_parameters() if p.device.type == "meta"]
    if still_meta:
        raise RuntimeError(f"{method} checkpoint is missing tensors: {still_meta[:5]}")
    model._illm_prequant = method
    return model.eval()
