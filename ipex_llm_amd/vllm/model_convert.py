"""vLLM integration: low-bit linears inside a vLLM model and a load-model
hook for vLLM's GPU model runner (ROCm builds of vLLM use the same runner).

Reference: ``SRC/vllm/xpu/model_convert.py:36-205`` -- ``_ipex_llm_convert``
monkey-patches the runner's ``load_model`` so vLLM loads the model, then
``optimize_model(low_bit)`` swaps its ``*ParallelLinear`` layers for low-bit
ones (which return vLLM's ``(output, output_bias)`` pair), optionally
``save_low_bit`` per TP rank; ``padding_mlp`` pads the intermediate size for
the XPU kernels; ``low_bit_linear.py:758-948`` holds the vLLM-signature
linear wrappers.

MI355X design: the weights are already sharded and resident on the GPU when
vLLM's loader returns, so each shard is quantized *on device* straight into
the MFMA tile layout (no CPU round trip, no padding: the kernels handle any
K that is a multiple of the format's block).  Row-parallel layers keep vLLM's
semantics -- partial GEMM, all-reduce over the TP group (RCCL, or the one-shot
xGMI all-reduce for decode-size messages), bias added once after it.
vLLM itself is optional: :func:`convert_vllm_linears` works on any module
tree whose layers carry vLLM's attribute names.
"""
from __future__ import annotations

import os
import types
from typing import Iterable, Optional

import torch
import torch.nn as nn

from ..parallel.comm import all_gather_last_dim
from ..quantize import qtypes as Q
from ..transformers.low_bit_linear import LowBitLinear

COLUMN_KINDS = ("ColumnParallelLinear", "MergedColumnParallelLinear", "QKVParallelLinear")
ROW_KINDS = ("RowParallelLinear",)
REPLICATED_KINDS = ("ReplicatedLinear",)


class VLLMLowBitLinear(nn.Module):
    """Low-bit replacement for a vLLM parallel linear: ``forward`` returns
    ``(output, output_bias)`` like the layer it replaces."""

    def __init__(self, inner: LowBitLinear, kind: str, gather_output: bool = False, skip_bias_add: bool = False,
                 out_bias: Optional[torch.Tensor] = None, tp_group=None):
        super().__init__()
        self.inner, self.kind = inner, kind
        self.gather_output, self.skip_bias_add = gather_output, skip_bias_add
        self.out_bias = nn.Parameter(out_bias, requires_grad=False) if out_bias is not None else None
        self.tp_group = tp_group
        self.input_size, self.output_size = inner.in_features, inner.out_features

    @property
    def weight(self):
        return self.inner.weight

    def forward(self, x: torch.Tensor):
        y = self.inner(x)
        if self.gather_output:
            y = all_gather_last_dim(y, self.tp_group)
        return y, (self.out_bias if self.skip_bias_add else None)


def _tp_world(group) -> int:
    from ..parallel.comm import get_world_size
    return get_world_size(group)


def _convert_one(child: nn.Module, kind: str, qtype: int, tp_group):
    w = getattr(child, "weight", None)
    if not isinstance(w, torch.Tensor) or w.dim() != 2 or w.is_meta:
        return None
    fmt = Q.get_format(qtype)
    if fmt is not None and w.shape[1] % fmt.k_align:
        return None                                   # K not a multiple of the block: keep dense
    bias = getattr(child, "bias", None)
    skip = bool(getattr(child, "skip_bias_add", False))
    inner_bias = None if skip else bias
    row = kind in ROW_KINDS
    mp = tp_group if (row and getattr(child, "reduce_results", True) and _tp_world(tp_group) > 1) else None
    lin = types.SimpleNamespace(weight=w, bias=inner_bias)
    inner = LowBitLinear.from_linear(lin, qtype, device=w.device, mp_group=mp)
    gather = bool(getattr(child, "gather_output", False)) and kind in COLUMN_KINDS
    return VLLMLowBitLinear(inner, kind, gather, skip, bias.data if (skip and bias is not None) else None, tp_group)


def convert_vllm_linears(model: nn.Module, low_bit: str = "sym_int4",
                         modules_to_not_convert: Optional[Iterable[str]] = None, tp_group=None) -> int:
    """Swap every vLLM ``*ParallelLinear`` / ``ReplicatedLinear`` (duck-typed
    by class name) for :class:`VLLMLowBitLinear`, in place.  Returns the
    number of layers converted."""
    qtype = Q.resolve_qtype(low_bit)
    if Q.is_dense(qtype):
        return 0                                      # vLLM's own fp16/bf16 layers already are dense
    skip = set(modules_to_not_convert or [])
    n = 0

    def walk(mod: nn.Module, prefix: str):
        nonlocal n
        for name, child in list(mod.named_children()):
            full = f"{prefix}.{name}" if prefix else name
            if any(s == name or s in full for s in skip):
                continue
            kind = type(child).__name__
            if kind in COLUMN_KINDS + ROW_KINDS + REPLICATED_KINDS:
                new = _convert_one(child, kind, qtype, tp_group)
                if new is not None:
                    setattr(mod, name, new)
                    n += 1
                    continue
            walk(child, full)

    with torch.no_grad():
        walk(model, "")
    return n


def get_load_function(low_bit: str, modules_to_not_convert=None):
    """Replacement for vLLM's ``ModelRunner.load_model``: run vLLM's own
    loader, then quantize the loaded shards on device.  ``IPEX_LLM_LOW_BIT_SAVE_PATH``
    (per-rank subdirectory) writes the converted weights like the
    reference's ``low_bit_save_path``."""

    def load_model(self, *args, **kwargs):
        load_model._orig(self, *args, **kwargs)
        tp_group = None
        try:
            from vllm.distributed import get_tp_group
            tp_group = get_tp_group().device_group
        except Exception:      # single GPU / older vLLM layouts
            tp_group = None
        convert_vllm_linears(self.model, low_bit, modules_to_not_convert, tp_group)
        save = os.environ.get("IPEX_LLM_LOW_BIT_SAVE_PATH")
        if save:
            from safetensors.torch import save_file
            rank = os.environ.get("LOCAL_RANK", "0")
            os.makedirs(os.path.join(save, rank), exist_ok=True)
            save_file({k: v.detach().cpu().contiguous() for k, v in self.model.state_dict().items()},
                      os.path.join(save, rank, "model.safetensors"))

    return load_model


def patch_vllm(low_bit: str = "sym_int4", modules_to_not_convert=None):
    """Monkey-patch vLLM's GPU model runner(s) so every model vLLM loads runs
    on low-bit MI355X kernels (reference ``_ipex_llm_convert``)."""
    try:
        import importlib
        runners = []
        for mod, cls in (("vllm.v1.worker.gpu_model_runner", "GPUModelRunner"),
                         ("vllm.worker.model_runner", "ModelRunner")):
            try:
                runners.append(getattr(importlib.import_module(mod), cls))
            except (ImportError, AttributeError):
                continue
    except ImportError as e:                          # pragma: no cover
        raise ImportError("vLLM is not installed") from e
    if not runners:
        raise ImportError("vLLM is not installed (no GPU model runner found)")
    for r in runners:
        if getattr(r.load_model, "_illm_patched", False):
            continue
        fn = get_load_function(low_bit, modules_to_not_convert)
        fn._orig = r.load_model
        fn._illm_patched = True
        r.load_model = fn
    return runners
