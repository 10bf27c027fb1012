"""Data-parallel fine-tuning over RCCL.

Reference: HF Trainer DDP with ``ddp_backend="ccl"``
(``alpaca_qlora_finetuning.py:156-160, 263-269``).  For LoRA only the
adapter gradients (a few MB) are all-reduced; one bucket covers them all,
so a single RCCL all-reduce per step overlaps with the tail of backward.
"""
from __future__ import annotations

import torch
import torch.nn as nn


def wrap_ddp(model: nn.Module, device_ids=None, bucket_cap_mb: float = 64.0, **kwargs) -> nn.Module:
    from torch.nn.parallel import DistributedDataParallel as DDP
    if device_ids is None and torch.cuda.is_available() and next(model.parameters()).is_cuda:
        device_ids = [torch.cuda.current_device()]
    return DDP(model, device_ids=device_ids, bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True,
               find_unused_parameters=kwargs.pop("find_unused_parameters", False), **kwargs)
