"""Reference-compatible QLoRA module (``ipex_llm.transformers.qlora``).

The reference defines its adapter layers here as peft ``LoraLayer``
subclasses patched into ``LoraModel._create_new_module``
(``SRC/transformers/qlora.py:66-143`` LoraLowBitLinear, ``146-211``
LoraBF16Linear, ``214-251`` _create_new_module, ``282-301`` get_peft_model).
This library's adapters live in ``training/lora.py`` (no peft dependency,
the QLoRA linear is one autograd node); this module keeps the reference's
class names and their base-layer contracts:

* ``LoraLowBitLinear`` -- LoRA over a frozen ``LowBitLinear`` (QLoRA /
  QA-LoRA), refuses a dense base;
* ``LoraBF16Linear`` -- LoRA over a dense base held in bf16 (the reference's
  ``bf16`` training mode), refuses a low-bit base.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..training.args import TrainingArguments  # noqa: F401
from ..training.lora import (LoraConfig, LoraLinear, PeftModel,  # noqa: F401
                             cast_lora_weight, get_peft_model, prepare_model_for_kbit_training)
from .low_bit_linear import LowBitLinear


class LoraLowBitLinear(LoraLinear):
    """LoRA adapter over a frozen low-bit base (reference qlora.py:66-143)."""

    def __init__(self, base: nn.Module, r: int = 8, lora_alpha: int = 16, lora_dropout: float = 0.0,
                 qa_lora: bool = False, **kw):
        if not isinstance(base, LowBitLinear):
            raise TypeError(f"LoraLowBitLinear needs a LowBitLinear base, got {type(base).__name__}")
        super().__init__(base, r, lora_alpha, lora_dropout, qa_lora=qa_lora, **kw)


class LoraBF16Linear(LoraLinear):
    """LoRA adapter over a dense base cast to bf16 (reference qlora.py:146-211)."""

    def __init__(self, base: nn.Module, r: int = 8, lora_alpha: int = 16, lora_dropout: float = 0.0, **kw):
        if isinstance(base, LowBitLinear):
            raise TypeError("LoraBF16Linear needs a dense base; use LoraLowBitLinear for low-bit weights")
        base = base.to(torch.bfloat16)
        super().__init__(base, r, lora_alpha, lora_dropout, dtype=torch.bfloat16, **kw)
