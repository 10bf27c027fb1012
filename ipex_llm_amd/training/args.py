"""TrainingArguments defaults for MI355X (reference qlora.py:268-280 forces
bf16 and whitelists optimizers; DDP over ``ccl`` there, RCCL here)."""
from __future__ import annotations

import logging

from transformers import TrainingArguments as _HFArgs

SUPPORTED_OPTIM = ("adamw_torch", "adamw_hf", "adafactor", "sgd", "adagrad", "rmsprop", "adamw_torch_fused")
log = logging.getLogger("ipex_llm_amd")


class TrainingArguments(_HFArgs):
    def __init__(self, *args, **kwargs):
        kwargs["fp16"] = False
        kwargs["bf16"] = kwargs.get("bf16", True)
        optim = str(kwargs.get("optim", "adamw_torch"))
        if optim not in SUPPORTED_OPTIM and not optim.endswith(tuple(SUPPORTED_OPTIM)):
            log.info("optimizer %s not supported, using adamw_torch", optim)
            kwargs["optim"] = "adamw_torch"
        kwargs.setdefault("ddp_backend", "nccl")     # RCCL on ROCm
        super().__init__(*args, **kwargs)
