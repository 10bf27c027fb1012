"""Fine-tuning: LoRA / QLoRA / QA-LoRA / ReLoRA / LISA on low-bit bases,
fused AdamW, DDP helpers."""
from .lora import (LoraConfig, LoraLinear, PeftModel, cast_lora_weight, get_peft_model,  # noqa: F401
                   prepare_model_for_kbit_training)
from .optim import FusedAdamW  # noqa: F401
from .relora import (ReLoRAScheduler, find_lora_modules, load_weight_checkpoint, merge_and_save,  # noqa: F401
                     relora_restart, reset_optimizer)
from .lisa import LayerActivation, find_layers  # noqa: F401
from .ddp import GradBucketSync, wrap_ddp  # noqa: F401
