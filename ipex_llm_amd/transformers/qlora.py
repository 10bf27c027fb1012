"""Reference-compatible import path (``ipex_llm.transformers.qlora``)."""
from ..training.lora import (LoraConfig, LoraLinear as LoraLowBitLinear, PeftModel,  # noqa: F401
                             cast_lora_weight, get_peft_model, prepare_model_for_kbit_training)
from ..training.args import TrainingArguments  # noqa: F401
