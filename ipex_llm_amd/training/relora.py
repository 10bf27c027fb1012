"""ReLoRA: periodic merge-and-restart of LoRA adapters on a low-bit base.

Reference: ``SRC/transformers/relora.py`` -- ``ReLoRACallback`` (149-283:
every ``relora_steps`` merge the adapters into the base weights, re-init
them and reset optimizer state), ``ReLoRAScheduler`` (286-316: jagged
cosine with a short re-warmup after each restart), ``ReLoRATrainer``
(64-108).  Merging into a low-bit base = dequantize, add B@A*s, re-quantize
(on the GPU this is the device quantize kernel, milliseconds per layer).
"""
from __future__ import annotations

import math

import torch
from torch.optim.lr_scheduler import LambdaLR

from .lora import LoraLinear


def reset_optimizer(optimizer: torch.optim.Optimizer, params=None, reset_ratio: float = 1.0):
    """Zero (a random ``reset_ratio`` fraction of) the moments of ``params``
    (reference prunes the Adam state of the restarted adapters)."""
    targets = set(id(p) for p in params) if params is not None else None
    for group in optimizer.param_groups:
        for p in group["params"]:
            if targets is not None and id(p) not in targets:
                continue
            st = optimizer.state.get(p)
            if not st:
                continue
            for k in ("exp_avg", "exp_avg_sq"):
                if k in st:
                    if reset_ratio >= 1.0:
                        st[k].zero_()
                    else:
                        st[k].mul_((torch.rand_like(st[k], dtype=torch.float32) > reset_ratio).to(st[k].dtype))


@torch.no_grad()
def relora_restart(model, optimizer=None, reset_ratio: float = 1.0):
    """merge every adapter into its base weight and restart it"""
    mods = [m for m in model.modules() if isinstance(m, LoraLinear)]
    for m in mods:
        m.merge()
        m.merged = False
        m.reset_lora_parameters()
    if optimizer is not None:
        params = [p for m in mods for p in (m.lora_A.weight, m.lora_B.weight)]
        reset_optimizer(optimizer, params, reset_ratio)
    return len(mods)


def relora_lr_lambda(total_steps: int, relora_steps: int, warmup_steps: int, restart_warmup_steps: int,
                     min_lr_ratio: float = 0.1):
    """jagged cosine: global cosine decay x a linear re-warmup after each restart"""
    def f(step: int) -> float:
        if step < warmup_steps:
            return step / max(1, warmup_steps)
        progress = (step - warmup_steps) / max(1, total_steps - warmup_steps)
        cos = min_lr_ratio + (1 - min_lr_ratio) * 0.5 * (1 + math.cos(math.pi * min(1.0, progress)))
        since = step % relora_steps if relora_steps else step
        if step >= relora_steps and since < restart_warmup_steps:
            cos *= (since + 1) / restart_warmup_steps
        return cos
    return f


def ReLoRAScheduler(optimizer, total_steps: int, relora_steps: int, warmup_steps: int = 0,
                    restart_warmup_steps: int = 10, min_lr_ratio: float = 0.1):
    return LambdaLR(optimizer, relora_lr_lambda(total_steps, relora_steps, warmup_steps, restart_warmup_steps,
                                                min_lr_ratio))


try:
    from transformers import Trainer, TrainerCallback

    class ReLoRACallback(TrainerCallback):
        def __init__(self, relora_steps: int = 150, reset_ratio: float = 1.0):
            self.relora_steps, self.reset_ratio = relora_steps, reset_ratio
            self.restarts = 0

        def on_step_begin(self, args, state, control, model=None, optimizer=None, **kwargs):
            if state.global_step > 0 and self.relora_steps and state.global_step % self.relora_steps == 0:
                relora_restart(model, optimizer, self.reset_ratio)
                self.restarts += 1
            return control

    class ReLoRATrainer(Trainer):
        def __init__(self, *args, relora_steps: int = 150, relora_warmup_steps: int = 10, reset_ratio: float = 1.0,
                     **kwargs):
            cb = ReLoRACallback(relora_steps, reset_ratio)
            kwargs["callbacks"] = list(kwargs.get("callbacks") or []) + [cb]
            super().__init__(*args, **kwargs)
            self.relora_steps, self.relora_warmup_steps = relora_steps, relora_warmup_steps

        def create_scheduler(self, num_training_steps: int, optimizer=None):
            optimizer = optimizer or self.optimizer
            if self.lr_scheduler is None:
                self.lr_scheduler = ReLoRAScheduler(optimizer, num_training_steps, self.relora_steps,
                                                    self.args.get_warmup_steps(num_training_steps),
                                                    self.relora_warmup_steps)
            return self.lr_scheduler
except ImportError:  # pragma: no cover
    pass
