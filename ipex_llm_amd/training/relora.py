"""ReLoRA: periodic merge-and-restart of LoRA adapters on a low-bit base.

Reference: ``SRC/transformers/relora.py`` -- ``ReLoRACallback`` (149-283:
every ``relora_steps`` merge the adapters into the base weights, re-init
them and reset optimizer state), ``ReLoRAScheduler`` (286-316: jagged
cosine with a short re-warmup after each restart), ``ReLoRATrainer``
(64-108).  Merging into a low-bit base = dequantize, add B@A*s, re-quantize
(on the GPU this is the device quantize kernel, milliseconds per layer).

Merged full-weight checkpoints (``merge_and_save`` / ``load_weight_checkpoint``,
reference relora.py:383-471): at each restart the adapters are merged into the
FULL-precision base read from the previous full-weight save (the original
checkpoint at the first restart), the merged weights are written as fp16
safetensors shards with the source's shard layout, and the low-bit base is
re-quantized from exactly those saved values -- the base never accumulates
re-quantization error across restarts, and a resumed run that loads the last
save (``load_weight_checkpoint``) continues on the same base as the
uninterrupted one.
"""
from __future__ import annotations

import glob
import json
import math
import os
import shutil
from typing import Dict, Iterable, Optional

import torch
from torch.optim.lr_scheduler import LambdaLR

from ..transformers.low_bit_linear import LowBitLinear
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


def find_lora_modules(model) -> Dict[str, LoraLinear]:
    """name -> adapter wrapper, named as the base model's own modules (the
    checkpoint keys are ``name + ".weight"``), for a PeftModel or a bare model"""
    root = getattr(model, "base_model", model)
    return {n: m for n, m in root.named_modules() if isinstance(m, LoraLinear)}


def sharded_paths(path: str, module_names: Iterable[str]) -> Dict[str, str]:
    """tensor key -> shard file of a HF checkpoint directory (index json, or
    the single ``model.safetensors`` / ``pytorch_model.bin``)"""
    for name in ("model.safetensors", "pytorch_model.bin"):
        idx = os.path.join(path, name + ".index.json")
        if os.path.exists(idx):
            with open(idx, encoding="utf-8") as f:
                return dict(json.load(f)["weight_map"])
        if os.path.exists(os.path.join(path, name)):
            return {m + ".weight": name for m in module_names}
    raise FileNotFoundError(f"no model.safetensors / pytorch_model.bin (or index) under {path}")


def _load_shard(path: str) -> Dict[str, torch.Tensor]:
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path)
    sd = torch.load(path, map_location="cpu", weights_only=True)   # never unpickles code
    return sd.get("state_dict", sd) if isinstance(sd, dict) else sd


def lora_delta_weight(layer: LoraLinear, device=None) -> torch.Tensor:
    """B @ A * scaling as a dense [out, in] f32 update"""
    d = layer.delta_weight()
    return d.to(device) if device is not None else d


@torch.no_grad()
def update_weights(target: LoraLinear, new_weight: torch.Tensor, reinit: bool, device=None):
    """replace the base weight of ``target`` (re-quantized for a low-bit base);
    ``reinit`` restarts the adapter (A random, B = 0)"""
    if reinit:
        target.reset_lora_parameters()
    base = target.base_layer
    dev = device if device is not None else base.weight.device
    if isinstance(base, LowBitLinear) or hasattr(base, "load_dense"):
        base.load_dense(new_weight.float(), device=dev)
    else:
        base.weight.data.copy_(new_weight.to(base.weight.device, base.weight.dtype))
    target.merged = False


@torch.no_grad()
def merge_and_save(model, model_src: str, model_dst: str, reinit: bool = False, cpu_offload: bool = False,
                   actually_save: bool = True, save_dtype=torch.float16) -> Dict[str, str]:
    """merge every adapter into the full-precision weights of ``model_src``
    and write them (with every other tensor of the shard) to ``model_dst`` in
    the source's shard layout; the low-bit bases are re-quantized from the
    saved (``save_dtype``-rounded) merged values.  Returns key -> shard of the
    output.  ``actually_save=False`` (non-main DDP ranks): update only."""
    modules = find_lora_modules(model)
    os.makedirs(model_dst, exist_ok=True)
    shard_of = sharded_paths(model_src, modules.keys())
    out_map: Dict[str, str] = {}
    shards = sorted(set(shard_of[k + ".weight"] for k in modules if k + ".weight" in shard_of)
                    | (set(shard_of.values()) if actually_save else set()))
    for shard in shards:
        tensors = _load_shard(os.path.join(model_src, shard))
        out: Dict[str, torch.Tensor] = {}
        for name, target in modules.items():
            key = name + ".weight"
            if shard_of.get(key) != shard or key not in tensors:
                continue
            dev = "cpu" if cpu_offload else target.lora_A.weight.device
            merged = (tensors[key].float().to(dev) + lora_delta_weight(target, dev)).to(save_dtype)
            out[key] = merged.cpu().contiguous()
            update_weights(target, merged.float(), reinit=reinit)
        if actually_save:
            name = shard
            if name.startswith("pytorch_model"):
                name = "model" + name[len("pytorch_model"):-len(".bin")] + ".safetensors"
            for k, v in tensors.items():
                if k not in out:
                    out[k] = (v.to(save_dtype) if v.is_floating_point() else v).contiguous()
                out_map[k] = name
            from safetensors.torch import save_file
            save_file(out, os.path.join(model_dst, name), metadata={"format": "pt"})
    if actually_save:
        if len(set(out_map.values())) > 1:
            with open(os.path.join(model_dst, "model.safetensors.index.json"), "w", encoding="utf-8") as f:
                json.dump({"metadata": {}, "weight_map": out_map}, f)
        for extra in ("config.json", "generation_config.json"):
            src = os.path.join(model_src, extra)
            if os.path.exists(src) and not os.path.exists(os.path.join(model_dst, extra)):
                shutil.copy(src, os.path.join(model_dst, extra))
    return out_map


@torch.no_grad()
def load_weight_checkpoint(model, checkpoint_path: str) -> int:
    """resume: load the merged full weights of a ``merge_and_save`` directory
    into the adapters' base layers (adapters untouched); returns the count"""
    modules = find_lora_modules(model)
    shard_of = sharded_paths(checkpoint_path, modules.keys())
    n = 0
    for shard in sorted(set(shard_of[k + ".weight"] for k in modules if k + ".weight" in shard_of)):
        tensors = _load_shard(os.path.join(checkpoint_path, shard))
        for name, target in modules.items():
            key = name + ".weight"
            if shard_of.get(key) == shard and key in tensors:
                update_weights(target, tensors[key].float(), reinit=False)
                n += 1
    return n


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
        """every ``relora_steps``: merge + restart.  With ``base_model`` (a local
        full-precision checkpoint) the merge goes through ``merge_and_save``
        into ``<output_dir>/checkpoint-<step>/relora`` (reference relora.py:149-283),
        a resume loads the last such save (``resume_from_checkpoint``) and the
        end of training writes the final merged weights to ``output_dir``;
        without it the adapters merge into the in-memory low-bit base"""

        def __init__(self, relora_steps: int = 150, reset_ratio: float = 1.0, base_model: Optional[str] = None,
                     resume_from_checkpoint: Optional[str] = None, relora_cpu_offload: bool = False):
            self.relora_steps, self.reset_ratio = relora_steps, reset_ratio
            self.restarts = 0
            self.last_full_model = base_model
            self.resume_from_checkpoint = resume_from_checkpoint
            self.cpu_offload = relora_cpu_offload
            if base_model is not None and not os.path.isdir(base_model):
                raise ValueError("ReLoRA base_model must be a local checkpoint directory")

        @staticmethod
        def _main(args) -> bool:
            return getattr(args, "process_index", 0) == 0

        def on_train_begin(self, args, state, control, model=None, **kwargs):
            if self.resume_from_checkpoint:
                path = os.path.join(self.resume_from_checkpoint, "relora")
                if os.path.isdir(path):
                    load_weight_checkpoint(model, path)
                    self.last_full_model = path
            return control

        def on_step_begin(self, args, state, control, model=None, optimizer=None, **kwargs):
            if state.global_step > 0 and self.relora_steps and state.global_step % self.relora_steps == 0:
                if self.last_full_model is not None:
                    dst = os.path.join(args.output_dir, f"checkpoint-{state.global_step}", "relora")
                    merge_and_save(model, self.last_full_model, dst, reinit=True, cpu_offload=self.cpu_offload,
                                   actually_save=self._main(args))
                    if optimizer is not None:
                        reset_optimizer(optimizer, [p for m in find_lora_modules(model).values()
                                                    for p in (m.lora_A.weight, m.lora_B.weight)], self.reset_ratio)
                    self.last_full_model = dst
                else:
                    relora_restart(model, optimizer, self.reset_ratio)
                self.restarts += 1
            return control

        def on_save(self, args, state, control, model=None, **kwargs):
            # keep the newest full-weight save inside the newest checkpoint folder
            dst = os.path.join(args.output_dir, f"checkpoint-{state.global_step}", "relora")
            if (self.last_full_model is not None and self._main(args) and state.global_step >= self.relora_steps
                    and state.global_step % self.relora_steps != 0 and self.last_full_model != dst):
                os.makedirs(dst, exist_ok=True)
                for f in glob.glob(os.path.join(self.last_full_model, "model*.safetensors")) + \
                        glob.glob(os.path.join(self.last_full_model, "model*.index.json")) + \
                        glob.glob(os.path.join(self.last_full_model, "config.json")):
                    shutil.copy(f, dst)
                self.last_full_model = dst
            return control

        def on_log(self, args, state, control, logs=None, **kwargs):
            if logs is not None:
                logs["num_lora_restarts"] = self.restarts
            return control

        def on_train_end(self, args, state, control, model=None, **kwargs):
            if self.last_full_model is not None:
                merge_and_save(model, self.last_full_model, args.output_dir, reinit=False,
                               cpu_offload=self.cpu_offload, actually_save=self._main(args))
            return control

    class ReLoRATrainer(Trainer):
        def __init__(self, *args, relora_steps: int = 150, relora_warmup_steps: int = 10, reset_ratio: float = 1.0,
                     base_model: Optional[str] = None, resume_from_checkpoint: Optional[str] = None,
                     relora_cpu_offload: bool = False, **kwargs):
            cb = ReLoRACallback(relora_steps, reset_ratio, base_model, resume_from_checkpoint, relora_cpu_offload)
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
