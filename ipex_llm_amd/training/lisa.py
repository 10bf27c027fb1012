"""LISA: layerwise importance sampling -- train a random subset of decoder
layers, re-drawn every ``interval_steps``.

Reference: ``SRC/transformers/lisa.py:23-81`` (DynamicLayerActivationCallback,
with a fixed model-class -> layer-list map).  Here the layer list is found
structurally (the longest ``nn.ModuleList`` of the model), so every
architecture works.
"""
from __future__ import annotations

import numpy as np
import torch.nn as nn


def find_layers(model: nn.Module) -> nn.ModuleList:
    best = None
    for m in model.modules():
        if isinstance(m, nn.ModuleList) and (best is None or len(m) > len(best)):
            best = m
    if best is None:
        raise ValueError("LISA: model has no layer list")
    return best


class LayerActivation:
    def __init__(self, model: nn.Module, n_layers: int, interval_steps: int, seed: int = 0):
        self.layers = find_layers(model)
        self.n_layers, self.interval_steps = n_layers, interval_steps
        self.rng = np.random.default_rng(seed)
        self.active = []

    def switch(self):
        for layer in self.layers:
            for p in layer.parameters():
                p.requires_grad_(False)
        self.active = sorted(self.rng.choice(len(self.layers), self.n_layers, replace=False).tolist())
        for i in self.active:
            for p in self.layers[i].parameters():
                if p.is_floating_point():
                    p.requires_grad_(True)
        return self.active

    def maybe_switch(self, step: int):
        if step % self.interval_steps == 0:
            return self.switch()
        return None


try:
    from transformers import TrainerCallback

    class DynamicLayerActivationCallback(TrainerCallback):
        def __init__(self, n_layers: int, interval_steps: int, model: nn.Module):
            self.act = LayerActivation(model, n_layers, interval_steps)

        def on_step_begin(self, args, state, control, **kwargs):
            self.act.maybe_switch(state.global_step)
            return control
except ImportError:  # pragma: no cover
    pass
