"""``optimize_model()`` -- one-line low-bit optimization of any nn.Module.

Reference: ``SRC/optimize.py`` (``optimize_model`` 199-267, ``load_low_bit``
137-196, ``low_memory_init`` via ``utils/lazy_load_torch.py``).
"""
from __future__ import annotations

import contextlib
import json
import os

import torch
import torch.nn as nn

from .quantize import qtypes as Q
from .transformers.convert import ggml_convert_low_bit
from .transformers.model import _attach, save_low_bit

BIGDL_CONFIG = "bigdl_config.json"


def optimize_model(model: nn.Module, low_bit: str = "sym_int4", optimize_llm: bool = True,
                   modules_to_not_convert=None, cpu_embedding: bool = False, lightweight_bmm: bool = False,
                   device=None, **kwargs) -> nn.Module:
    """Quantize every eligible ``nn.Linear`` of ``model`` to ``low_bit`` and
    install the MI355X forwards for supported LLM architectures.
    ``low_bit=None`` keeps the weights dense and only swaps the forwards."""
    qtype = low_bit if low_bit is not None else "bf16"
    ggml_convert_low_bit(model, qtype, optimize_llm, device, modules_to_not_convert,
                         cpu_embedding=cpu_embedding, mixed_precision=kwargs.get("mixed_precision", False),
                         embedding_qtype=kwargs.get("embedding_qtype"),
                         torch_dtype=kwargs.get("torch_dtype"))
    _attach(model, qtype, {"modules_to_not_convert": modules_to_not_convert})
    if not hasattr(model, "config"):
        # generic module: remember how to rebuild for load_low_bit
        model._bigdl_config = {"bigdl_transformers_low_bit": Q.qtype_name(Q.resolve_qtype(qtype)),
                               "optimize_llm": optimize_llm}
        model.save_low_bit = lambda path: _save_generic(model, path)
    return model


def _save_generic(model, path):
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, BIGDL_CONFIG), "w") as f:
        json.dump(model._bigdl_config, f)
    torch.save(model.state_dict(), os.path.join(path, "model.bin"))


def load_low_bit(model: nn.Module, model_path: str) -> nn.Module:
    """Load a low-bit checkpoint written by ``optimize_model(...).save_low_bit``
    into a freshly built (possibly meta-initialised) module."""
    cfg_path = os.path.join(model_path, BIGDL_CONFIG)
    if os.path.exists(cfg_path):
        cfg = json.load(open(cfg_path))
        qtype = cfg["bigdl_transformers_low_bit"]
        ggml_convert_low_bit(model, qtype, cfg.get("optimize_llm", True), convert_shape_only=True)
        sd = torch.load(os.path.join(model_path, "model.bin"), map_location="cpu", weights_only=True)
    else:
        from safetensors.torch import load_file
        meta = json.load(open(os.path.join(model_path, "illm_low_bit.json")))
        qtype = meta["qtype"]
        ggml_convert_low_bit(model, qtype, meta.get("optimize_model", True), convert_shape_only=True)
        sd = load_file(os.path.join(model_path, "model.safetensors"))
    model.load_state_dict(sd, strict=False, assign=True)
    _attach(model, qtype, {})
    return model


@contextlib.contextmanager
def low_memory_init():
    """Build a module on the meta device (weights materialised later by
    ``load_low_bit``) -- the reference's low_memory_init equivalent."""
    from accelerate import init_empty_weights
    with init_empty_weights():
        yield
