"""Importance matrices (llama.cpp ``imatrix.dat``) for weighted quantization.

Reference: ``from_pretrained(imatrix=...)`` (``model.py:333-337``) ->
``SRC/transformers/utils.py`` ``load_imatrix_data`` / ``module_name_process``
and ``ggml_quantize_tensor_with_weights`` (k-quants / IQ formats need it).

File format (llama.cpp): int32 n_entries, then per entry int32 name_len,
name bytes, int32 ncall, int32 nval, float32[nval] (sums of squared
activations per input channel); an optional trailer (last_call, dataset)
is ignored.  Values are divided by ncall.  GGUF tensor names are mapped to
HF module names so ``ggml_convert_low_bit`` can look them up per layer (the
merged ``qkv_proj`` / ``gate_up_proj`` reuse the q / gate entry: same input).
"""
from __future__ import annotations

import re
import struct
from typing import Dict, Optional, Union

import numpy as np
import torch

_MAP = {
    "attn_q": ["self_attn.q_proj", "self_attn.qkv_proj"],
    "attn_k": ["self_attn.k_proj"],
    "attn_v": ["self_attn.v_proj"],
    "attn_qkv": ["self_attn.qkv_proj"],
    "attn_output": ["self_attn.o_proj"],
    "ffn_gate": ["mlp.gate_proj", "mlp.gate_up_proj"],
    "ffn_up": ["mlp.up_proj"],
    "ffn_down": ["mlp.down_proj"],
    "ffn_gate_inp": ["mlp.gate"],
}


def read_imatrix(path: str) -> Dict[str, torch.Tensor]:
    out = {}
    with open(path, "rb") as f:
        (n,) = struct.unpack("<i", f.read(4))
        for _ in range(n):
            (ln,) = struct.unpack("<i", f.read(4))
            name = f.read(ln).decode("utf-8")
            ncall, nval = struct.unpack("<ii", f.read(8))
            vals = np.frombuffer(f.read(4 * nval), dtype=np.float32).copy()
            if ncall > 0:
                vals /= ncall
            out[name] = torch.from_numpy(vals)
    return out


def write_imatrix(path: str, data: Dict[str, torch.Tensor], ncall: int = 1):
    """(for tests / tooling) write a llama.cpp-format imatrix file"""
    with open(path, "wb") as f:
        f.write(struct.pack("<i", len(data)))
        for name, v in data.items():
            b = name.encode()
            arr = (v.float().numpy() * ncall).astype(np.float32)
            f.write(struct.pack("<i", len(b)) + b + struct.pack("<ii", ncall, arr.size) + arr.tobytes())


def gguf_to_hf_name(name: str, prefix: str = "model.layers") -> Optional[list]:
    m = re.match(r"blk\.(\d+)\.([a-z_]+)(\.weight)?$", name)
    if m:
        i, kind = m.group(1), m.group(2)
        return [f"{prefix}.{i}.{t}" for t in _MAP.get(kind, [])] or None
    if name.startswith("output"):
        return ["lm_head"]
    return None


def load_imatrix(imatrix: Union[str, Dict[str, torch.Tensor]], model=None) -> Dict[str, torch.Tensor]:
    """path or {gguf_name: values} -> {hf_module_name: importance [in_features]}"""
    data = read_imatrix(imatrix) if isinstance(imatrix, str) else dict(imatrix)
    out = {}
    for name, v in data.items():
        names = gguf_to_hf_name(name)
        if names is None:
            out[name] = v
            continue
        for n in names:
            out.setdefault(n, v)
    if model is not None:
        # keep only names of linear layers the model has (or will have after merging)
        mods = dict(model.named_modules())
        keep = {}
        for n, v in out.items():
            parent = n.rsplit(".", 1)[0]
            if n in mods or parent in mods:
                keep[n] = v
        out = keep
    return out
