"""HF-facing projection views over merged weights.

``_optimize_pre`` (convert.py) merges q/k/v into ``qkv_proj`` and gate/up
into a 16-row tile-interleaved ``gate_up_proj`` for the native decoder (the
reference's ``merge_qkv`` / ``fuse_mlp_base`` rewrites,
``SRC/transformers/models/common.py:23-143``).  When a model of a native
architecture turns out to be a variant the native decoder cannot run, its own
HF forward must keep working: these views give it back ``q_proj`` /
``k_proj`` / ``v_proj`` / ``gate_proj`` / ``up_proj`` (the merged GEMM runs
once per input tensor; each view returns its columns).
"""
from __future__ import annotations

import torch
import torch.nn as nn


class ProjView(nn.Module):
    def __init__(self, owner: nn.Module, merged: str, cols, last: bool):
        super().__init__()
        object.__setattr__(self, "_owner", owner)      # not a submodule: no cycle, no extra state
        self.merged, self.last = merged, last
        self.register_buffer("cols", torch.as_tensor(cols, dtype=torch.long), persistent=False)
        c0, c1 = int(cols[0]), int(cols[-1]) + 1
        self._range = (c0, c1) if c1 - c0 == len(cols) else None

    def forward(self, x):
        o = self._owner
        memo = o.__dict__.get("_illm_view_memo")
        if memo is None or memo[0] is not x:
            memo = (x, getattr(o, self.merged)(x))
            o.__dict__["_illm_view_memo"] = memo
        y = memo[1]
        if self.last:
            o.__dict__["_illm_view_memo"] = None
        if self._range is not None:
            return y[..., self._range[0]:self._range[1]]
        return y.index_select(-1, self.cols.to(y.device))


class FusedGLUView(nn.Module):
    """phi3-style fused ``gate_up_proj`` (interleaved for the GLU GEMV):
    restores the HF [gate; up] output order."""

    def __init__(self, inner: nn.Module, perm):
        super().__init__()
        self.inner = inner
        self.register_buffer("perm", torch.as_tensor(perm, dtype=torch.long), persistent=False)

    def forward(self, x):
        y = self.inner(x)
        return y.index_select(-1, self.perm.to(y.device))


def glu_rows(I: int, tile: int = 16):
    """merged row of gate row i / up row i (models/decoder.py interleave_glu_rows)"""
    g = [(i // tile) * 2 * tile + i % tile for i in range(I)]
    return g, [r + tile for r in g]


def restore_hf_views(model: nn.Module) -> nn.Module:
    base = getattr(model, "model", None)
    for layer in getattr(base, "layers", []) or []:
        attn = getattr(layer, "self_attn", None) or getattr(layer, "attention", None)
        sp = getattr(attn, "_illm_qkv_split", None) if attn is not None else None
        if sp is not None and hasattr(attn, "qkv_proj") and not hasattr(attn, "q_proj"):
            o = 0
            for i, (n, w) in enumerate(zip(("q_proj", "k_proj", "v_proj"), sp)):
                setattr(attn, n, ProjView(attn, "qkv_proj", list(range(o, o + w)), i == 2))
                o += w
        mlp = getattr(layer, "mlp", None) or getattr(layer, "feed_forward", None)
        if mlp is not None and hasattr(mlp, "experts"):
            mlp = getattr(mlp, "shared_expert", None)
        if mlp is None or not getattr(mlp, "_illm_interleaved", False) or not hasattr(mlp, "gate_up_proj") \
                or isinstance(mlp.gate_up_proj, FusedGLUView) or hasattr(mlp, "gate_proj"):
            continue
        g, u = glu_rows(mlp.gate_up_proj.out_features // 2)
        if type(mlp).__name__.startswith(("Phi3", "Glm")):           # its forward calls the fused projection
            mlp.gate_up_proj = FusedGLUView(mlp.gate_up_proj, g + u)
        else:
            mlp.gate_proj = ProjView(mlp, "gate_up_proj", g, False)
            mlp.up_proj = ProjView(mlp, "gate_up_proj", u, True)
    return model
