"""Embedding variants: host-resident, disk-backed and low-bit.

Reference: ``SRC/transformers/embedding.py:29-241`` -- ``CPUEmbedding``
(weights pinned to the host), ``DiskEmbedding`` (fp16 rows read from a file
per token), ``LowBitEmbedding`` (q2_k/q4_k rows dequantized by
``xe_linear.dequantize_rows``).

Here ``LowBitEmbedding`` keeps the canonical (row-major) low-bit blob and
gathers + dequantizes only the looked-up rows with a HIP kernel
(``embedding_lowbit``); a 128256 x 4096 vocabulary drops from 1 GB (bf16)
to ~280 MB (sym_int4).  With 288 GB per MI355X the host/disk variants are
rarely needed; they exist for parity and for very large vocabularies.
"""
from __future__ import annotations

import os
import tempfile
from typing import Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..quantize import qtypes as Q


class CPUEmbedding(nn.Module):
    """Embedding table kept on the host; outputs move to the ids' device."""

    def __init__(self, weight: torch.Tensor, padding_idx: Optional[int] = None):
        super().__init__()
        self.weight = nn.Parameter(weight.detach().cpu(), requires_grad=False)
        self.padding_idx = padding_idx
        self.num_embeddings, self.embedding_dim = weight.shape

    @classmethod
    def from_embedding(cls, emb: nn.Embedding):
        return cls(emb.weight.data, emb.padding_idx)

    def _apply(self, fn, recurse=True):
        # never leaves the host (model.to("cuda") keeps it here)
        w = self.weight
        probe = fn(torch.empty(0, dtype=w.dtype))
        if probe.dtype != w.dtype and probe.is_floating_point():
            self.weight = nn.Parameter(w.to(probe.dtype), requires_grad=False)
        return self

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        return F.embedding(ids.cpu(), self.weight, self.padding_idx).to(ids.device)


class DiskEmbedding(nn.Module):
    """fp16 rows in a memory-mapped file; only looked-up rows are read."""

    def __init__(self, weight: torch.Tensor, path: Optional[str] = None, padding_idx: Optional[int] = None):
        super().__init__()
        self.num_embeddings, self.embedding_dim = weight.shape
        self.padding_idx = padding_idx
        self.path = path or os.path.join(tempfile.mkdtemp(prefix="illm_emb_"), "embeddings.bin")
        mm = np.memmap(self.path, dtype=np.float16, mode="w+", shape=tuple(weight.shape))
        mm[:] = weight.detach().to(torch.float16).cpu().numpy()
        mm.flush()
        del mm
        self._mm = np.memmap(self.path, dtype=np.float16, mode="r", shape=tuple(weight.shape))
        self.register_buffer("_dtype_probe", torch.empty(0, dtype=weight.dtype), persistent=False)

    @classmethod
    def from_embedding(cls, emb: nn.Embedding, path: Optional[str] = None):
        return cls(emb.weight.data, path, emb.padding_idx)

    @property
    def weight(self):      # materialized only when someone asks (e.g. tied lm_head)
        return torch.from_numpy(np.asarray(self._mm)).to(self._dtype_probe.dtype)

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        flat = ids.reshape(-1).cpu().numpy()
        rows = torch.from_numpy(np.asarray(self._mm[flat]))
        return rows.to(ids.device, self._dtype_probe.dtype).reshape(*ids.shape, self.embedding_dim)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        destination[prefix + "weight"] = self.weight


class LowBitEmbedding(nn.Module):
    """Quantized embedding table (canonical row-major blob on any device)."""

    def __init__(self, num_embeddings: int, embedding_dim: int, qtype="sym_int4", padding_idx=None,
                 dtype=torch.bfloat16, device=None):
        super().__init__()
        self.num_embeddings, self.embedding_dim = num_embeddings, embedding_dim
        self.qtype = Q.resolve_qtype(qtype)
        f = Q.get_format(self.qtype)
        if f is None:
            raise ValueError("LowBitEmbedding needs a low-bit qtype")
        if embedding_dim % f.k_align:
            raise ValueError(f"embedding_dim must be a multiple of {f.k_align}")
        self.fmt = f.fmt
        self.padding_idx = padding_idx
        self.dtype = dtype
        from .low_bit_linear import _canon_total
        self.weight = nn.Parameter(torch.zeros(_canon_total(self.fmt, num_embeddings, embedding_dim),
                                               dtype=torch.uint8, device=device or "cpu"), requires_grad=False)

    @classmethod
    @torch.no_grad()
    def from_embedding(cls, emb: nn.Embedding, qtype="sym_int4"):
        w = emb.weight.data
        m = cls(w.shape[0], w.shape[1], qtype, emb.padding_idx, w.dtype if w.is_floating_point() else torch.bfloat16,
                device="meta")
        m.weight = nn.Parameter(ops.quantize(w.float().cpu(), m.fmt), requires_grad=False)
        return m

    def _apply(self, fn, recurse=True):
        # the canonical blob is valid on any device: move bytes, keep dtype
        w = self.weight
        probe = fn(torch.empty(0, dtype=torch.float32, device=w.device))
        if probe.dtype in (torch.float16, torch.bfloat16, torch.float32):
            self.dtype = probe.dtype if probe.dtype != torch.float32 else self.dtype
        if probe.device != w.device:
            self.weight = nn.Parameter(w.to(probe.device), requires_grad=False)
        return self

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        n, k = self.num_embeddings, self.embedding_dim
        dt = self.dtype if self.dtype in (torch.float16, torch.bfloat16) else torch.bfloat16
        if self.weight.is_cuda and ops.native_gpu(self.weight):
            out = torch.ops.ipex_llm_amd.embedding_lowbit(self.weight, self.fmt, n, k, ids.to(self.weight.device), dt)
        else:
            rows = ops.dequantize(self.weight, self.fmt, n, k, torch.float32)[ids.reshape(-1).cpu()]
            out = rows.reshape(*ids.shape, k).to(ids.device)
        return out.to(self.dtype) if out.dtype != self.dtype else out


def replace_embeddings(model: nn.Module, embedding_qtype=None, cpu_embedding: bool = False,
                       disk_embedding: bool = False):
    """Swap the input embedding (reference convert.py embedding policy)."""
    emb = model.get_input_embeddings() if hasattr(model, "get_input_embeddings") else None
    if not isinstance(emb, nn.Embedding):
        return model
    if disk_embedding:
        new = DiskEmbedding.from_embedding(emb)
    elif embedding_qtype is not None:
        new = LowBitEmbedding.from_embedding(emb, embedding_qtype)
    elif cpu_embedding:
        new = CPUEmbedding.from_embedding(emb)
    else:
        return model
    model.set_input_embeddings(new)
    if hasattr(model, "config"):
        model.config.bigdl_disk_embedding = bool(disk_embedding)
    return model
