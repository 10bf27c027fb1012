"""Native AutoTP: tensor-parallel sharding of HF decoder models.

Reference behaviour: DeepSpeed ``init_inference(mp_size, replace_method=
"auto")`` shards the model, then ``optimize_model`` swaps DeepSpeed's
``LinearLayer``/``LinearAllreduce`` for ``LowBitLinear`` carrying ``mp_group``
(``SRC/transformers/convert.py:217-228``,
``example/GPU/Deepspeed-AutoTP/deepspeed_autotp.py:81-106``); the all-reduce
runs inside ``LowBitLinear.forward`` (``low_bit_linear.py:715-722``).  The
reference library itself has no sharder.

MI355X design: a built-in sharder on the dense HF module tree, run on every
rank before quantization (each rank quantizes only its shard):
  * column-parallel (output rows split): q/k/v, gate/up and their fused
    variants -- attention heads are split as whole heads; when there are
    fewer KV heads than ranks each rank keeps the one KV head its query
    heads use (replication, as vLLM does);
  * row-parallel (input columns split): o_proj / down_proj -- the module
    gets ``mp_group`` so the converted low-bit layer all-reduces its output
    (RCCL, or the one-shot xGMI kernel for decode-sized messages);
  * lm_head: vocab-parallel rows + all-gather of the logits
    (:class:`VocabParallelHead`); embeddings stay replicated (a gather of
    a few rows is cheaper than an all-reduce per step).
With 288 GB per MI355X, TP is for latency (Llama-3-70B INT4 on 8 GPUs: each
GPU streams 1/8 of the weights per token), not for capacity.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from .comm import all_gather_last_dim, get_rank, get_world_size, setup_custom_all_reduce

COLUMN = {"q_proj", "k_proj", "v_proj", "gate_proj", "up_proj", "w1", "w3", "c_fc", "fc1",
          "dense_h_to_4h", "query", "key", "value"}
ROW = {"o_proj", "down_proj", "w2", "c_proj", "fc2", "dense_4h_to_h", "out_proj", "dense"}
KV = {"k_proj", "v_proj", "key", "value"}


class VocabParallelHead(nn.Module):
    """lm_head sharded over the vocabulary; logits all-gathered."""

    def __init__(self, local: nn.Module, group, vocab: int):
        super().__init__()
        self.local, self.group, self.vocab = local, group, vocab

    def forward(self, x):
        y = self.local(x)
        y = all_gather_last_dim(y, self.group)
        return y[..., :self.vocab] if y.shape[-1] != self.vocab else y

    @property
    def weight(self):
        return self.local.weight


def _slice_linear(lin: nn.Linear, dim: int, start: int, stop: int) -> nn.Linear:
    w = lin.weight.data
    ws = w[start:stop] if dim == 0 else w[:, start:stop]
    bias = lin.bias is not None and dim == 0
    new = nn.Linear(ws.shape[1], ws.shape[0], bias=bias or (lin.bias is not None), device="meta", dtype=w.dtype)
    new.weight = nn.Parameter(ws.contiguous().clone(), requires_grad=False)
    if lin.bias is not None:
        b = lin.bias.data[start:stop] if dim == 0 else lin.bias.data
        new.bias = nn.Parameter(b.contiguous().clone(), requires_grad=False)
    return new


def _kv_rows(n_kv: int, head_dim: int, rank: int, world: int, n_q: int):
    """row range of this rank's KV heads"""
    if n_kv % world == 0:
        per = n_kv // world
        return rank * per * head_dim, (rank + 1) * per * head_dim
    # fewer KV heads than ranks: keep the KV head of this rank's first q head
    q_per = n_q // world
    group = n_q // n_kv
    h = (rank * q_per) // group
    return h * head_dim, (h + 1) * head_dim


def _div(a: int, b: int, what: str):
    if a % b:
        raise ValueError(f"tensor parallel: {what}={a} is not divisible by world size {b}")
    return a // b


@torch.no_grad()
def auto_tp(model: nn.Module, group=None, rank: Optional[int] = None, world: Optional[int] = None,
            shard_lm_head: bool = True) -> nn.Module:
    """Shard a dense HF CausalLM in place for tensor parallelism.  Call on
    every rank (same weights everywhere, e.g. same checkpoint or seed)."""
    rank = get_rank(group) if rank is None else rank
    world = get_world_size(group) if world is None else world
    if world == 1:
        return model
    if group is None:
        import torch.distributed as dist
        group = dist.group.WORLD             # explicit: mp_group=None means "no all-reduce"
    cfg = model.config
    n_q = cfg.num_attention_heads
    n_kv = getattr(cfg, "num_key_value_heads", None) or n_q
    head_dim = getattr(cfg, "head_dim", None) or cfg.hidden_size // n_q
    _div(n_q, world, "num_attention_heads")
    if n_kv % world and world % n_kv:
        raise ValueError(f"tensor parallel: num_key_value_heads={n_kv} incompatible with world size {world}")

    for mod_name, mod in list(model.named_modules()):
        for cname, child in list(mod.named_children()):
            if not isinstance(child, nn.Linear):
                continue
            if cname in ("lm_head", "embed_out", "output"):
                continue
            if cname in KV:
                a, b = _kv_rows(n_kv, head_dim, rank, world, n_q)
                setattr(mod, cname, _slice_linear(child, 0, a, b))
            elif cname in COLUMN:
                per = _div(child.out_features, world, f"{mod_name}.{cname}.out_features")
                setattr(mod, cname, _slice_linear(child, 0, rank * per, (rank + 1) * per))
            elif cname in ROW and (cname != "dense" or "attention" in mod_name or "attn" in mod_name):
                per = _div(child.in_features, world, f"{mod_name}.{cname}.in_features")
                new = _slice_linear(child, 1, rank * per, (rank + 1) * per)
                if child.bias is not None and rank != 0:
                    new.bias.zero_()            # bias added once after the all-reduce sum
                new.mp_group = group
                setattr(mod, cname, new)
        # per-module head bookkeeping used by some HF forwards
        if hasattr(mod, "num_key_value_groups") and n_kv % world:
            mod.num_key_value_groups = n_q // world
        for attr, val in (("num_heads", n_q // world), ("num_key_value_heads", max(1, n_kv // world))):
            if hasattr(mod, attr) and isinstance(getattr(mod, attr), int):
                setattr(mod, attr, val)

    if shard_lm_head:
        head = model.get_output_embeddings()
        if isinstance(head, nn.Linear) and not getattr(cfg, "tie_word_embeddings", False):
            V = head.out_features
            per = (V + world - 1) // world
            a, b = rank * per, min(V, (rank + 1) * per)
            local = _slice_linear(head, 0, a, b)
            if b - a < per:                      # pad the last shard so all_gather sizes match
                pad = nn.Linear(local.in_features, per, bias=False, device="meta", dtype=local.weight.dtype)
                if local.weight.device.type == "meta":      # shape-only rebuild (load_low_bit of a TP save)
                    w = torch.empty(per, local.in_features, dtype=local.weight.dtype, device="meta")
                else:
                    w = torch.zeros(per, local.in_features, dtype=local.weight.dtype)
                    w[:b - a] = local.weight.data
                pad.weight = nn.Parameter(w, requires_grad=False)
                local = pad
            model.set_output_embeddings(VocabParallelHead(local, group, V))
    model._tp = {"group": group, "rank": rank, "world": world, "num_heads": n_q // world,
                 "num_kv_heads": max(1, n_kv // world)}
    return model


def tp_info(model: nn.Module):
    return getattr(model, "_tp", None)


def enable_fast_all_reduce(group=None, max_bytes: int = 1 << 20):
    """Collective: install the one-shot xGMI all-reduce for ``group`` (GPU,
    intra-node).  Row-parallel layers then use it for messages <= max_bytes."""
    return setup_custom_all_reduce(group, max_bytes)
