"""Expert parallelism for MoE models (Mixtral / Qwen2-MoE / Qwen3-MoE).

The reference library has no EP (only vLLM's ``expert_map``
in the patched fused-MoE, ``VLLM_PATCH:11514-11516``; DeepSeek decode
requires ``ep_size == 1``, ``models/deepseek.py:335``).  BASELINE config 3
(Mixtral 8x7B on 8x MI355X) needs it, so it is native here:

* :func:`shard_experts` -- rank r keeps experts [r*E/W, (r+1)*E/W) of every
  MoE block (before or after quantization).  Attention / dense layers stay
  replicated (or tensor-parallel via ``parallel.tp``).
* decode ("replicated tokens") mode, used by :class:`models.moe.NativeMoE`:
  every rank routes all tokens, runs its local experts through the grouped
  GEMV, and ONE all-reduce over the EP group sums the partial outputs.  For
  decode batches this is a single small message per MoE layer, which the
  one-shot xGMI all-reduce handles in one launch.
* prefill / data-parallel mode, :func:`ep_moe_all_to_all`: each rank owns
  different tokens; token copies are dispatched to the owners of their
  experts with ``all_to_all_single`` (RCCL alltoallv over xGMI: every GPU
  talks to all 7 peers on separate links), computed there, and returned with
  a second all-to-all; routing weights are applied at the source.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .comm import get_rank, get_world_size


def expert_range(num_experts: int, rank: int, world: int):
    if num_experts % world:
        raise ValueError(f"expert parallel: {num_experts} experts not divisible by {world} ranks")
    per = num_experts // world
    return rank * per, per


@torch.no_grad()
def shard_experts(model: nn.Module, group=None) -> nn.Module:
    """Keep only this rank's experts in every MoE block (HF module tree,
    dense 3-D expert params or converted :class:`HFLowBitExperts`)."""
    from ..models.moe import HFLowBitExperts
    rank, world = get_rank(group), get_world_size(group)
    if world == 1:
        return model
    if group is None:
        group = dist.group.WORLD
    for mod in model.modules():
        ex = getattr(mod, "experts", None)
        if ex is None or not hasattr(mod, "gate"):
            continue
        if isinstance(ex, HFLowBitExperts):
            E = ex.gate_up.num_experts
            e0, per = expert_range(E, rank, world)
            for bank in (ex.gate_up, ex.down):
                bank.weight = nn.Parameter(bank.weight[e0:e0 + per].contiguous(), requires_grad=False)
                bank.num_experts = per
            ex.num_experts = per
        elif isinstance(getattr(ex, "gate_up_proj", None), nn.Parameter):
            E = ex.gate_up_proj.shape[0]
            e0, per = expert_range(E, rank, world)
            ex.gate_up_proj = nn.Parameter(ex.gate_up_proj.data[e0:e0 + per].contiguous(), requires_grad=False)
            ex.down_proj = nn.Parameter(ex.down_proj.data[e0:e0 + per].contiguous(), requires_grad=False)
            ex.num_experts = per
        else:
            continue
        mod._ep = {"e0": e0, "local": per, "group": group, "num_experts": E}
        ex._ep = mod._ep
    model._ep = {"group": group, "rank": rank, "world": world}
    return model


def ep_moe_all_to_all(x: torch.Tensor, moe, group=None) -> torch.Tensor:
    """Token-sharded MoE: x [T_local, H] are THIS rank's tokens; ``moe`` is
    the rank's :class:`NativeMoE` (local experts [e0, e0+El)).  Returns the
    routed-experts output for the local tokens (shared expert not included).

    Dropless fixed-capacity dispatch (every rank may send all of its T*k
    pairs to one peer): pairs are sorted by destination rank on the device
    (``moe_align`` over rank ids), packed into [world, T*k, H] slots and
    exchanged with equal-split ``all_to_all_single`` (RCCL alltoall over
    xGMI); the receiver marks empty slots with expert -1, so the grouped
    expert GEMMs skip them.  No host synchronisation and no per-expert
    Python loop: the whole dispatch / compute / combine is capturable."""
    from .. import ops
    world = get_world_size(group)
    El = moe.local_experts
    T, H = x.shape
    w, ids = moe.route(x)                                     # [T, k]
    k = ids.shape[1]
    P = T * k
    dev = x.device
    ids32 = ids.reshape(-1).to(torch.int32).contiguous()
    dest = torch.div(ids32, El, rounding_mode="floor").to(torch.int32)
    off, rows = ops.moe_align(dest, 0, world)                  # pairs sorted by destination rank
    rows_l = rows.long()
    dst_sorted = dest.long()[rows_l]
    slot = torch.arange(P, device=dev) - off.long()[dst_sorted]   # position inside the destination's slots
    flat = dst_sorted * P + slot
    send_x = x.new_zeros(world * P, H)
    send_x.index_copy_(0, flat, x[rows_l // k])
    send_e = torch.full((world * P,), -1, dtype=torch.int32, device=dev)
    send_e.index_copy_(0, flat, ids32[rows_l])
    recv_x = torch.empty_like(send_x)
    recv_e = torch.empty_like(send_e)
    dist.all_to_all_single(recv_x, send_x, group=group)
    dist.all_to_all_single(recv_e, send_e, group=group)
    # expert id -1 (empty slot) and other ranks' experts fall outside [e0, e0 + El)
    if x.is_cuda and ops.native_gpu(x) and moe.grouped_gemm_ok(x):
        off2, rows2 = ops.moe_align(recv_e, moe.e0, El)
        gu, dn = moe.gate_up, moe.down
        a = ops.moe_gemm(recv_x, gu.weight, gu.fmt, gu.out_features, gu.in_features, off2, rows2, 1,
                         False, True, True, moe.act)
        out = ops.moe_gemm(a, dn.weight, dn.fmt, dn.out_features, dn.in_features, off2, rows2, 1,
                           True, False, False, 0, True)
        out = torch.where((recv_e >= 0)[:, None], out, out.new_zeros(()))   # unwritten rows of empty slots
    else:                                                     # CPU / non-native fallback
        import torch.nn.functional as F
        from ..models.decoder import deinterleave_glu
        out = torch.zeros(recv_x.shape[0], H, dtype=torch.float32, device=dev)
        for e in range(El):
            sel = (recv_e == moe.e0 + e).nonzero(as_tuple=True)[0]
            if sel.numel() == 0:
                continue
            g, u = deinterleave_glu(moe.gate_up.matmul(recv_x[sel], e))
            a = (F.silu(g.float()) if moe.act == 0 else F.gelu(g.float(), approximate="tanh")) * u.float()
            out[sel] = moe.down.matmul(a.to(x.dtype), e).float()
    back = torch.empty_like(out)
    dist.all_to_all_single(back, out, group=group)
    y = torch.zeros(T, H, dtype=torch.float32, device=dev)
    wf = w.reshape(-1).float()[rows_l]
    y.index_add_(0, rows_l // k, back[flat] * wf[:, None])
    return y.to(x.dtype)
