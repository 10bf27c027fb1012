"""SnapKV-style KV compression at prefill.

Reference: ``SRC/transformers/kv.py:221-293, 296-423`` (``compress_kv``:
keep the last ``window`` tokens plus, per KV head, the top
``capacity - window`` earlier tokens ranked by the observation window's
pooled attention; on by default for 1800-4500-token prompts on small
iGPUs) and ``models/utils.py:360-380`` (``IPEX_LLM_COMPRESS_KV_CACHE``).

Paged-cache design: the kept entries are written to cache indices
0..capacity-1 of the sequence (each KV head keeps its own token set -- the
[block, head, slot, dim] layout allows that) while the rotary position keeps
counting from the prompt length; decode uses ``pos_offset = L - capacity``
so new tokens land at cache index ``pos - offset``.
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F

from .. import ops
from ..models.cache import SequenceState, make_block_table, slots_for


@torch.no_grad()
def snapkv_compress(model, cache, seq: SequenceState, L: int, q_window: Dict[int, torch.Tensor],
                    capacity: int = 1024, window: int = 32, pool: int = 7) -> int:
    """Compress one prefilled sequence of length L in place; returns the new
    cache length (``capacity``)."""
    s = model.spec
    if L <= capacity:
        return L
    dev = cache.k[0].device
    bt = make_block_table([seq], len(seq.blocks), dev)
    Hkv, G, D = s.num_kv_heads, s.num_heads // s.num_kv_heads, s.head_dim
    keep_n = capacity - window
    dst = slots_for(seq, 0, capacity, cache.bs).to(dev)
    lf = getattr(cache, "lf", None)
    if lf is not None:
        # Yuan LFA: the next step's filter reads the previous position's h /
        # conv rows at cache index L - 1 - offset = capacity - 1
        src_last = slots_for(seq, L - 1, 1, cache.bs).to(dev)
        for t in lf:
            t[dst[-1:]] = t[src_last]
    for li in range(len(model.layers)):
        kk = ops.api.gather_kv(cache.k[li], bt, 0, L, cache.kv_fp8, cache.k_scale, model.dtype)   # [L, Hkv, D]
        vv = ops.api.gather_kv(cache.v[li], bt, 0, L, cache.kv_fp8, cache.v_scale, model.dtype)
        q = q_window[li].float()                                     # [W, Hq, D]
        W = q.shape[0]
        qg = q.view(W, Hkv, G, D)
        sc = torch.einsum("whgd,lhd->hgwl", qg, kk.float()) * s.scale  # [Hkv, G, W, L]
        kpos = torch.arange(L, device=dev)
        qpos = L - W + torch.arange(W, device=dev)
        sc = sc.masked_fill(kpos[None, None, None, :] > qpos[None, None, :, None], float("-inf"))
        p = torch.softmax(sc, -1).sum((1, 2))                         # [Hkv, L]
        pre = p[:, :L - window]
        pre = F.avg_pool1d(pre[:, None], pool, stride=1, padding=pool // 2)[:, 0]
        idx = pre.topk(keep_n, dim=-1).indices.sort(-1).values        # [Hkv, keep_n]
        idx = torch.cat([idx, torch.arange(L - window, L, device=dev).expand(Hkv, window)], 1)   # [Hkv, cap]
        hsel = torch.arange(Hkv, device=dev)[:, None]
        kc = kk[idx, hsel].transpose(0, 1)                              # [cap, Hkv, D]
        vc = vv[idx, hsel].transpose(0, 1)
        blk, off = dst // cache.bs, dst % cache.bs
        if cache.kv_fp8:
            e5 = cache.kv_fp8 == 1
            cache.k[li][blk, :, off] = ops.to_fp8_bytes((kc / cache.k_scale).float(), e5).to(dev)
            cache.v[li][blk, :, off] = ops.to_fp8_bytes((vc / cache.v_scale).float(), e5).to(dev)
        else:
            cache.k[li][blk, :, off] = kc.to(cache.k[li].dtype)
            cache.v[li][blk, :, off] = vc.to(cache.v[li].dtype)
    seq.length = capacity
    return capacity
