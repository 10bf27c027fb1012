"""Plain-PyTorch reference implementations of every native op.

Used (a) as the fp32 numerics reference in the kernel unit tests and (b) as
the execution path on CPU-only machines for the ops that have no C++ CPU
kernel.  They mirror the HF module semantics the HIP kernels reproduce.
"""
from __future__ import annotations

import math
from functools import lru_cache
from typing import Optional

import torch
import torch.nn.functional as F

from ..quantize import qtypes as Q

FMT_BITS = {Q.FMT_SYM_INT4: 4, Q.FMT_ASYM_INT4: 4, Q.FMT_NF4: 4, Q.FMT_FP4: 4, Q.FMT_NF3: 4}
HAS_MIN = {Q.FMT_ASYM_INT4, Q.FMT_ASYM_INT5}
TILE_N, CHUNK_K, QBLOCK = 16, 128, 64


def fmt_bits(fmt: int) -> int:
    return FMT_BITS.get(fmt, 8)


def _pad(v, m):
    return (v + m - 1) // m * m


def dev_tile_bytes(fmt, KC):
    """bytes of one 16-row tile region: KC code chunks, then [16][KC] scale
    dwords, then (asym) [16][KC] min dwords."""
    return KC * fmt_bits(fmt) * 256 + TILE_N * KC * 4 * (2 if fmt in HAS_MIN else 1)


def dev_total(fmt, n, k):
    return (_pad(n, TILE_N) // TILE_N) * dev_tile_bytes(fmt, _pad(k, CHUNK_K) // CHUNK_K) + 16


def canon_sizes(fmt, n, k):
    return n * k * fmt_bits(fmt) // 8, n * (k // QBLOCK)


def _e4m3_table():
    out = torch.zeros(256)
    for v in range(256):
        s, e, m = v >> 7, (v >> 3) & 15, v & 7
        r = m * 2.0 ** -9 if e == 0 else (8 + m) * 2.0 ** (e - 10)
        if e == 15 and m == 7:
            r = float("nan")
        out[v] = -r if s else r
    return out


def _e5m2_table():
    out = torch.zeros(256)
    for v in range(256):
        s, e, m = v >> 7, (v >> 2) & 31, v & 3
        if e == 0:
            r = m * 2.0 ** -16
        elif e == 31:
            r = float("inf") if m == 0 else float("nan")
        else:
            r = (4 + m) * 2.0 ** (e - 17)
        out[v] = -r if s else r
    return out


@lru_cache(None)
def code_table(fmt: int) -> torch.Tensor:
    """value of each code before scale/min (f32)."""
    if fmt == Q.FMT_SYM_INT4:
        return torch.arange(16, dtype=torch.float32) - 8
    if fmt == Q.FMT_ASYM_INT4:
        return torch.arange(16, dtype=torch.float32)
    if fmt == Q.FMT_NF4:
        return torch.tensor(Q.NF4_TABLE, dtype=torch.float32)
    if fmt == Q.FMT_NF3:
        return torch.tensor(Q.NF3_TABLE + [0.0] * 8, dtype=torch.float32)
    if fmt == Q.FMT_FP4:
        return torch.tensor(Q.FP4_TABLE, dtype=torch.float32)
    if fmt in (Q.FMT_SYM_INT8, Q.FMT_SYM_INT5):
        return torch.arange(256, dtype=torch.int32).to(torch.uint8).view(torch.int8).float()
    if fmt == Q.FMT_ASYM_INT5:
        return torch.arange(256, dtype=torch.float32)
    if fmt in (Q.FMT_FP8E4, Q.FMT_FP6):
        return _e4m3_table()
    if fmt == Q.FMT_FP8E5:
        return _e5m2_table()
    raise ValueError(fmt)


def dequantize_canonical(blob: torch.Tensor, fmt: int, n: int, k: int) -> torch.Tensor:
    """Canonical planar blob -> f32 [n, k] (pure torch; mirrors quant.cpp)."""
    blob = blob.reshape(-1).to(torch.uint8)
    cb, se = canon_sizes(fmt, n, k)
    codes = blob[:cb]
    scales = blob[cb:cb + 2 * se].view(torch.float16).float().view(n, k // QBLOCK)
    mins = blob[cb + 2 * se:cb + 4 * se].view(torch.float16).float().view(n, k // QBLOCK) \
        if fmt in HAS_MIN else None
    if fmt_bits(fmt) == 4:
        c = codes.view(n, k // QBLOCK, 32).long()
        q = torch.cat([c & 15, c >> 4], dim=-1)
    else:
        q = codes.view(n, k // QBLOCK, QBLOCK).long()
    v = code_table(fmt).to(blob.device)[q] * scales[..., None]
    if mins is not None:
        v = v + mins[..., None]
    return v.reshape(n, k)


@lru_cache(None)
def _perm_pos(fmt):
    # fragment element j -> nibble position inside the code dword
    if fmt in (Q.FMT_SYM_INT4, Q.FMT_ASYM_INT4):
        return [((4 + (j >> 1)) if (j & 1) else (j >> 1)) for j in range(8)]
    return list(range(8))


def device_index(fmt: int, n: int, k: int, device="cpu"):
    """(code byte offset, nibble shift, fp16 index of the scale) of every
    (row, k) element in the MI355X tiled blob -- the spec of
    csrc/common/formats.h in torch.  The min (asym) is 32 halves after the scale."""
    kpad = _pad(k, CHUNK_K)
    KC = kpad // CHUNK_K
    row = torch.arange(n, device=device)[:, None]
    kk = torch.arange(k, device=device)[None, :]
    t, r = row // TILE_N, row % TILE_N
    c, kin = kk // CHUNK_K, kk % CHUNK_K
    s, g, j = kin // 32, (kin % 32) // 8, kin % 8
    lane = g * 16 + r
    tile = t * dev_tile_bytes(fmt, KC)
    rec = tile + c * fmt_bits(fmt) * 256
    if fmt_bits(fmt) == 4:
        pos = torch.tensor(_perm_pos(fmt), device=device)[j]
        off = rec + lane * 16 + s * 4 + pos // 2
        shift = 4 * (pos % 2)
    else:
        off = rec + ((s // 2) * 64 + lane) * 16 + (s % 2) * 8 + j
        shift = torch.zeros_like(off)
    blk = (kk // QBLOCK) % 2
    sidx = (tile + KC * fmt_bits(fmt) * 256 + (c * TILE_N + r) * 4) // 2 + blk
    return off, shift, sidx


def dequantize_device_blob(blob: torch.Tensor, fmt: int, n: int, k: int) -> torch.Tensor:
    """MI355X tiled blob -> f32 [n, k] (pure torch reference)."""
    blob = blob.reshape(-1)[:dev_total(fmt, n, k)]
    off, shift, sidx = device_index(fmt, n, k, blob.device)
    byte = blob[off].long()
    q = (byte >> shift) & 15 if fmt_bits(fmt) == 4 else byte
    halves = blob.view(torch.float16)
    v = code_table(fmt).to(blob.device)[q] * halves[sidx].float()
    if fmt in HAS_MIN:
        v = v + halves[sidx + TILE_N * (_pad(k, CHUNK_K) // CHUNK_K) * 2].float()
    return v


# ---------------------------------------------------------------- layers
def rms_norm(x, w, eps, unit_offset=False):
    dt = x.dtype
    h = x.float()
    h = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps)
    ww = (1.0 + w.float()).to(dt) if unit_offset else w
    return ww * h.to(dt)


def add_rms_norm(x, residual, w, eps, unit_offset=False):
    """returns (normed, new_residual) with HF rounding semantics."""
    if residual is not None:
        x = residual + x
    return rms_norm(x, w, eps, unit_offset), x


def layer_norm(x, w, b, eps):
    return F.layer_norm(x.float(), (x.shape[-1],), None if w is None else w.float(),
                        None if b is None else b.float(), eps).to(x.dtype)


def glu(gu, act=0):
    g, u = gu.chunk(2, dim=-1)
    a = F.silu(g) if act == 0 else F.gelu(g, approximate="tanh")
    return a * u


def rope_cos_sin(pos, inv_freq, dtype):
    freqs = pos.float()[:, None] * inv_freq.float()[None, :]
    emb = torch.cat([freqs, freqs], dim=-1)
    return emb.cos().to(dtype), emb.sin().to(dtype)


def apply_rope(x, cos, sin, interleaved=False, rot_dim=None):
    """x: [T, H, D]; cos/sin: [T, rot_dim] (rotate_half layout)."""
    D = x.shape[-1]
    rot_dim = rot_dim or D
    xr, xp = x[..., :rot_dim], x[..., rot_dim:]
    c, s = cos[:, None, :], sin[:, None, :]
    if interleaved:
        x1, x2 = xr[..., 0::2], xr[..., 1::2]
        ch, sh = c[..., :rot_dim // 2], s[..., :rot_dim // 2]
        o1 = x1 * ch - x2 * sh
        o2 = x2 * ch + x1 * sh
        out = torch.stack([o1, o2], dim=-1).flatten(-2)
    else:
        x1, x2 = xr[..., :rot_dim // 2], xr[..., rot_dim // 2:]
        rot = torch.cat([-x2, x1], dim=-1)
        out = xr * c + rot * s
    return torch.cat([out, xp], dim=-1) if rot_dim < D else out


def attention(q, k, v, causal=True, scale=None, softcap=0.0, window=0, q_offset=None, alibi=None):
    """q: [B, Tq, Hq, D], k/v: [B, L, Hkv, D] -> [B, Tq, Hq, D] (f32 math).
    query t sits at absolute position q_offset + t (default L - Tq)."""
    B, Tq, Hq, D = q.shape
    L, Hkv = k.shape[1], k.shape[2]
    scale = scale or 1.0 / math.sqrt(D)
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(Hq // Hkv, dim=1)
    vf = v.float().transpose(1, 2).repeat_interleave(Hq // Hkv, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if softcap and softcap > 0:
        s = softcap * torch.tanh(s / softcap)
    kpos = torch.arange(L, device=q.device)
    if alibi is not None:
        s = s + alibi.float()[None, :, None, None] * kpos[None, None, None, :]
    off = (L - Tq) if q_offset is None else q_offset
    qpos = off + torch.arange(Tq, device=q.device)
    mask = torch.ones(Tq, L, dtype=torch.bool, device=q.device)
    if causal:
        mask &= kpos[None, :] <= qpos[:, None]
    if window and window > 0:
        mask &= kpos[None, :] > (qpos[:, None] - window)
    s = s.masked_fill(~mask, float("-inf"))
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, vf)
    return o.transpose(1, 2).to(q.dtype)


def moe_group_topk(logits, bias, k, n_group, topk_group, renorm=True, scale=1.0):
    """DeepSeek-V3 noaux_tc router (HF DeepseekV3TopkRouter.forward after the logits)."""
    lf = logits.float().reshape(-1, logits.shape[-1])
    T, E = lf.shape
    scores = lf.sigmoid()
    sfc = scores + (bias.float() if bias is not None else 0.0)
    gscore = sfc.view(T, n_group, E // n_group).topk(min(2, E // n_group), dim=-1)[0].sum(-1)
    gidx = torch.topk(gscore, k=topk_group, dim=-1, sorted=False)[1]
    gmask = torch.zeros_like(gscore).scatter_(1, gidx, 1.0)
    smask = gmask.unsqueeze(-1).expand(T, n_group, E // n_group).reshape(T, E)
    sfc = sfc.masked_fill(~smask.bool(), float("-inf"))
    idx = torch.topk(sfc, k=k, dim=-1)[1]
    w = scores.gather(1, idx)
    if renorm:
        w = w / (w.sum(-1, keepdim=True) + 1e-20)
    return w * scale, idx.to(torch.int32)


def moe_topk(logits, k, renorm=True, scoring=0):
    if scoring == 0:
        p = torch.softmax(logits.float(), dim=-1)
    else:
        p = torch.sigmoid(logits.float())
    w, ids = torch.topk(p, k, dim=-1)
    if renorm:
        w = w / w.sum(-1, keepdim=True)
    return w, ids.int()


def lowbit_linear_ref(x, blob, fmt, n, k, bias=None, device_layout=True):
    w = dequantize_device_blob(blob, fmt, n, k) if device_layout else dequantize_canonical(blob, fmt, n, k)
    y = x.float() @ w.t().to(x.device)
    if bias is not None:
        y = y + bias.float()
    return y


def moe_align(ids: torch.Tensor, e0: int, num_local: int):
    flat = ids.reshape(-1).long()
    e = flat - e0
    valid = (e >= 0) & (e < num_local)
    order = torch.argsort(torch.where(valid, e, num_local) * flat.numel() + torch.arange(flat.numel(), device=flat.device))
    counts = torch.bincount(e[valid], minlength=num_local)
    off = torch.zeros(num_local + 1, dtype=torch.int32, device=ids.device)
    off[1:] = counts.cumsum(0).to(torch.int32)
    rows = order[:int(valid.sum())].to(torch.int32)
    full = torch.zeros(max(flat.numel(), 1), dtype=torch.int32, device=ids.device)
    full[:rows.numel()] = rows
    return off, full


def moe_combine(part, w, ids, e0, num_local, dtype):
    ks, P, H = part.shape
    k = w.shape[-1]
    T = w.numel() // k
    s = part.float().sum(0).view(T, k, H)
    e = ids.reshape(T, k).long() - e0
    valid = ((e >= 0) & (e < num_local)).float()
    return (s * (w.reshape(T, k).float() * valid)[..., None]).sum(1).to(dtype)


def moe_gemm(x, blob, fmt, n, k, off, rows, xdiv, x_sorted, out_sorted, glu, act=0, out_f32=False):
    """fp32 reference of the grouped MoE GEMM (ops.moe_gemm)."""
    import torch.nn.functional as F
    P = rows.numel()
    nout = n // 2 if glu else n
    out = torch.zeros(P, nout, dtype=torch.float32, device=x.device)
    offl = off.tolist()
    rl = rows.tolist()
    for e in range(len(offl) - 1):
        s0, s1 = offl[e], offl[e + 1]
        if s1 <= s0:
            continue
        w = (dequantize_device_blob(blob[e], fmt, n, k) if blob.is_cuda else dequantize_canonical(blob[e], fmt, n, k))
        pos = list(range(s0, s1))
        xr = [p if x_sorted else rl[p] // xdiv for p in pos]
        y = x[xr].float() @ w.float().t()
        if glu:
            g = y.view(len(pos), n // 32, 2, 16)
            gate, up = g[:, :, 0].reshape(len(pos), -1), g[:, :, 1].reshape(len(pos), -1)
            y = (F.silu(gate) if act == 0 else F.gelu(gate, approximate="tanh")) * up
        orow = pos if out_sorted else [rl[p] for p in pos]
        out[orow] = y
    return out if out_f32 else out.to(x.dtype)
