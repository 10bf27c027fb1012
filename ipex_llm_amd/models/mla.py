"""Multi-head Latent Attention (DeepSeek-V2 / V3, MiniCPM3) on the native engine.

Reference: ``SRC/transformers/models/deepseek.py:182-343`` and
``deepseek_v3.py:45-233`` (absorbed-weight MLA decode over a compressed KV
cache) and ``minicpm3.py``.

The paged cache holds ONE latent row per token: ``[c_kv (kv_lora_rank) |
k_pe (qk_rope_head_dim)]`` -- 576 values for DeepSeek-V3 instead of
128 heads x (192 + 128) for the expanded K/V, i.e. 71x less KV traffic per
decoded token (the point of MLA).  Attention runs in the latent space with
the up-projections absorbed:

    q_lat[h]  = W_UK[h]^T q_nope[h]                       [r]
    score     = (q_lat[h] . c_kv + q_pe[h] . k_pe) * scale
    o_lat[h]  = softmax(score) @ c_kv                      [r]
    o[h]      = W_UV[h] o_lat[h]                           [v_head_dim]

(W_UK / W_UV are the two halves of ``kv_b_proj``, kept dense: 2 x H x 128 x
512 per layer).  Every step is device-side (the latent gather reads the
block table, the causal / length mask comes from ``seq_lens``), so a decode
step captures into a hipGraph like the dense decoder.  The MoE / dense MLP
blocks run their converted low-bit modules (grouped-router kernel, low-bit
expert banks).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..ops import reference as R
from .decoder import DecoderSpec, NativeCausalLM

MLA_ARCHS = {"deepseek_v3", "deepseek_v2", "minicpm3"}


def _dense_weight(mod: nn.Module) -> torch.Tensor:
    if hasattr(mod, "dequantize"):
        return mod.dequantize(torch.float32)
    return mod.weight.data.float()


class MLAAttention(nn.Module):
    def __init__(self, at: nn.Module, cfg, dtype):
        super().__init__()
        self.H = cfg.num_attention_heads
        self.dn, self.dr = cfg.qk_nope_head_dim, cfg.qk_rope_head_dim
        self.r, self.dv = cfg.kv_lora_rank, cfg.v_head_dim
        self.q_proj = getattr(at, "q_proj", None)
        self.q_a_proj = getattr(at, "q_a_proj", None)
        self.q_b_proj = getattr(at, "q_b_proj", None)
        qn = getattr(at, "q_a_layernorm", None)
        self.q_a_norm = nn.Parameter(qn.weight.data, requires_grad=False) if qn is not None else None
        self.q_a_eps = getattr(qn, "variance_epsilon", getattr(qn, "eps", 1e-6)) if qn is not None else 1e-6
        self.kv_a_proj = at.kv_a_proj_with_mqa
        kn = at.kv_a_layernorm
        self.kv_a_norm = nn.Parameter(kn.weight.data, requires_grad=False)
        self.kv_a_eps = getattr(kn, "variance_epsilon", getattr(kn, "eps", 1e-6))
        self.o_proj = at.o_proj
        wkv = _dense_weight(at.kv_b_proj).view(self.H, self.dn + self.dv, self.r)
        self.w_uk = nn.Parameter(wkv[:, :self.dn].contiguous().to(dtype), requires_grad=False)   # [H, dn, r]
        self.w_uv = nn.Parameter(wkv[:, self.dn:].contiguous().to(dtype), requires_grad=False)   # [H, dv, r]
        self.scale = float(at.scaling)


class MLALayer(nn.Module):
    def __init__(self, attn: MLAAttention, mlp: nn.Module, ln1, ln2):
        super().__init__()
        self.self_attn, self.mlp = attn, mlp
        self.input_layernorm = nn.Parameter(ln1, requires_grad=False)
        self.post_attention_layernorm = nn.Parameter(ln2, requires_grad=False)
        self.pre_feedforward_layernorm = self.post_feedforward_layernorm = None


class MLACausalLM(NativeCausalLM):
    def __init__(self, spec: DecoderSpec, cfg, embed, layers: List[MLALayer], norm, lm_head, inv_freq,
                 rope_scaling: float, dtype, interleaved: bool, embed_scale: float = 1.0, residual_scale: float = 1.0):
        super().__init__(spec, embed, layers, norm, lm_head, inv_freq, dtype)
        a0 = layers[0].self_attn
        self.r, self.dr = a0.r, a0.dr
        self.interleaved = interleaved
        self.embed_scale = embed_scale
        self.residual_scale = residual_scale
        self.logits_div = 1.0
        spec.rope_attention_scaling = rope_scaling

    # one latent row per token: K holds [c_kv | k_pe]; V aliases it (never written
    # separately).  One extra block is a scratch target for padded (-1) slots.
    def make_cache(self, max_tokens: int, batch: int = 1, block_size: int = 64, kv_fp8: int = 0,
                   num_blocks: Optional[int] = None):
        from .cache import BlockAllocator, PagedKVCache
        nblk = num_blocks or batch * ((max_tokens + block_size - 1) // block_size)
        self.ensure_rope_cache(max_tokens + 1)
        c = PagedKVCache.__new__(PagedKVCache)
        c.num_layers, c.num_blocks = len(self.layers), nblk
        c.Hkv, c.D, c.bs = 1, self.r + self.dr, block_size
        c.dtype, c.kv_fp8, c.k_scale, c.v_scale = self.dtype, 0, 1.0, 1.0
        c.k = [torch.zeros(nblk + 1, 1, block_size, self.r + self.dr, dtype=self.dtype, device=self.device)
               for _ in self.layers]
        c.v = c.k
        c.allocator = BlockAllocator(nblk)
        c.device = self.device
        return c

    def graph_max_batch(self) -> int:
        lim = 16
        for L in self.layers:
            if hasattr(L.mlp, "graph_max_tokens"):
                lim = min(lim, L.mlp.graph_max_tokens())
        return lim

    def _rope(self, x: torch.Tensor, pos: torch.Tensor) -> torch.Tensor:
        """x [T, h, dr]; cos/sin looked up on the device from the table"""
        tab = self.ensure_rope_cache(1) if self.rope_cache is None else self.rope_cache
        cs = tab[pos.long()]                                   # [T, dr/2, 2] (scaled)
        cos = torch.cat([cs[..., 0]] * 2, -1).to(x.dtype)
        sin = torch.cat([cs[..., 1]] * 2, -1).to(x.dtype)
        return R.apply_rope(x, cos, sin, self.interleaved, self.dr)

    def _norm(self, x, w, eps):
        return ops.rms_norm(x.contiguous(), w, eps)

    def _mla(self, li: int, a: MLAAttention, x, pos, slots, meta, cache):
        T = x.shape[0]
        H, dn, dr, r = a.H, a.dn, a.dr, a.r
        if a.q_proj is not None:
            q = a.q_proj(x)
        else:
            q = a.q_b_proj(self._norm(a.q_a_proj(x), a.q_a_norm, a.q_a_eps))
        q = q.view(T, H, dn + dr)
        q_nope, q_pe = q[..., :dn], self._rope(q[..., dn:], pos)
        kv = a.kv_a_proj(x)
        c = self._norm(kv[:, :r], a.kv_a_norm, a.kv_a_eps)
        kpe = self._rope(kv[:, None, r:], pos)[:, 0]
        flat = cache.k[li].view(-1, r + dr)
        scratch = cache.num_blocks * cache.bs
        s = torch.where(slots >= 0, slots, torch.full_like(slots, scratch))
        flat.index_copy_(0, s.long(), torch.cat([c, kpe], -1).to(flat.dtype))
        # absorbed attention in the latent space
        cdt = torch.float32 if not x.is_cuda else x.dtype
        q_lat = torch.einsum("thd,hdr->thr", q_nope.to(cdt), a.w_uk.to(cdt))
        B, Tq = meta.B, meta.Tq
        bt = meta.block_tables.long()
        lat = cache.k[li][bt].view(B, -1, r + dr).to(cdt)              # [B, Lmax, r + dr]
        ql, qp = q_lat.view(B, Tq, H, r), q_pe.to(cdt).view(B, Tq, H, dr)
        sc = (torch.einsum("bthr,blr->bthl", ql, lat[..., :r]) +
              torch.einsum("bthd,bld->bthl", qp, lat[..., r:])).float() * a.scale
        kpos = torch.arange(lat.shape[1], device=x.device)
        qpos = meta.seq_lens.long()[:, None] - Tq + torch.arange(Tq, device=x.device)[None, :]
        mask = kpos[None, None, :] <= qpos[..., None]                    # [B, Tq, Lmax]
        sc = sc.masked_fill(~mask[:, :, None, :], float("-inf"))
        p = torch.softmax(sc, -1).to(cdt)
        o_lat = torch.einsum("bthl,blr->bthr", p, lat[..., :r])
        o = torch.einsum("bthr,hvr->bthv", o_lat, a.w_uv.to(cdt))
        return a.o_proj(o.reshape(T, H * a.dv).to(x.dtype).contiguous())

    def forward_tokens(self, ids: torch.Tensor, pos: torch.Tensor, slots: torch.Tensor, meta, cache,
                       logits_idx: Optional[torch.Tensor] = None, return_hidden: bool = False,
                       hidden_in: Optional[torch.Tensor] = None):
        s = self.spec
        if hidden_in is not None:
            h = hidden_in.to(self.dtype).contiguous()
        else:
            h = self.embed_module(ids).to(self.dtype) if self.embed_module is not None else \
                F.embedding(ids, self.embed_tokens)
            if self.embed_scale != 1.0:
                h = h * self.embed_scale
        rs = self.residual_scale
        for li, layer in enumerate(self.layers):
            x = ops.rms_norm(h.contiguous(), layer.input_layernorm, s.rms_eps)
            a = self._mla(li, layer.self_attn, x, pos, slots, meta, cache)
            h = h + (a * rs if rs != 1.0 else a)
            x = ops.rms_norm(h.contiguous(), layer.post_attention_layernorm, s.rms_eps)
            m = layer.mlp(x)
            h = h + (m * rs if rs != 1.0 else m)
        if not self.last_stage:
            return h
        if logits_idx is not None:
            h = h.index_select(0, logits_idx)
        x = ops.rms_norm(h.contiguous(), self.norm, s.rms_eps)
        if return_hidden:
            return x
        if self.logits_div != 1.0:                    # MiniCPM3: hidden / (hidden_size / dim_model_base)
            x = x / self.logits_div
        return self.lm_head(x.contiguous()).float()


def mla_from_hf(hf_model, dtype=None) -> Optional[MLACausalLM]:
    cfg = hf_model.config
    if getattr(cfg, "model_type", None) not in MLA_ARCHS:
        return None
    if getattr(hf_model, "_pp", None) is not None or getattr(hf_model, "_tp", None) is not None:
        return None
    base = hf_model.model
    emb_mod = base.embed_tokens
    emb = emb_mod.weight.data if isinstance(emb_mod, nn.Embedding) else emb_mod
    dt = dtype or (emb.dtype if isinstance(emb, torch.Tensor) else base.norm.weight.dtype)
    layers = []
    for L in base.layers:
        at = L.self_attn
        if not hasattr(at, "kv_a_proj_with_mqa"):
            return None
        layers.append(MLALayer(MLAAttention(at, cfg, dt), L.mlp, L.input_layernorm.weight.data,
                               L.post_attention_layernorm.weight.data))
    rot = base.rotary_emb
    inv_freq = rot.inv_freq.float()
    H = cfg.hidden_size
    spec = DecoderSpec(model_type=cfg.model_type, hidden_size=H, num_layers=len(layers),
                       num_heads=cfg.num_attention_heads, num_kv_heads=1,
                       head_dim=cfg.kv_lora_rank + cfg.qk_rope_head_dim,
                       intermediate_size=cfg.intermediate_size, vocab_size=cfg.vocab_size,
                       rms_eps=cfg.rms_norm_eps, rot_dim=cfg.qk_rope_head_dim,
                       max_position=cfg.max_position_embeddings)
    mt = cfg.model_type
    interleaved = mt == "deepseek_v2" or (mt == "deepseek_v3" and getattr(cfg, "rope_interleave", True))
    embed_scale = float(getattr(cfg, "scale_emb", 1.0) or 1.0) if mt == "minicpm3" else 1.0
    rs = 1.0
    if mt == "minicpm3":
        import math
        rs = cfg.scale_depth / math.sqrt(cfg.num_hidden_layers)
    model = MLACausalLM(spec, cfg, emb, layers, base.norm.weight.data, hf_model.get_output_embeddings(),
                        inv_freq.to(layers[0].input_layernorm.device), float(getattr(rot, "attention_scaling", 1.0)),
                        dt, interleaved, embed_scale, rs)
    if mt == "minicpm3":
        model.logits_div = float(getattr(cfg, "logits_scaling", None) or cfg.hidden_size / cfg.dim_model_base)
    return model.eval()
