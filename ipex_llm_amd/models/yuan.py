"""Yuan 2.0: localized-filtering attention (LFA).

Reference: ``SRC/transformers/gguf/models/yuan2.py:29-130`` (GGUF loader
building the remote-code ``YuanForCausalLM``), the remote-code layer
``gguf/models/model_implement/yuan2/yuan_hf_model.py:46-384`` and the
optimized forward ``SRC/transformers/models/yuan.py:35-200`` (q/k merged,
conv weights in half precision, the last two hidden states kept in the
cache for the decode-step convolutions).

The architecture, in the terms used here (h = input_layernorm output):

    o1[t] = C1a h[t-1] + C1b h[t] + b1            conv1, kernel 2 (H -> H/2)
    o2[t] = C2a o1[t-1] + C2b o1[t] + b2          conv2, kernel 2 (H/2 -> H)
    f[t]  = rms_norm(o2[t] + h[t]) * w_lf
    [q | k] = [Wq; Wk] f, viewed per head as [nh, 2, hd] (head i's query is
              the first half of row block i of the concatenation, its key
              the second half) ; v = Wv h
    rotate_half RoPE (theta 10000), MHA, o_proj, SiLU GLU MLP

Two pieces here:

* :class:`YuanForCausalLM` -- a self-contained PyTorch model of that
  architecture with the remote-code module names (so a GGUF file or an HF
  checkpoint maps onto it without remote code), full-sequence forward.
  It is the parity reference and the model the converter starts from.
* :class:`YuanLF` -- the native decoder's form (models/decoder.py): the
  two convolutions as linears over [previous; current] rows, and an
  ``lf`` cache per layer that stores h and o1 of EVERY position in the
  paged-cache slot layout (``[slots + 1, H + H/2]``, the extra row is the
  zero "position -1").  A step gathers the previous position's rows via the
  block table, so chunked prefill, batched decode, speculative verify and
  hipGraph capture all work unchanged (no per-sequence host state; the
  reference keeps ``hidden_states[-2:]`` per request instead).
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

try:
    from transformers import PretrainedConfig, PreTrainedModel
    from transformers.generation import GenerationMixin
    from transformers.modeling_outputs import CausalLMOutputWithPast
except ImportError:  # pragma: no cover
    PretrainedConfig = object
    PreTrainedModel = nn.Module
    GenerationMixin = object
    CausalLMOutputWithPast = None


class YuanConfig(PretrainedConfig):
    model_type = "yuan"

    def __init__(self, vocab_size=135040, hidden_size=2048, intermediate_size=8192, num_hidden_layers=24,
                 num_attention_heads=32, hidden_act="silu", max_position_embeddings=8192, rms_norm_eps=1e-6,
                 rope_theta=10000.0, tie_word_embeddings=False, initializer_range=0.02, use_cache=True,
                 pad_token_id=None, bos_token_id=None, eos_token_id=None, **kw):
        self.vocab_size = vocab_size
        self.hidden_size = hidden_size
        self.intermediate_size = intermediate_size
        self.num_hidden_layers = num_hidden_layers
        self.num_attention_heads = num_attention_heads
        self.num_key_value_heads = num_attention_heads
        self.hidden_act = hidden_act
        self.max_position_embeddings = max_position_embeddings
        self.rms_norm_eps = rms_norm_eps
        self.rope_theta = rope_theta
        self.initializer_range = initializer_range
        self.use_cache = use_cache
        kw.pop("num_key_value_heads", None)
        super().__init__(pad_token_id=pad_token_id, bos_token_id=bos_token_id, eos_token_id=eos_token_id,
                         tie_word_embeddings=tie_word_embeddings, **kw)


class YuanRMSNorm(nn.Module):
    def __init__(self, n, eps=1e-6):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(n))
        self.variance_epsilon = eps

    def forward(self, x):
        xf = x.float()
        xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.variance_epsilon)
        return self.weight * xf.to(x.dtype)


def _shift(x: torch.Tensor) -> torch.Tensor:
    """[B, S, C] -> the previous position's rows (zeros at position 0)"""
    return F.pad(x, (0, 0, 1, 0))[:, :-1]


class YuanLocalizedFiltering(nn.Module):
    """two causal kernel-2 convolutions along the sequence + residual RMSNorm
    (Conv2d modules: the checkpoint layout [out, in, 2, 1])"""

    def __init__(self, hidden_size: int, eps: float = 1e-6):
        super().__init__()
        self.embed_dim = hidden_size
        self.conv1 = nn.Conv2d(hidden_size, hidden_size // 2, (2, 1), padding=(1, 0))
        self.conv2 = nn.Conv2d(hidden_size // 2, hidden_size, (2, 1), padding=(1, 0))
        self.output_layernorm = YuanRMSNorm(hidden_size, eps)

    @staticmethod
    def _conv(x, conv):
        w = conv.weight[:, :, :, 0]                          # [out, in, 2]: tap 0 = previous, tap 1 = current
        return F.linear(_shift(x), w[:, :, 0]) + F.linear(x, w[:, :, 1], conv.bias)

    def forward(self, h):                                    # [B, S, H]
        o1 = self._conv(h, self.conv1)
        o2 = self._conv(o1, self.conv2)
        return self.output_layernorm(o2 + h)


def _rotate_half(x):
    a, b = x.chunk(2, -1)
    return torch.cat([-b, a], -1)


class YuanAttention(nn.Module):
    def __init__(self, cfg: YuanConfig):
        super().__init__()
        H, nh = cfg.hidden_size, cfg.num_attention_heads
        self.num_heads, self.head_dim = nh, H // nh
        self.q_proj = nn.Linear(H, H, bias=False)
        self.k_proj = nn.Linear(H, H, bias=False)
        self.v_proj = nn.Linear(H, H, bias=False)
        self.o_proj = nn.Linear(H, H, bias=False)
        self.lf_gate = YuanLocalizedFiltering(H, cfg.rms_norm_eps)
        self.rope_theta = getattr(cfg, "rope_theta", 10000.0)

    def forward(self, h, pos):
        B, S, H = h.shape
        nh, hd = self.num_heads, self.head_dim
        v = self.v_proj(h).view(B, S, nh, hd).transpose(1, 2)
        f = self.lf_gate(h)
        qk = self.qk_proj(f) if hasattr(self, "qk_proj") else torch.cat([self.q_proj(f), self.k_proj(f)], -1)
        qk = qk.view(B, S, nh, 2, hd)
        q, k = qk[:, :, :, 0].transpose(1, 2), qk[:, :, :, 1].transpose(1, 2)
        inv = 1.0 / (self.rope_theta ** (torch.arange(0, hd, 2, device=h.device, dtype=torch.float32) / hd))
        fr = pos.float()[:, None] * inv[None]
        emb = torch.cat([fr, fr], -1)
        cos, sin = emb.cos().to(q.dtype), emb.sin().to(q.dtype)
        q = q * cos + _rotate_half(q) * sin
        k = k * cos + _rotate_half(k) * sin
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True, scale=1.0 / math.sqrt(hd))
        return self.o_proj(o.transpose(1, 2).reshape(B, S, H))


class YuanMLP(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.gate_proj = nn.Linear(cfg.hidden_size, cfg.intermediate_size, bias=False)
        self.up_proj = nn.Linear(cfg.hidden_size, cfg.intermediate_size, bias=False)
        self.down_proj = nn.Linear(cfg.intermediate_size, cfg.hidden_size, bias=False)

    def forward(self, x):
        return self.down_proj(F.silu(self.gate_proj(x)) * self.up_proj(x))


class YuanDecoderLayer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.self_attn = YuanAttention(cfg)
        self.mlp = YuanMLP(cfg)
        self.input_layernorm = YuanRMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.post_attention_layernorm = YuanRMSNorm(cfg.hidden_size, cfg.rms_norm_eps)

    def forward(self, x, pos):
        x = x + self.self_attn(self.input_layernorm(x), pos)
        return x + self.mlp(self.post_attention_layernorm(x))


class YuanPreTrainedModel(PreTrainedModel):
    config_class = YuanConfig
    base_model_prefix = "model"
    _no_split_modules = ["YuanDecoderLayer"]

    def _init_weights(self, m):
        std = getattr(self.config, "initializer_range", 0.02)
        if isinstance(m, (nn.Linear, nn.Conv2d)):
            m.weight.data.normal_(0.0, std)
            if m.bias is not None:
                m.bias.data.zero_()
        elif isinstance(m, nn.Embedding):
            m.weight.data.normal_(0.0, std)
        elif isinstance(m, YuanRMSNorm):
            m.weight.data.fill_(1.0)


class YuanModel(YuanPreTrainedModel):
    def __init__(self, cfg):
        super().__init__(cfg)
        self.embed_tokens = nn.Embedding(cfg.vocab_size, cfg.hidden_size)
        self.layers = nn.ModuleList([YuanDecoderLayer(cfg) for _ in range(cfg.num_hidden_layers)])
        self.norm = YuanRMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.post_init()

    def forward(self, input_ids):
        x = self.embed_tokens(input_ids)
        pos = torch.arange(input_ids.shape[1], device=input_ids.device)
        for L in self.layers:
            x = L(x, pos)
        return self.norm(x)


class YuanForCausalLM(YuanPreTrainedModel, GenerationMixin):
    """full-recompute forward (no KV cache): the parity reference; the
    converted model runs on the native decoder (cached, fused kernels)"""
    _tied_weights_keys = {"lm_head.weight": "model.embed_tokens.weight"}

    def __init__(self, cfg):
        super().__init__(cfg)
        self.model = YuanModel(cfg)
        self.lm_head = nn.Linear(cfg.hidden_size, cfg.vocab_size, bias=False)
        self.post_init()

    def get_input_embeddings(self):
        return self.model.embed_tokens

    def get_output_embeddings(self):
        return self.lm_head

    def forward(self, input_ids=None, attention_mask=None, labels=None, **kw):
        logits = self.lm_head(self.model(input_ids)).float()
        loss = None
        if labels is not None:
            loss = F.cross_entropy(logits[:, :-1].reshape(-1, logits.shape[-1]), labels[:, 1:].reshape(-1),
                                   ignore_index=-100)
        return CausalLMOutputWithPast(loss=loss, logits=logits)


def yuan_config_from_remote(c: dict) -> YuanConfig:
    """remote-code Yuan config.json -> YuanConfig (only the LFA layout: the
    ``use_shareqk`` variant is refused)"""
    if c.get("use_shareqk"):
        raise NotImplementedError("Yuan use_shareqk checkpoints are not supported")
    keep = ("vocab_size", "hidden_size", "intermediate_size", "num_hidden_layers", "num_attention_heads",
            "hidden_act", "max_position_embeddings", "rms_norm_eps", "rope_theta", "tie_word_embeddings",
            "pad_token_id", "bos_token_id", "eos_token_id")
    return YuanConfig(**{k: c[k] for k in keep if c.get(k) is not None})


def register():
    """make ``AutoConfig`` / ``AutoModelForCausalLM`` know model_type "yuan" (idempotent)"""
    from transformers import AutoConfig, AutoModelForCausalLM
    try:
        AutoConfig.register("yuan", YuanConfig)
    except ValueError:
        pass
    try:
        AutoModelForCausalLM.register(YuanConfig, YuanForCausalLM)
    except ValueError:
        pass


# ---------------------------------------------------------------- native form
class YuanLF(nn.Module):
    """the LFA q/k/v producer of one native layer (see the module docstring)"""

    def __init__(self, conv1: nn.Module, conv2: nn.Module, norm_w: torch.Tensor, eps: float,
                 qk_proj: nn.Module, v_proj: nn.Module, num_heads: int, head_dim: int):
        super().__init__()
        self.conv1, self.conv2 = conv1, conv2                # linears over [previous; current]
        self.norm_w = nn.Parameter(norm_w, requires_grad=False)
        self.eps = eps
        self.qk_proj, self.v_proj = qk_proj, v_proj
        self.num_heads, self.head_dim = num_heads, head_dim
        self.H = conv2.out_features

    @staticmethod
    def conv_linear(conv: nn.Conv2d, dtype, device) -> nn.Module:
        """Conv2d [out, in, 2, 1] -> dense linear [out, 2 in] over [prev; cur]
        (half precision, as the reference keeps the convolutions)"""
        from ..transformers.low_bit_linear import DenseLinear
        w = conv.weight.data[:, :, :, 0]
        lin = DenseLinear(2 * w.shape[1], w.shape[0], conv.bias is not None, dtype, "meta")
        lin.weight = nn.Parameter(torch.cat([w[:, :, 0], w[:, :, 1]], 1).to(device, dtype).contiguous(),
                                  requires_grad=False)
        if conv.bias is not None:
            lin.bias = nn.Parameter(conv.bias.data.to(device, dtype), requires_grad=False)
        return lin

    @staticmethod
    def prev_slots(slots, pos, meta, bs: int, zero_row: int) -> torch.Tensor:
        """cache slot of each token's previous position (zero_row at position 0)"""
        T = slots.shape[0]
        b = torch.arange(T, device=slots.device) // meta.Tq
        pp = pos.long() - 1
        if meta.pos_offset is not None:              # compressed KV: cache index = position - offset
            pp = pp - meta.pos_offset.long()[b]
        pp = pp.clamp_min(0)
        blk = meta.block_tables.long()[b, pp // bs]
        ps = blk * bs + pp % bs
        return torch.where(pos.long() > 0, ps, torch.full_like(ps, zero_row))

    def qkv(self, x: torch.Tensor, lfc: torch.Tensor, slots, pos, meta, bs: int) -> torch.Tensor:
        """x: [T, H] input_layernorm output -> [T, 3 nh hd] (q | k | v rows)"""
        from .. import ops
        H, T = self.H, x.shape[0]
        zero_row = lfc.shape[0] - 1
        sl = slots.long()
        lfc[sl, :H] = x
        prev = self.prev_slots(slots, pos, meta, bs, zero_row)
        o1 = self.conv1(torch.cat([lfc[prev, :H], x], -1))
        lfc[sl, H:] = o1.to(lfc.dtype)
        o2 = self.conv2(torch.cat([lfc[prev, H:], o1.to(lfc.dtype)], -1))
        f = ops.rms_norm((o2.float() + x.float()).to(x.dtype), self.norm_w, self.eps)
        qk = self.qk_proj(f).view(T, self.num_heads, 2, self.head_dim)
        v = self.v_proj(x)
        return torch.cat([qk[:, :, 0].reshape(T, -1), qk[:, :, 1].reshape(T, -1), v.reshape(T, -1)], -1)


def yuan_lf_from_hf(at: nn.Module, eps: float, dtype, device) -> YuanLF:
    """HF YuanAttention (converted: qk_proj = [q; k] rows, v_proj) -> YuanLF"""
    lf = at.lf_gate
    qk = getattr(at, "qk_proj", None)
    if qk is None:
        raise ValueError("yuan attention without the merged qk_proj (convert with ipex_llm_amd)")
    H = lf.embed_dim
    return YuanLF(YuanLF.conv_linear(lf.conv1, dtype, device), YuanLF.conv_linear(lf.conv2, dtype, device),
                  lf.output_layernorm.weight.data.to(device, dtype), eps, qk, at.v_proj,
                  at.num_heads, H // at.num_heads)
