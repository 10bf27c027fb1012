"""Native decoder for the non-llama block layouts.

Reference: the per-arch forwards of ``SRC/transformers/models/`` for bloom
(``bloom.py``: ALiBi + fused per-head QKV), mpt (``mpt.py``: ALiBi, bias-free
LayerNorm), gpt_bigcode / starcoder2 (``gptbigcode.py``, ``starcoder2.py``:
MQA, learned positions, biased LayerNorm MLPs), gpt-neox / phi / gpt-j /
falcon (parallel attention + MLP residual) and stablelm, hooked in by
``SRC/transformers/convert.py:1275-2139``.

MI355X design: these layouts differ from the llama decoder only in data --
norm kind (RMS / LayerNorm with or without bias), position scheme (RoPE
full / partial / interleaved, ALiBi slopes, learned absolute positions), the
residual wiring (sequential, parallel with one shared norm, parallel with two
norms), the MLP (GLU or fc -> act -> fc) and the order of the rows of a fused
QKV weight.  ``generic_pre`` rewrites every fused QKV into the ``[q; k; v]``
row order once, on the dense weights before quantization, so all of them run
the same kernels as the llama family: the low-bit skinny GEMV/GEMM for the
projections, ``rope_kv`` (an identity cos/sin table for ALiBi / learned
positions) appending K/V to the paged cache, the flash-decoding kernel (ALiBi
slopes added in-kernel) and the LayerNorm kernel.  A variant outside what is
covered here (qk-layernorm, clip_qkv, Falcon-RW ALiBi, ...) keeps the HF
forward over low-bit linears, with the original fused projection restored as
a view.
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .decoder import DecoderSpec, NativeAttention, NativeCausalLM, NativeMLP, compute_inv_freq

GENERIC_ARCHS = {"bloom", "mpt", "gpt_bigcode", "gpt2", "starcoder2", "gpt_neox", "phi", "falcon", "gptj",
                 "stablelm"}

# per model_type: module paths (after ``generic_pre``) of the pieces the native
# decoder reads.  ``ln2`` None: parallel residual with one shared norm.
_LAYOUT = {
    "bloom": dict(layers="transformer.h", attn="self_attention", o="dense", fc1="mlp.dense_h_to_4h",
                  fc2="mlp.dense_4h_to_h", ln1="input_layernorm", ln2="post_attention_layernorm",
                  embed="transformer.word_embeddings", embed_ln="transformer.word_embeddings_layernorm",
                  lnf="transformer.ln_f", qkv_src="query_key_value"),
    "mpt": dict(layers="transformer.blocks", attn="attn", o="out_proj", fc1="ffn.up_proj", fc2="ffn.down_proj",
                ln1="norm_1", ln2="norm_2", embed="transformer.wte", lnf="transformer.norm_f", qkv_src="Wqkv"),
    "gpt_bigcode": dict(layers="transformer.h", attn="attn", o="c_proj", fc1="mlp.c_fc", fc2="mlp.c_proj",
                        ln1="ln_1", ln2="ln_2", embed="transformer.wte", wpe="transformer.wpe",
                        lnf="transformer.ln_f", qkv_src="c_attn"),
    "gpt2": dict(layers="transformer.h", attn="attn", o="c_proj", fc1="mlp.c_fc", fc2="mlp.c_proj", ln1="ln_1",
                 ln2="ln_2", embed="transformer.wte", wpe="transformer.wpe", lnf="transformer.ln_f",
                 qkv_src="c_attn"),
    "starcoder2": dict(layers="model.layers", attn="self_attn", o="o_proj", fc1="mlp.c_fc", fc2="mlp.c_proj",
                       ln1="input_layernorm", ln2="post_attention_layernorm", embed="model.embed_tokens",
                       lnf="model.norm", qkv_src=("q_proj", "k_proj", "v_proj")),
    "gpt_neox": dict(layers="gpt_neox.layers", attn="attention", o="dense", fc1="mlp.dense_h_to_4h",
                     fc2="mlp.dense_4h_to_h", ln1="input_layernorm", ln2="post_attention_layernorm",
                     embed="gpt_neox.embed_in", lnf="gpt_neox.final_layer_norm", qkv_src="query_key_value"),
    "phi": dict(layers="model.layers", attn="self_attn", o="dense", fc1="mlp.fc1", fc2="mlp.fc2",
                ln1="input_layernorm", ln2=None, embed="model.embed_tokens", lnf="model.final_layernorm",
                qkv_src=("q_proj", "k_proj", "v_proj")),
    "falcon": dict(layers="transformer.h", attn="self_attention", o="dense", fc1="mlp.dense_h_to_4h",
                   fc2="mlp.dense_4h_to_h", ln1="input_layernorm", ln2="post_attention_layernorm",
                   embed="transformer.word_embeddings", lnf="transformer.ln_f", qkv_src="query_key_value"),
    "gptj": dict(layers="transformer.h", attn="attn", o="out_proj", fc1="mlp.fc_in", fc2="mlp.fc_out", ln1="ln_1",
                 ln2=None, embed="transformer.wte", lnf="transformer.ln_f", qkv_src=("q_proj", "k_proj", "v_proj")),
    "stablelm": dict(layers="model.layers", attn="self_attn", o="o_proj", gate_up="mlp.gate_up_proj",
                     fc2="mlp.down_proj", ln1="input_layernorm", ln2="post_attention_layernorm",
                     embed="model.embed_tokens", lnf="model.norm", qkv_src=("q_proj", "k_proj", "v_proj")),
}

# HF activation names -> (torch function, GLU kernel code or None)
_ACTS = {
    "gelu": (lambda x: F.gelu(x), None),
    "gelu_new": (lambda x: F.gelu(x, approximate="tanh"), 1),
    "gelu_pytorch_tanh": (lambda x: F.gelu(x, approximate="tanh"), 1),
    "gelu_fast": (lambda x: F.gelu(x, approximate="tanh"), 1),
    "bloom_gelu": (lambda x: F.gelu(x, approximate="tanh"), 1),
    "relu": (F.relu, None),
    "silu": (F.silu, 0),
    "swish": (F.silu, 0),
}


def _get(obj, path: str):
    for p in path.split("."):
        obj = getattr(obj, p, None)
        if obj is None:
            return None
    return obj


def _cfg(cfg, *names, default=None):
    for n in names:
        v = getattr(cfg, n, None)
        if v is not None:
            return v
    return default


def _rope_params(cfg) -> dict:
    p = getattr(cfg, "rope_parameters", None) or getattr(cfg, "rope_scaling", None) or {}
    return p if isinstance(p, dict) else {}


def alibi_slopes(n_heads: int, kind: str = "bloom", bias_max: float = 8.0) -> torch.Tensor:
    """Per-head ALiBi slopes.  ``bloom`` (also baichuan-13B / falcon-rw): the
    geometric series of the closest power of two, odd powers of the next one
    for the remaining heads; ``mpt``: 2^-(i * bias_max / n2), heads re-ordered
    odd-then-even when n is not a power of two."""
    if kind == "mpt":
        n2 = 2 ** math.ceil(math.log2(n_heads))
        s = [1.0 / 2 ** ((i + 1) * bias_max / n2) for i in range(n2)]
        if n2 != n_heads:
            s = (s[1::2] + s[::2])[:n_heads]
        return torch.tensor(s, dtype=torch.float32)
    c = 2 ** math.floor(math.log2(n_heads))
    base = 2.0 ** (-(2.0 ** -(math.log2(c) - 3)))
    s = [base ** (i + 1) for i in range(c)]
    if c != n_heads:
        eb = 2.0 ** (-(2.0 ** -(math.log2(2 * c) - 3)))
        s += [eb ** (2 * i + 1) for i in range(min(c, n_heads - c))]
    return torch.tensor(s, dtype=torch.float32)


def generic_supported(cfg) -> bool:
    mt = getattr(cfg, "model_type", None)
    if mt not in GENERIC_ARCHS:
        return False
    if mt in ("phi", "stablelm") and _cfg(cfg, "qk_layernorm", default=False):
        return False
    if mt == "mpt":
        ac = cfg.attn_config
        ac = ac if isinstance(ac, dict) else ac.to_dict()
        if ac.get("clip_qkv") or ac.get("qk_ln") or ac.get("prefix_lm") or not ac.get("alibi", True):
            return False
    if mt == "falcon" and _cfg(cfg, "alibi", default=False):
        return False
    if mt == "gpt2" and (_cfg(cfg, "scale_attn_by_inverse_layer_idx", default=False)
                         or _cfg(cfg, "reorder_and_upcast_attn", default=False)
                         or not _cfg(cfg, "scale_attn_weights", default=True)):
        return False
    if mt == "gpt_bigcode" and not _cfg(cfg, "scale_attn_weights", default=True):
        return False
    if mt == "stablelm" and _cfg(cfg, "use_parallel_residual", default=False):
        return False                     # (rare variant: keep the HF forward)
    return True


def generic_spec(cfg) -> DecoderSpec:
    mt = cfg.model_type
    H = _cfg(cfg, "hidden_size", "n_embd", "d_model")
    nh = _cfg(cfg, "num_attention_heads", "n_head", "n_heads")
    D = H // nh
    nkv = _cfg(cfg, "num_key_value_heads", default=nh) or nh
    if mt == "gpt_bigcode" and _cfg(cfg, "multi_query", default=True):
        nkv = 1
    if mt == "falcon":
        if cfg.new_decoder_architecture:
            nkv = _cfg(cfg, "num_kv_heads", default=nh)
        elif cfg.multi_query:
            nkv = 1
    rp = _rope_params(cfg)
    prf = rp.get("partial_rotary_factor", _cfg(cfg, "partial_rotary_factor", "rotary_pct", default=1.0))
    rot = int(D * prf)
    if mt == "gptj":
        rot = _cfg(cfg, "rotary_dim", default=D) or D
    inter = _cfg(cfg, "intermediate_size", "n_inner", "ffn_hidden_size", default=None) or 4 * H
    if mt == "mpt":
        inter = int(cfg.expansion_ratio * H)
    eps = _cfg(cfg, "layer_norm_eps", "layer_norm_epsilon", "norm_epsilon", "rms_norm_eps", default=1e-5)
    act = _cfg(cfg, "hidden_act", "activation_function", default="gelu")
    if mt == "bloom":
        act = "bloom_gelu"
    if mt in ("mpt", "falcon"):
        act = "gelu"
    s = DecoderSpec(model_type=mt, hidden_size=H, num_layers=_cfg(cfg, "num_hidden_layers", "n_layer", "n_layers"),
                    num_heads=nh, num_kv_heads=nkv, head_dim=D, intermediate_size=inter,
                    vocab_size=cfg.vocab_size, rms_eps=eps, rot_dim=rot,
                    max_position=_cfg(cfg, "max_position_embeddings", "n_positions", "max_seq_len", default=2048))
    s.norm_type = "layer"
    s.act_fn = act
    if act not in _ACTS:
        raise ValueError(f"{mt}: activation {act!r} not supported by the native decoder")
    s.act = 0 if _ACTS[act][1] == 0 else 1          # GLU kernel code (stablelm)
    s.rope_interleaved = mt == "gptj"
    s.pos_type = {"bloom": "alibi", "mpt": "alibi", "gpt_bigcode": "learned", "gpt2": "learned"}.get(mt, "rope")
    s.glu = mt == "stablelm"
    s.parallel_residual = "none"
    if mt == "gpt_neox" and _cfg(cfg, "use_parallel_residual", default=True):
        s.parallel_residual = "two"
    if mt in ("phi", "gptj"):
        s.parallel_residual = "shared"
    if mt == "falcon" and cfg.parallel_attn:
        two = cfg.new_decoder_architecture and (_cfg(cfg, "num_ln_in_parallel_attn", default=2) or 2) == 2
        s.parallel_residual = "two" if two else "shared"
    if mt == "starcoder2":
        sw = _cfg(cfg, "sliding_window", default=None)
        s.sliding_window = int(sw) if sw else 0
    if mt == "mpt":
        ac = cfg.attn_config if isinstance(cfg.attn_config, dict) else cfg.attn_config.to_dict()
        if ac.get("softmax_scale"):
            s.query_scale = float(ac["softmax_scale"])
    if s.pos_type != "rope":
        s.rot_dim = D
    s.tie_embeddings = bool(_cfg(cfg, "tie_word_embeddings", default=False))
    return s


# ----------------------------------------------------------------- pre-conversion
def _qkv_perm(mt: str, cfg, nh: int, nkv: int, D: int) -> Optional[List[int]]:
    """rows of the HF fused QKV weight in [q heads; k heads; v heads] order
    (None: already in that order)"""
    if mt in ("bloom", "gpt_neox") or (mt == "falcon" and not cfg.new_decoder_architecture
                                       and not cfg.multi_query) or \
            (mt == "gpt_bigcode" and not _cfg(cfg, "multi_query", default=True)):
        return [h * 3 * D + p * D + d for p in range(3) for h in range(nh) for d in range(D)]
    if mt == "falcon" and cfg.new_decoder_architecture:
        g = nh // nkv
        q = [j * (g + 2) * D + i * D + d for j in range(nkv) for i in range(g) for d in range(D)]
        k = [j * (g + 2) * D + g * D + d for j in range(nkv) for d in range(D)]
        v = [j * (g + 2) * D + (g + 1) * D + d for j in range(nkv) for d in range(D)]
        return q + k + v
    return None


def _linear_from(w: torch.Tensor, b: Optional[torch.Tensor]) -> nn.Linear:
    lin = nn.Linear(w.shape[1], w.shape[0], bias=b is not None, device="meta", dtype=w.dtype)
    lin.weight = nn.Parameter(w, requires_grad=False)
    if b is not None:
        lin.bias = nn.Parameter(b, requires_grad=False)
    return lin


def _conv1d_to_linear(m: nn.Module) -> nn.Module:
    if type(m).__name__ != "Conv1D":
        return m
    return _linear_from(m.weight.data.t().contiguous(), m.bias.data if m.bias is not None else None)


def generic_pre(model: nn.Module) -> bool:
    """Rewrite fused / split QKV weights into ``qkv_proj`` ([q; k; v] rows),
    gpt2's Conv1D projections into Linears, stablelm's gate/up into the
    interleaved GLU weight.  Returns False (model untouched) for unsupported
    variants."""
    cfg = model.config
    if not generic_supported(cfg):
        return False
    mt = cfg.model_type
    lay = _LAYOUT[mt]
    s = generic_spec(cfg)
    layers = _get(model, lay["layers"])
    if layers is None:
        return False
    from ..transformers.convert import _merge_gate_up, _merge_qkv
    for L in layers:
        attn = _get(L, lay["attn"])
        if mt == "gpt2":
            for path in ("attn.c_attn", "attn.c_proj", "mlp.c_fc", "mlp.c_proj"):
                parent, name = path.rsplit(".", 1)
                par = _get(L, parent)
                setattr(par, name, _conv1d_to_linear(getattr(par, name)))
        src = lay["qkv_src"]
        if hasattr(attn, "qkv_proj"):
            pass
        elif isinstance(src, tuple):
            _merge_qkv(attn)
        else:
            fused = getattr(attn, src)
            perm = _qkv_perm(mt, cfg, s.num_heads, s.num_kv_heads, s.head_dim)
            if type(fused).__name__ == "KQuantLinear":
                # GGUF k-quant blocks (gguf/api.py keep_kquant): permute whole block rows
                from ..transformers.low_bit_linear import KQuantLinear
                n = fused.out_features
                rows = fused.weight.data.view(n, -1)
                idx = torch.tensor(perm if perm is not None else list(range(n)), dtype=torch.long)
                b = fused.bias.data.index_select(0, idx) if fused.bias is not None else None
                attn.qkv_proj = KQuantLinear.from_blocks(rows.index_select(0, idx).reshape(-1), fused.qtype, n,
                                                         fused.in_features, bias=b)
                inv = [0] * n
                for i, r in enumerate(idx.tolist()):
                    inv[r] = i
                attn._illm_fused_src = (src, inv)
                delattr(attn, src)
                continue
            if not isinstance(fused, nn.Linear):
                return False
            w, b = fused.weight.data, fused.bias.data if fused.bias is not None else None
            if perm is not None:
                idx = torch.tensor(perm, dtype=torch.long, device=w.device)
                w = w.index_select(0, idx)
                b = b.index_select(0, idx) if b is not None else None
                inv = [0] * len(perm)
                for i, r in enumerate(perm):
                    inv[r] = i
            else:
                inv = list(range(w.shape[0]))
            attn.qkv_proj = _linear_from(w, b)
            attn._illm_fused_src = (src, inv)
            delattr(attn, src)
        if s.glu:
            _merge_gate_up(_get(L, "mlp"))
    model._illm_generic = True
    return True


def restore_generic_views(model: nn.Module):
    """HF forward over the rewritten weights (the native decoder declined)"""
    from ..transformers.hf_views import ProjView, restore_hf_views
    lay = _LAYOUT.get(model.config.model_type)
    for L in (_get(model, lay["layers"]) if lay else None) or []:
        attn = _get(L, lay["attn"])
        src = getattr(attn, "_illm_fused_src", None)
        if src is not None and not hasattr(attn, src[0]):
            setattr(attn, src[0], ProjView(attn, "qkv_proj", src[1], True))
    restore_hf_views(model)
    return model


# ----------------------------------------------------------------- model
class PlainMLP(nn.Module):
    """fc_in -> act -> fc_out (biases inside the low-bit linears)"""

    def __init__(self, fc_in: nn.Module, fc_out: nn.Module, act: str):
        super().__init__()
        self.fc_in, self.fc_out, self.act_name = fc_in, fc_out, act
        self.act = _ACTS[act][0]

    def forward(self, x):
        return self.fc_out(self.act(self.fc_in(x)).contiguous())


class GenericLayer(nn.Module):
    def __init__(self, attn: NativeAttention, mlp: nn.Module, ln1, ln1_b, ln2=None, ln2_b=None):
        super().__init__()
        self.self_attn, self.mlp = attn, mlp
        p = lambda t: nn.Parameter(t, requires_grad=False) if t is not None else None
        self.input_layernorm, self.input_layernorm_b = p(ln1), p(ln1_b)
        self.post_attention_layernorm, self.post_attention_layernorm_b = p(ln2), p(ln2_b)
        self.pre_feedforward_layernorm = self.post_feedforward_layernorm = None


class GenericCausalLM(NativeCausalLM):
    """LayerNorm / ALiBi / learned-position / parallel-residual decoders on
    the native kernels (same cache, engine, hipGraph decode and generate glue
    as :class:`NativeCausalLM`)."""

    def __init__(self, spec: DecoderSpec, embed, layers: List[GenericLayer], norm, norm_b, lm_head, inv_freq,
                 dtype, pos_embed=None, embed_ln=None, alibi=None):
        super().__init__(spec, embed, layers, norm, lm_head, inv_freq, dtype)
        p = lambda t: nn.Parameter(t, requires_grad=False) if t is not None else None
        self.norm_b = p(norm_b)
        self.pos_embed = p(pos_embed)
        self.embed_ln = p(embed_ln[0]) if embed_ln is not None else None
        self.embed_ln_b = p(embed_ln[1]) if embed_ln is not None else None
        self.__dict__.pop("alibi", None)
        self.register_buffer("alibi", alibi.float() if alibi is not None else None, persistent=False)

    def graph_max_batch(self) -> int:
        return super().graph_max_batch()

    def _norm(self, x, w, b):
        s = self.spec
        if s.norm_type == "layer":
            return ops.layer_norm(x.contiguous(), w, b, s.rms_eps)
        return ops.rms_norm(x.contiguous(), w, s.rms_eps, s.norm_unit_offset)

    def _ffn(self, x, mlp):
        if isinstance(mlp, NativeMLP):
            return mlp.down_proj(self._mlp(x, mlp))
        return mlp(x)

    def forward_tokens(self, ids: torch.Tensor, pos: torch.Tensor, slots: torch.Tensor, meta, cache,
                       logits_idx: Optional[torch.Tensor] = None, return_hidden: bool = False,
                       hidden_in: Optional[torch.Tensor] = None):
        s = self.spec
        if hidden_in is not None:
            h = hidden_in.to(self.dtype).contiguous()
        else:
            h = self.embed_module(ids).to(self.dtype) if self.embed_module is not None else \
                F.embedding(ids, self.embed_tokens)
            if self.pos_embed is not None:
                h = h + F.embedding(pos, self.pos_embed).to(h.dtype)
            if self.embed_ln is not None:
                h = self._norm(h, self.embed_ln, self.embed_ln_b)
        T = ids.shape[0]
        rope = self.rope_cache if self.rope_cache is not None else self.inv_freq
        for li, layer in enumerate(self.layers):
            attn = layer.self_attn
            x1 = self._norm(h, layer.input_layernorm, layer.input_layernorm_b)
            qkv = attn.qkv_proj(x1).contiguous()
            q = torch.empty(T, s.num_heads, s.head_dim, dtype=h.dtype, device=h.device)
            ops.rope_kv(qkv, q, cache.k[li], cache.v[li], slots, pos, rope, s.num_heads, s.num_kv_heads,
                        s.head_dim, s.rot_dim, s.rope_interleaved, None, None, s.rms_eps, 1.0, cache.kv_fp8,
                        cache.k_scale, cache.v_scale)
            a = attn.o_proj(self._attention(li, attn, q.view(T, -1), meta, cache))
            if s.parallel_residual == "none":
                h = h + a
                h = h + self._ffn(self._norm(h, layer.post_attention_layernorm, layer.post_attention_layernorm_b),
                                  layer.mlp)
            else:
                x2 = x1 if s.parallel_residual == "shared" else \
                    self._norm(h, layer.post_attention_layernorm, layer.post_attention_layernorm_b)
                h = h + (a + self._ffn(x2, layer.mlp))
        if not self.last_stage:
            return h
        if logits_idx is not None:
            h = h.index_select(0, logits_idx)
        x = self._norm(h, self.norm, self.norm_b)
        if return_hidden:
            return x
        return self.lm_head(x.contiguous()).float()


def _ln(mod):
    if mod is None:
        return None, None
    return mod.weight.data if mod.weight is not None else None, \
        mod.bias.data if getattr(mod, "bias", None) is not None else None


def generic_from_hf(hf_model, dtype=None) -> Optional[GenericCausalLM]:
    cfg = hf_model.config
    mt = getattr(cfg, "model_type", None)
    if mt not in GENERIC_ARCHS or not getattr(hf_model, "_illm_generic", False):
        return None
    if getattr(hf_model, "_pp", None) is not None or getattr(hf_model, "_tp", None) is not None:
        return None
    lay = _LAYOUT[mt]
    spec = generic_spec(cfg)
    layers = []
    for L in _get(hf_model, lay["layers"]):
        at = _get(L, lay["attn"])
        if not hasattr(at, "qkv_proj"):
            return None
        attn = NativeAttention(spec, at.qkv_proj, _get(at, lay["o"]), sliding_window=spec.sliding_window)
        if spec.glu:
            mlp = NativeMLP(spec, _get(L, lay["gate_up"]), _get(L, lay["fc2"]))
        else:
            mlp = PlainMLP(_get(L, lay["fc1"]), _get(L, lay["fc2"]), spec.act_fn)
        ln1n, ln2n = lay["ln1"], lay["ln2"]
        if mt == "falcon":
            if spec.parallel_residual == "two":
                ln1n, ln2n = "ln_attn", "ln_mlp"
            elif spec.parallel_residual == "shared":
                ln2n = None
        ln1 = _ln(_get(L, ln1n))
        ln2 = _ln(_get(L, ln2n)) if ln2n else (None, None)
        if ln1[0] is None:
            return None
        layers.append(GenericLayer(attn, mlp, ln1[0], ln1[1], ln2[0], ln2[1]))
    emb_mod = _get(hf_model, lay["embed"])
    emb = emb_mod.weight.data if isinstance(emb_mod, nn.Embedding) else emb_mod
    wpe = _get(hf_model, lay["wpe"]).weight.data if lay.get("wpe") else None
    eln = _ln(_get(hf_model, lay["embed_ln"])) if lay.get("embed_ln") else None
    nf = _ln(_get(hf_model, lay["lnf"]))
    lm_head = hf_model.get_output_embeddings()
    dev = layers[0].input_layernorm.device
    alibi = None
    if spec.pos_type == "alibi":
        if mt == "mpt":
            ac = cfg.attn_config if isinstance(cfg.attn_config, dict) else cfg.attn_config.to_dict()
            alibi = alibi_slopes(spec.num_heads, "mpt", ac.get("alibi_bias_max", 8))
        else:
            alibi = alibi_slopes(spec.num_heads)
        alibi = alibi.to(dev)
    if spec.pos_type == "rope":
        import copy
        c2 = copy.copy(cfg)
        if mt == "gptj":
            c2.rope_parameters = {"rope_type": "default", "rope_theta": 10000.0}
        inv_freq, att_scale = compute_inv_freq(c2, spec.head_dim, spec.rot_dim)
        spec.rope_attention_scaling = att_scale
    else:
        inv_freq = torch.zeros(spec.head_dim // 2)       # identity rotation: rope_kv only appends K/V
    model = GenericCausalLM(spec, emb, layers, nf[0], nf[1], lm_head, inv_freq.to(dev),
                            dtype or (emb.dtype if isinstance(emb, torch.Tensor) else layers[0].input_layernorm.dtype),
                            pos_embed=wpe, embed_ln=eln, alibi=alibi)
    return model.eval()
