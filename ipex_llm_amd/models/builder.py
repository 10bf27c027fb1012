"""Build a :class:`NativeCausalLM` from an HF config / model / state dict.

* ``spec_from_config``     HF config -> DecoderSpec (per model_type quirks)
* ``native_from_hf``       converted HF model -> NativeCausalLM sharing its
                           (already low-bit) modules -- the ``_optimize_post``
                           step of the reference (convert.py:1275-2139)
* ``random_native_model``  random-init weights generated and quantized on
                           the GPU layer by layer (BASELINE: synthetic data /
                           random-init weights; an 8B model builds in seconds)
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn

from .. import ops
from ..quantize import qtypes as Q
from ..transformers.low_bit_linear import LowBitLinear, DenseLinear
from .decoder import (DecoderSpec, NativeAttention, NativeCausalLM, NativeLayer, NativeMLP,
                      compute_inv_freq, interleave_glu_rows)

# model types executed by the native decoder (others fall back to the HF
# forward with low-bit linears, like the reference does for e.g. mixtral)
NATIVE_DENSE = {"llama", "mistral", "qwen2", "qwen3", "gemma", "gemma2", "phi3", "internlm2", "yi",
                "aquila", "olmo2", "deepseek", "minicpm", "baichuan", "yuan", "glm", "glm4"}
NATIVE_MOE = {"mixtral", "qwen2_moe", "qwen3_moe"}


def _get(cfg, *names, default=None):
    for n in names:
        v = getattr(cfg, n, None)
        if v is not None:
            return v
    return default


def spec_from_config(cfg) -> DecoderSpec:
    mt = getattr(cfg, "model_type", "llama")
    H = cfg.hidden_size
    nh = cfg.num_attention_heads
    nkv = _get(cfg, "num_key_value_heads", default=nh)
    hd = _get(cfg, "head_dim", default=H // nh) or H // nh
    rp = _get(cfg, "rope_parameters", default=None)
    prf = _get(cfg, "partial_rotary_factor", default=None) or \
        (rp.get("partial_rotary_factor") if isinstance(rp, dict) else None) or 1.0
    act_name = _get(cfg, "hidden_act", "hidden_activation", default="silu")
    spec = DecoderSpec(
        model_type=mt, hidden_size=H, num_layers=cfg.num_hidden_layers, num_heads=nh, num_kv_heads=nkv,
        head_dim=hd, intermediate_size=_get(cfg, "intermediate_size", default=4 * H),
        vocab_size=cfg.vocab_size, rms_eps=_get(cfg, "rms_norm_eps", "layer_norm_eps", default=1e-6),
        rot_dim=int(hd * prf), max_position=_get(cfg, "max_position_embeddings", default=8192),
        qkv_bias=bool(_get(cfg, "attention_bias", default=mt in ("qwen2", "qwen2_moe"))),
        mlp_bias=bool(_get(cfg, "mlp_bias", default=False)),
        qk_norm=mt in ("qwen3", "qwen3_moe", "olmo2"),
        act=0 if "silu" in str(act_name) or "swish" in str(act_name) else 1,
        tie_embeddings=bool(_get(cfg, "tie_word_embeddings", default=False)),
    )
    if mt in ("qwen2", "qwen2_moe"):
        spec.qkv_bias = True
    if mt in ("glm", "glm4"):
        # GLM / ChatGLM-4: RoPE on the first half of each head, rotating
        # interleaved pairs (SRC/transformers/models/chatglm4.py:163-205)
        spec.rope_interleaved = True
    if mt == "glm4":
        spec.sandwich_norm = True         # post_self_attn / post_mlp norms
    if mt in ("gemma", "gemma2", "gemma3_text"):
        spec.embed_scale = math.sqrt(H)
        spec.norm_unit_offset = True
        spec.tie_embeddings = True
    if mt in ("gemma2", "gemma3_text"):
        spec.sandwich_norm = True
        spec.attn_softcap = _get(cfg, "attn_logit_softcapping", default=0.0) or 0.0
        spec.final_softcap = _get(cfg, "final_logit_softcapping", default=0.0) or 0.0
        qps = _get(cfg, "query_pre_attn_scalar", default=None)
        if qps:
            spec.query_scale = qps ** -0.5
    sw = _get(cfg, "sliding_window", default=None)
    use_sw = _get(cfg, "use_sliding_window", default=mt in ("mistral", "mixtral", "gemma2", "phi3"))
    if sw and use_sw:
        spec.sliding_window = int(sw)
        if mt == "gemma2":  # alternate local / global layers
            spec.sliding_window_layers = [(i % 2 == 0) for i in range(spec.num_layers)]
    if mt in NATIVE_MOE:
        spec.num_experts = _get(cfg, "num_local_experts", "num_experts", default=0)
        spec.top_k = _get(cfg, "num_experts_per_tok", default=2)
        spec.moe_intermediate = _get(cfg, "moe_intermediate_size", default=spec.intermediate_size)
        spec.norm_topk = bool(_get(cfg, "norm_topk_prob", default=mt == "mixtral"))
        spec.shared_expert_intermediate = _get(cfg, "shared_expert_intermediate_size", default=0) or 0
        step = _get(cfg, "decoder_sparse_step", default=1) or 1
        only = _get(cfg, "mlp_only_layers", default=[]) or []
        spec.moe_layer_mask = [(i not in only) and ((i + 1) % step == 0) for i in range(spec.num_layers)]
    return spec


def lowbit_from_dense(w: torch.Tensor, qtype, device, bias: Optional[torch.Tensor] = None,
                      imatrix=None) -> nn.Module:
    qtype = Q.resolve_qtype(qtype)
    if Q.is_dense(qtype):
        dt = torch.bfloat16 if qtype == Q.BF16 else torch.float16
        m = DenseLinear(w.shape[1], w.shape[0], bias is not None, dt, "meta")
        m.weight = nn.Parameter(w.to(device, dt), requires_grad=False)
        if bias is not None:
            m.bias = nn.Parameter(bias.to(device, dt), requires_grad=False)
        return m
    if qtype in (Q.TORCH_FP8E4, Q.TORCH_FP8E5):
        from ..transformers.low_bit_linear import TorchFp8Linear
        lin = nn.Linear(w.shape[1], w.shape[0], bias=bias is not None, device="meta")
        lin.weight = nn.Parameter(w, requires_grad=False)
        if bias is not None:
            lin.bias = nn.Parameter(bias, requires_grad=False)
        return TorchFp8Linear.from_linear(lin, qtype, device=device)
    f = Q.get_format(qtype)
    if f is not None and f.kquant:
        from ..transformers.low_bit_linear import KQuantLinear
        m = KQuantLinear(w.shape[1], w.shape[0], qtype, bias=False, device="meta")
        m.load_dense(w, device=device, imatrix=imatrix)
        if bias is not None:
            m.bias = nn.Parameter(bias.detach().to(device), requires_grad=False)
        return m
    m = LowBitLinear(w.shape[1], w.shape[0], qtype, bias=False, device="meta")
    m.load_dense(w, device=device, imatrix=imatrix)
    if bias is not None:
        m.bias = nn.Parameter(bias.detach().to(device), requires_grad=False)
    return m


@torch.no_grad()
def random_native_model(cfg, qtype="sym_int4", device="cuda", dtype=torch.bfloat16, seed: int = 0,
                        lm_head_qtype=None, std: float = 0.02, tp_group=None, ep_group=None,
                        tp_shard_lm_head: bool = True, ep_tokens: bool = False,
                        ep_max_tokens: Optional[int] = None) -> NativeCausalLM:
    """Random-init model of ``cfg``'s architecture, quantized on ``device``.

    ``tp_group``: tensor parallel (AutoTP layout, SRC example
    ``Deepspeed-AutoTP/deepspeed_autotp.py:81-106``): every rank draws the SAME
    full-size random weights (one seed) and keeps/quantizes its shard -- whole
    query heads and their KV heads (column-parallel qkv), the matching o_proj
    columns (row-parallel, all-reduced), an I / world slice of gate/up
    (column) and down (row), a vocab slice of lm_head (logits all-gathered).
    ``ep_group``: expert parallel -- rank r keeps experts [r E/W, (r+1) E/W);
    ``ep_tokens``: token-sharded EP (each rank runs its own sequences, MoE
    pairs travel through ``parallel.ep``'s exact all-to-all; collective) --
    otherwise every rank sees all tokens and the MoE output is all-reduced.
    Either way the result equals the single-GPU model of the same seed."""
    spec = spec_from_config(cfg)
    s = spec
    g = torch.Generator(device=device).manual_seed(seed)
    W = R = 1
    if tp_group is not None:
        import torch.distributed as dist
        W, R = dist.get_world_size(tp_group), dist.get_rank(tp_group)
    if W > 1:
        if s.num_heads % W or s.intermediate_size % (16 * W):
            raise ValueError(f"tensor parallel {W}: heads {s.num_heads} / intermediate {s.intermediate_size}")
        if s.num_kv_heads % W and W % s.num_kv_heads:
            raise ValueError(f"tensor parallel {W}: {s.num_kv_heads} KV heads")

    def rnd(*shape, scale=std):
        return (torch.randn(*shape, generator=g, device=device, dtype=torch.float32) * scale).to(dtype)

    def ones_ish(n):
        return (1.0 + rnd(n, scale=0.02).float()).to(dtype) if not s.norm_unit_offset else rnd(n, scale=0.02)

    D = s.head_dim
    nq, nkv = s.num_heads * D, s.num_kv_heads * D
    hq = s.num_heads // W                                   # local query heads
    if s.num_kv_heads % W == 0:
        kv0, hkv = R * (s.num_kv_heads // W), s.num_kv_heads // W
    else:                                                   # fewer KV heads than ranks: replicate
        kv0, hkv = (R * hq) // (s.num_heads // s.num_kv_heads), 1
    Il = s.intermediate_size // W
    mp = tp_group if W > 1 else None
    layers = []
    for li in range(s.num_layers):
        wqkv = rnd(nq + 2 * nkv, s.hidden_size)
        bqkv = rnd(nq + 2 * nkv) if s.qkv_bias else None
        if W > 1:
            rows = torch.cat([torch.arange(R * hq * D, (R + 1) * hq * D),
                              nq + torch.arange(kv0 * D, (kv0 + hkv) * D),
                              nq + nkv + torch.arange(kv0 * D, (kv0 + hkv) * D)]).to(wqkv.device)
            wqkv = wqkv.index_select(0, rows)
            bqkv = bqkv.index_select(0, rows) if bqkv is not None else None
        qkv = lowbit_from_dense(wqkv, qtype, device, bqkv)
        del wqkv
        wo = rnd(s.hidden_size, nq)
        if W > 1:
            wo = wo[:, R * hq * D:(R + 1) * hq * D]
        o = lowbit_from_dense(wo.contiguous(), qtype, device)
        o.mp_group = mp
        if s.is_moe_layer(li):
            mlp = _random_moe(s, qtype, device, rnd, ep_group)
        else:
            wg, wu = rnd(s.intermediate_size, s.hidden_size), rnd(s.intermediate_size, s.hidden_size)
            wd = rnd(s.hidden_size, s.intermediate_size)
            if W > 1:
                wg, wu, wd = wg[R * Il:(R + 1) * Il], wu[R * Il:(R + 1) * Il], wd[:, R * Il:(R + 1) * Il]
            gu = lowbit_from_dense(interleave_glu_rows(wg.contiguous(), wu.contiguous()), qtype, device)
            down = lowbit_from_dense(wd.contiguous(), qtype, device)
            down.mp_group = mp
            mlp = NativeMLP(s, gu, down)
        attn = NativeAttention(s, qkv, o, ones_ish(s.head_dim) if s.qk_norm else None,
                               ones_ish(s.head_dim) if s.qk_norm else None, s.sliding_window)
        layers.append(NativeLayer(s, attn, mlp, ones_ish(s.hidden_size), ones_ish(s.hidden_size)))
        torch.cuda.empty_cache() if torch.device(device).type == "cuda" else None
    embed = rnd(s.vocab_size, s.hidden_size)
    head_w = embed if s.tie_embeddings else rnd(s.vocab_size, s.hidden_size)
    if W > 1 and tp_shard_lm_head:
        from ..parallel.tp import VocabParallelHead
        per = (s.vocab_size + W - 1) // W
        a, b = R * per, min(s.vocab_size, (R + 1) * per)
        hw = torch.zeros(per, s.hidden_size, dtype=head_w.dtype, device=head_w.device)
        hw[:b - a] = head_w[a:b]
        lm_head = VocabParallelHead(lowbit_from_dense(hw, lm_head_qtype or qtype, device), tp_group, s.vocab_size)
    else:
        lm_head = lowbit_from_dense(head_w, lm_head_qtype or qtype, device)
    inv_freq, att_scale = compute_inv_freq(cfg, s.head_dim, s.rot_dim or s.head_dim)
    s.rope_attention_scaling = att_scale
    if W > 1:
        import copy
        s = copy.copy(s)
        s.num_heads, s.num_kv_heads = hq, hkv
        for L in layers:
            L.self_attn.spec = s
            L.mlp.spec = s
    model = NativeCausalLM(s, embed, layers, ones_ish(spec.hidden_size), lm_head, inv_freq.to(device), dtype)
    if W > 1:
        model.tp_group = tp_group
    if ep_group is not None and ep_tokens:
        from ..parallel.ep import enable_token_sharded_ep
        enable_token_sharded_ep(model, ep_max_tokens)
    return model.eval()


@torch.no_grad()
def _random_moe(s: DecoderSpec, qtype, device, rnd, ep_group=None) -> nn.Module:
    """random-init sparse MoE block (router, E experts quantized one by one on
    the device, optional shared expert + gate) of ``s``'s geometry; with an EP
    group only this rank's experts are kept (all are drawn: same weights as
    the single-GPU model)"""
    from .moe import LowBitExperts, NativeMoE, SharedExpertMLP
    E, I, H = s.num_experts, s.moe_intermediate, s.hidden_size
    e0, El = 0, E
    if ep_group is not None:
        import torch.distributed as dist
        W, R = dist.get_world_size(ep_group), dist.get_rank(ep_group)
        if E % W:
            raise ValueError(f"expert parallel {W}: {E} experts")
        El = E // W
        e0 = R * El
    fmt = Q.get_format(qtype).fmt
    gu = LowBitExperts(El, 2 * I, H, qtype, "meta")
    dn = LowBitExperts(El, H, I, qtype, "meta")
    gub, dnb = [], []
    for e in range(E):
        wg = interleave_glu_rows(rnd(I, H), rnd(I, H))
        if e0 <= e < e0 + El:
            gub.append(ops.quantize(wg, fmt))
    for e in range(E):
        wd = rnd(H, I)
        if e0 <= e < e0 + El:
            dnb.append(ops.quantize(wd, fmt))
    gu.weight = nn.Parameter(torch.stack(gub), requires_grad=False)
    dn.weight = nn.Parameter(torch.stack(dnb), requires_grad=False)
    shared, sgate = None, None
    if s.shared_expert_intermediate:
        Is = s.shared_expert_intermediate
        shared = SharedExpertMLP(lowbit_from_dense(interleave_glu_rows(rnd(Is, H), rnd(Is, H)), qtype, device),
                                 lowbit_from_dense(rnd(H, Is), qtype, device), s.act)
        sgate = rnd(1, H)
    renorm = s.norm_topk if s.model_type != "mixtral" else True
    return NativeMoE(rnd(E, H, scale=0.5), gu, dn, s.top_k, renorm, s.act, shared, sgate, expert_offset=e0,
                     num_experts=E, ep_group=ep_group)


def _module_weight(m: nn.Module):
    return m.weight if not isinstance(m, LowBitLinear) else None


def _moe_from_hf(spec: DecoderSpec, block) -> Optional[nn.Module]:
    from .moe import HFLowBitExperts, NativeMoE, SharedExpertMLP
    ex = block.experts
    if not isinstance(ex, HFLowBitExperts):
        return None
    shared, sgate = None, None
    se = getattr(block, "shared_expert", None)
    if se is not None:
        if not hasattr(se, "gate_up_proj"):
            return None
        shared = SharedExpertMLP(se.gate_up_proj, se.down_proj, spec.act)
        g = getattr(block, "shared_expert_gate", None)
        sgate = g.weight.data if g is not None else None
    ep = getattr(block, "_ep", None)
    return NativeMoE(block.gate.weight.data, ex.gate_up, ex.down, spec.top_k,
                     spec.norm_topk if spec.model_type != "mixtral" else True, spec.act, shared, sgate,
                     expert_offset=ep["e0"] if ep else 0, num_experts=spec.num_experts,
                     ep_group=ep["group"] if ep else None)


def native_from_hf(hf_model, dtype=None) -> Optional[NativeCausalLM]:
    """Wrap a converted HF CausalLM (qkv_proj / gate_up_proj merged by
    ``_optimize_pre``, linears already low-bit) into a NativeCausalLM that
    shares its parameters.  Returns None for unsupported layouts."""
    cfg = hf_model.config
    from .generic import GENERIC_ARCHS, generic_from_hf
    if getattr(cfg, "model_type", None) in GENERIC_ARCHS:
        return generic_from_hf(hf_model, dtype)
    from .mla import MLA_ARCHS, mla_from_hf
    if getattr(cfg, "model_type", None) in MLA_ARCHS:
        return mla_from_hf(hf_model, dtype)
    from .vl import VL_ARCHS, vl_native
    if getattr(cfg, "model_type", None) in VL_ARCHS:
        nm = vl_native(hf_model)
        if nm is not None:
            rp = getattr(cfg.text_config, "rope_parameters", None) or getattr(cfg.text_config, "rope_scaling", {})
            nm._mrope_section = list(rp.get("mrope_section", []))
        return nm
    spec = spec_from_config(cfg)
    tp = getattr(hf_model, "_tp", None)
    if tp is not None:                      # tensor-parallel shard: local heads
        spec.num_heads, spec.num_kv_heads = tp["num_heads"], tp["num_kv_heads"]
    base = getattr(hf_model, "model", None)
    if base is None or not hasattr(base, "layers"):
        return None
    pp = getattr(hf_model, "_pp", None)
    layers = []
    for i, L in enumerate(base.layers):
        if pp is not None and not (pp["start"] <= i < pp["end"]):
            continue                        # owned by another pipeline stage
        at = L.self_attn
        if spec.model_type == "yuan":
            from .yuan import yuan_lf_from_hf
            lf = yuan_lf_from_hf(at, spec.rms_eps, L.input_layernorm.weight.dtype, L.input_layernorm.weight.device)
            attn = NativeAttention(spec, None, at.o_proj)
            attn.lf = lf
            mlp = NativeMLP(spec, L.mlp.gate_up_proj, L.mlp.down_proj)
            layers.append(NativeLayer(spec, attn, mlp, L.input_layernorm.weight.data,
                                      L.post_attention_layernorm.weight.data))
            continue
        if not hasattr(at, "qkv_proj"):
            return None
        qn = getattr(at, "q_norm", None)
        kn = getattr(at, "k_norm", None)
        sw = spec.sliding_window
        if spec.sliding_window_layers is not None:
            sw = spec.sliding_window if spec.sliding_window_layers[i] else 0
        attn = NativeAttention(spec, at.qkv_proj, at.o_proj, qn.weight.data if qn is not None else None,
                               kn.weight.data if kn is not None else None, sw)
        if hasattr(L.mlp, "experts"):
            mlp = _moe_from_hf(spec, L.mlp)
            if mlp is None:
                return None
        elif hasattr(L.mlp, "gate_up_proj"):
            mlp = NativeMLP(spec, L.mlp.gate_up_proj, L.mlp.down_proj)
        else:
            return None
        pre_ff = getattr(L, "pre_feedforward_layernorm", None)
        post_ff = getattr(L, "post_feedforward_layernorm", None)
        ln2 = L.post_attention_layernorm
        if spec.model_type == "glm4":     # same sandwich as gemma2 under other names
            ln2, pre_ff, post_ff = L.post_self_attn_layernorm, L.post_attention_layernorm, L.post_mlp_layernorm
        layers.append(NativeLayer(spec, attn, mlp, L.input_layernorm.weight.data,
                                  ln2.weight.data,
                                  pre_ff.weight.data if pre_ff is not None else None,
                                  post_ff.weight.data if post_ff is not None else None))
    first = pp is None or pp["rank"] == 0
    last = pp is None or pp["rank"] == pp["stages"] - 1
    ln0 = layers[0].input_layernorm
    if not first:
        emb = ln0.data.new_empty(0)
    elif isinstance(base.embed_tokens, nn.Embedding):
        emb = base.embed_tokens.weight.data
    else:
        emb = base.embed_tokens          # CPU / disk / low-bit embedding module
    lm_head = hf_model.get_output_embeddings() if last else None
    norm = base.norm.weight.data if last else ln0.data
    inv_freq, att_scale = compute_inv_freq(cfg, spec.head_dim, spec.rot_dim or spec.head_dim)
    spec.rope_attention_scaling = att_scale
    model = NativeCausalLM(spec, emb, layers, norm, lm_head, inv_freq.to(ln0.device),
                           dtype or (emb.dtype if isinstance(emb, torch.Tensor) and first else ln0.dtype))
    model.first_stage, model.last_stage = first, last
    if pp is not None:
        model.layer_offset = pp["start"]
    return model.eval()


@torch.no_grad()
def dense_copy(model: NativeCausalLM) -> NativeCausalLM:
    """The same decoder with every low-bit linear replaced by a bf16
    DenseLinear holding its dequantized weight: a target model that agrees
    with its INT4 draft like a real checkpoint and its INT4 copy (self-
    speculative benchmarks / tests on random weights)."""
    def dense(m):
        d = DenseLinear(m.in_features, m.out_features, m.bias is not None, torch.bfloat16, "meta")
        d.weight = nn.Parameter(m.dequantize(torch.bfloat16).contiguous(), requires_grad=False)
        if m.bias is not None:
            d.bias = nn.Parameter(m.bias.detach().to(torch.bfloat16), requires_grad=False)
        return d

    s = model.spec
    layers = []
    for L in model.layers:
        a = L.self_attn
        attn = NativeAttention(s, dense(a.qkv_proj), dense(a.o_proj), a.q_norm, a.k_norm, a.sliding_window)
        mlp = NativeMLP(s, dense(L.mlp.gate_up_proj), dense(L.mlp.down_proj))
        layers.append(NativeLayer(s, attn, mlp, L.input_layernorm.data, L.post_attention_layernorm.data))
    return NativeCausalLM(s, model.embed_tokens.data, layers, model.norm.data, dense(model.lm_head),
                          model.inv_freq, torch.bfloat16).eval()
