"""GGUF <-> HF layouts of the non-llama families.

Reference: ``SRC/transformers/gguf/models/{bloom,falcon,mpt,baichuan}.py``
(per-family loaders building the HF model from llama.cpp tensors) behind
``gguf/api.py:21-75``.  One table per family maps llama.cpp tensor names to
HF parameter names; the fused QKV weights llama.cpp stores as
``[q; k; v]`` (``convert_hf_to_gguf``'s bloom / falcon re-ordering) are put
back into the HF row order so the regular conversion path (and the native
generic decoder, models/generic.py) takes over.  baichuan-7B is a llama
layout (llama.cpp splits ``W_pack`` and permutes q/k like llama); the ALiBi
baichuan-13B is refused, as in the reference, whose GGUF baichuan loader
builds the RoPE model (``gguf/models/model_implement/baichuan/
modeling_baichuan.py:95,184``).
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

# llama.cpp tensor base name -> HF parameter path ({i} = layer)
_BLOOM = {
    "token_embd": "transformer.word_embeddings", "token_embd_norm": "transformer.word_embeddings_layernorm",
    "output_norm": "transformer.ln_f", "output": "lm_head",
    "attn_norm": "transformer.h.{i}.input_layernorm", "attn_qkv": "transformer.h.{i}.self_attention.query_key_value",
    "attn_output": "transformer.h.{i}.self_attention.dense", "ffn_norm": "transformer.h.{i}.post_attention_layernorm",
    "ffn_up": "transformer.h.{i}.mlp.dense_h_to_4h", "ffn_down": "transformer.h.{i}.mlp.dense_4h_to_h",
}
_FALCON = {
    "token_embd": "transformer.word_embeddings", "output_norm": "transformer.ln_f", "output": "lm_head",
    "attn_norm": "transformer.h.{i}.input_layernorm", "attn_norm_2": "transformer.h.{i}.ln_mlp",
    "attn_qkv": "transformer.h.{i}.self_attention.query_key_value",
    "attn_output": "transformer.h.{i}.self_attention.dense",
    "ffn_up": "transformer.h.{i}.mlp.dense_h_to_4h", "ffn_down": "transformer.h.{i}.mlp.dense_4h_to_h",
}
_MPT = {
    "token_embd": "transformer.wte", "output_norm": "transformer.norm_f", "output": "lm_head",
    "attn_norm": "transformer.blocks.{i}.norm_1", "attn_qkv": "transformer.blocks.{i}.attn.Wqkv",
    "attn_output": "transformer.blocks.{i}.attn.out_proj", "ffn_norm": "transformer.blocks.{i}.norm_2",
    "ffn_up": "transformer.blocks.{i}.ffn.up_proj", "ffn_down": "transformer.blocks.{i}.ffn.down_proj",
}
TABLES = {"bloom": _BLOOM, "falcon": _FALCON, "mpt": _MPT}


def _kv(r, arch, key, default=None):
    v = r.kv.get(f"{arch}.{key}")
    return default if v is None else v


def family_config(r):
    """GGUF metadata -> HF config of bloom / falcon / mpt / baichuan (None: other arch)"""
    from transformers import AutoConfig
    arch = r.architecture
    toks = r.kv.get("tokenizer.ggml.tokens")
    vocab = len(toks) if toks is not None else r.tensors["token_embd.weight"].shape[1]
    H = _kv(r, arch, "embedding_length")
    L = _kv(r, arch, "block_count")
    nh = _kv(r, arch, "attention.head_count")
    tie = "output.weight" not in r.tensors
    if arch == "bloom":
        return AutoConfig.for_model("bloom", vocab_size=vocab, hidden_size=H, n_layer=L, n_head=nh,
                                    layer_norm_epsilon=_kv(r, arch, "attention.layer_norm_epsilon", 1e-5),
                                    tie_word_embeddings=tie)
    if arch == "falcon":
        nkv = _kv(r, arch, "attention.head_count_kv", 1)
        new = "blk.0.attn_norm_2.weight" in r.tensors
        return AutoConfig.for_model("falcon", vocab_size=vocab, hidden_size=H, num_hidden_layers=L,
                                    num_attention_heads=nh, num_kv_heads=nkv, new_decoder_architecture=new,
                                    multi_query=(nkv == 1) and not new, parallel_attn=True, bias=False,
                                    layer_norm_epsilon=_kv(r, arch, "attention.layer_norm_epsilon", 1e-5),
                                    max_position_embeddings=_kv(r, arch, "context_length", 2048),
                                    tie_word_embeddings=tie)
    if arch == "mpt":
        ff = _kv(r, arch, "feed_forward_length", 4 * H)
        abm = float(_kv(r, arch, "attention.max_alibi_bias", 8.0))
        ac = {"alibi": True, "alibi_bias_max": int(abm) if abm.is_integer() else abm}
        clip = _kv(r, arch, "attention.clamp_kqv")
        if clip:
            ac["clip_qkv"] = clip
        return AutoConfig.for_model("mpt", vocab_size=vocab, d_model=H, n_layers=L, n_heads=nh,
                                    expansion_ratio=ff // H if ff % H == 0 else ff / H, max_seq_len=_kv(r, arch, "context_length", 2048),
                                    attn_config=ac, no_bias=True,
                                    layer_norm_epsilon=_kv(r, arch, "attention.layer_norm_epsilon", 1e-5),
                                    tie_word_embeddings=tie)
    if arch == "baichuan":
        if "blk.0.attn_q.weight" not in r.tensors or L == 40:
            raise NotImplementedError("GGUF baichuan-13B (ALiBi) needs the remote-code model; 7B loads as llama")
        return AutoConfig.for_model("llama", vocab_size=vocab, hidden_size=H, num_hidden_layers=L,
                                    num_attention_heads=nh,
                                    num_key_value_heads=_kv(r, arch, "attention.head_count_kv", nh),
                                    intermediate_size=_kv(r, arch, "feed_forward_length"),
                                    rms_norm_eps=_kv(r, arch, "attention.layer_norm_rms_epsilon", 1e-6),
                                    rope_theta=_kv(r, arch, "rope.freq_base", 10000.0),
                                    max_position_embeddings=_kv(r, arch, "context_length", 4096),
                                    tie_word_embeddings=tie)
    return None


def qkv_gguf_to_hf(arch: str, w: np.ndarray, cfg) -> np.ndarray:
    """[q; k; v] rows (llama.cpp) -> the HF fused-QKV row order"""
    if arch == "bloom":
        nh = cfg.n_head
        D = cfg.hidden_size // nh
        q, k, v = np.split(w, 3, axis=0)
        t = np.stack([x.reshape(nh, D, *w.shape[1:]) for x in (q, k, v)], 1)
        return t.reshape(w.shape)
    if arch == "falcon":
        nh, nkv = cfg.num_attention_heads, cfg.num_kv_heads if cfg.new_decoder_architecture else 1
        D = cfg.hidden_size // nh
        g = nh // nkv
        q = w[:nh * D].reshape(nkv, g, D, *w.shape[1:])
        k = w[nh * D:(nh + nkv) * D].reshape(nkv, 1, D, *w.shape[1:])
        v = w[(nh + nkv) * D:].reshape(nkv, 1, D, *w.shape[1:])
        return np.concatenate([q, k, v], 1).reshape(w.shape)
    return w                                             # mpt: already [q; k; v]


def qkv_hf_to_gguf(arch: str, w: np.ndarray, cfg) -> np.ndarray:
    """inverse of :func:`qkv_gguf_to_hf` (GGUF export)"""
    if arch == "bloom":
        nh = cfg.n_head
        D = cfg.hidden_size // nh
        t = w.reshape(nh, 3, D, *w.shape[1:])
        return np.concatenate([t[:, 0], t[:, 1], t[:, 2]], 0).reshape(w.shape)
    if arch == "falcon":
        nh, nkv = cfg.num_attention_heads, cfg.num_kv_heads if cfg.new_decoder_architecture else 1
        D = cfg.hidden_size // nh
        g = nh // nkv
        t = w.reshape(nkv, g + 2, D, *w.shape[1:])
        return np.concatenate([t[:, :g].reshape(nh * D, *w.shape[1:]), t[:, g].reshape(nkv * D, *w.shape[1:]),
                               t[:, g + 1].reshape(nkv * D, *w.shape[1:])], 0)
    return w


def hf_name(arch: str, gguf_name: str, cfg) -> Optional[str]:
    """llama.cpp tensor name -> HF parameter name (None: not used)"""
    table = TABLES[arch]
    parts = gguf_name.split(".")
    if parts[0] == "blk":
        i, base, wb = parts[1], ".".join(parts[2:-1]), parts[-1]
        if arch == "falcon" and base == "attn_norm" and cfg.new_decoder_architecture:
            return f"transformer.h.{i}.ln_attn.{wb}"
        t = table.get(base)
        return None if t is None else t.format(i=i) + "." + wb
    base, wb = ".".join(parts[:-1]), parts[-1]
    t = table.get(base)
    return None if t is None else t + "." + wb


def gguf_names(arch: str, cfg) -> Dict[str, str]:
    """HF parameter name -> llama.cpp tensor name (GGUF export)"""
    out = {}
    table = TABLES[arch]
    for base, path in table.items():
        if "{i}" in path:
            for i in range(cfg.num_hidden_layers):
                for wb in ("weight", "bias"):
                    p = path.format(i=i) + "." + wb
                    if arch == "falcon" and base == "attn_norm" and cfg.new_decoder_architecture:
                        p = f"transformer.h.{i}.ln_attn.{wb}"
                    out[p] = f"blk.{i}.{base}.{wb}"
        else:
            for wb in ("weight", "bias"):
                out[path + "." + wb] = f"{base}.{wb}"
    return out


def export_family_gguf(model, outfile: str, tq: int, mat_type) -> str:
    """write a bloom / falcon / mpt HF model as llama.cpp GGUF"""
    from .reader import F32, GGUFWriter
    cfg = model.config
    arch = cfg.model_type
    w = GGUFWriter(outfile, arch)
    H = cfg.hidden_size
    nh = cfg.num_attention_heads
    w.add(f"{arch}.embedding_length", int(H))
    w.add(f"{arch}.block_count", int(cfg.num_hidden_layers))
    w.add(f"{arch}.attention.head_count", int(nh))
    w.add(f"{arch}.attention.layer_norm_epsilon", float(getattr(cfg, "layer_norm_epsilon", 1e-5)))
    w.add(f"{arch}.vocab_size", int(cfg.vocab_size))
    if arch == "falcon":
        w.add(f"{arch}.attention.head_count_kv", int(cfg.num_kv_heads if cfg.new_decoder_architecture else 1))
        w.add(f"{arch}.context_length", int(cfg.max_position_embeddings))
    if arch == "mpt":
        w.add(f"{arch}.feed_forward_length", int(cfg.expansion_ratio * H))
        w.add(f"{arch}.context_length", int(cfg.max_seq_len))
        ac = cfg.attn_config if isinstance(cfg.attn_config, dict) else cfg.attn_config.to_dict()
        w.add(f"{arch}.attention.max_alibi_bias", float(ac.get("alibi_bias_max", 8)))
    names = gguf_names(arch, cfg)
    tied = getattr(cfg, "tie_word_embeddings", False)
    for k, v in model.state_dict().items():
        g = names.get(k)
        if g is None or (g == "output.weight" and tied):
            continue
        a = v.detach().float().cpu().numpy()
        if g.startswith("blk.") and ".attn_qkv." in g:
            a = qkv_hf_to_gguf(arch, a, cfg)
        is_mat = a.ndim == 2 and "norm" not in g and a.shape[1] % 32 == 0
        w.add_tensor(g, a, (mat_type(k, a) if g != "token_embd.weight" else tq) if is_mat else F32)
    w.write()
    return outfile
