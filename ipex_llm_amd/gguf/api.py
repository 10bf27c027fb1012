"""Build an HF model (+ tokenizer) from a GGUF file.

Reference: ``SRC/transformers/gguf/api.py:21-75`` (``load_gguf_model``
dispatching to per-family builders: llama, mistral, mixtral, baichuan,
bloom, falcon, mpt, yuan2 -- Yuan 2.0 builds models/yuan.py's in-library
LFA model) and ``gguf/models/llama.py:28-129`` (config from
the key/values, q/k row permutation undone, weights loaded tensor by
tensor).  Here one table-driven builder covers the llama-layout families
(llama / mistral / qwen2 / qwen3 and the MoE variants mixtral / qwen2moe /
qwen3moe); the tokenizer is rebuilt with transformers' GGUF converters.
Tensors are dequantized one at a time from the memory-mapped file and then
re-quantized by ``ggml_convert_low_bit`` into the MI355X formats -- except
the k-quant projections (Q2_K / Q4_K / Q5_K / Q6_K): with ``keep_kquant``
their super-block bytes become :class:`KQuantLinear` weights as they are
(the device layout IS the GGUF layout), no dequantize / re-quantize round
trip, bits per weight and numerics exactly those of the file.  llama.cpp's
q/k row permutation is undone on whole block rows.
"""
from __future__ import annotations

import re
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from .reader import GGUFReader

ARCH_TO_HF = {"llama": "llama", "mistral": "mistral", "qwen2": "qwen2", "qwen3": "qwen3",
              "qwen2moe": "qwen2_moe", "qwen3moe": "qwen3_moe"}
# bloom / falcon / mpt / baichuan: gguf/families.py

_LAYER = {
    "attn_norm": "input_layernorm.weight",
    "ffn_norm": "post_attention_layernorm.weight",
    "attn_q": "self_attn.q_proj",
    "attn_k": "self_attn.k_proj",
    "attn_v": "self_attn.v_proj",
    "attn_output": "self_attn.o_proj",
    "attn_q_norm": "self_attn.q_norm.weight",
    "attn_k_norm": "self_attn.k_norm.weight",
    "ffn_gate": "mlp.gate_proj",
    "ffn_up": "mlp.up_proj",
    "ffn_down": "mlp.down_proj",
    "ffn_gate_inp": "mlp.gate.weight",
    "ffn_gate_shexp": "mlp.shared_expert.gate_proj",
    "ffn_up_shexp": "mlp.shared_expert.up_proj",
    "ffn_down_shexp": "mlp.shared_expert.down_proj",
    "ffn_gate_inp_shexp": "mlp.shared_expert_gate.weight",
    # Yuan 2.0 localized filtering (reference gguf/models/yuan2.py:88-97)
    "lf_output_norm": "self_attn.lf_gate.output_layernorm.weight",
    "conv1": "self_attn.lf_gate.conv1",
    "conv2": "self_attn.lf_gate.conv2",
}


def is_yuan(r: GGUFReader) -> bool:
    """Yuan 2.0 GGUF: architecture "llama" + "yuan" in general.name (the
    reference's dispatch, gguf/api.py:45-56)"""
    return r.architecture == "llama" and "yuan" in str(r.kv.get("general.name", "")).lower()


def _yuan_config(r: GGUFReader):
    """reference gguf/models/yuan2.py:31-59 (llama.* keys)"""
    from ..models.yuan import YuanConfig, register
    register()
    g = lambda k, d=None: r.kv.get(f"llama.{k}", d)           # noqa: E731
    toks = r.kv.get("tokenizer.ggml.tokens")
    return YuanConfig(vocab_size=len(toks) if toks is not None else r.tensors["token_embd.weight"].shape[1],
                      hidden_size=g("embedding_length"), intermediate_size=g("feed_forward_length"),
                      num_hidden_layers=g("block_count"), num_attention_heads=g("attention.head_count"),
                      max_position_embeddings=g("context_length", 4096),
                      rms_norm_eps=g("attention.layer_norm_rms_epsilon", 1e-6),
                      tie_word_embeddings="output.weight" not in r.tensors,
                      pad_token_id=r.kv.get("tokenizer.ggml.padding_token_id"),
                      bos_token_id=r.kv.get("tokenizer.ggml.bos_token_id"),
                      eos_token_id=r.kv.get("tokenizer.ggml.eos_token_id"))


def _unpermute(w: np.ndarray, n_head: int) -> np.ndarray:
    """undo llama.cpp's q/k row permutation (HF rotate_half -> GGUF interleaved)"""
    out = w.shape[0]
    return w.reshape(n_head, 2, out // n_head // 2, *w.shape[1:]).swapaxes(1, 2).reshape(w.shape)


def _config(r: GGUFReader):
    from transformers import AutoConfig
    from transformers.integrations.ggml import GGUF_CONFIG_MAPPING
    arch = r.architecture
    mt = ARCH_TO_HF.get(arch)
    if mt is None:
        raise NotImplementedError(f"GGUF architecture '{arch}' is not supported")
    kw = {}
    mapping = GGUF_CONFIG_MAPPING.get(arch, GGUF_CONFIG_MAPPING["llama"])
    for key, hf in mapping.items():
        v = r.kv.get(f"{arch}.{key}")
        if hf is not None and v is not None:
            kw[hf] = v
    if "vocab_size" not in kw:
        toks = r.kv.get("tokenizer.ggml.tokens")
        if toks is not None:
            kw["vocab_size"] = len(toks)
        else:
            kw["vocab_size"] = r.tensors["token_embd.weight"].shape[1]
    n_exp = r.kv.get(f"{arch}.expert_count")
    if n_exp:
        kw["num_local_experts" if mt == "mixtral" else "num_experts"] = n_exp
        kw["num_experts_per_tok"] = r.kv.get(f"{arch}.expert_used_count", 2)
        if mt != "mixtral":
            ff = r.kv.get(f"{arch}.expert_feed_forward_length")
            if ff:
                kw["moe_intermediate_size"] = ff
    if arch == "llama" and n_exp:
        mt = "mixtral"
        kw["num_local_experts"] = kw.pop("num_experts", n_exp)
    kw.pop("head_dim", None) if mt in ("llama", "mistral", "mixtral") else None
    kw["tie_word_embeddings"] = "output.weight" not in r.tensors
    for t in ("bos", "eos", "padding"):
        v = r.kv.get(f"tokenizer.ggml.{t}_token_id")
        if v is not None:
            kw[{"padding": "pad"}.get(t, t) + "_token_id"] = v
    return AutoConfig.for_model(mt, **kw), mt


def _tokenizer(r: GGUFReader):
    try:
        from transformers import PreTrainedTokenizerFast
        from transformers.integrations.ggml import convert_gguf_tokenizer
    except ImportError:  # pragma: no cover
        return None
    tok = {k[len("tokenizer.ggml."):]: v for k, v in r.kv.items() if k.startswith("tokenizer.ggml.")}
    if "tokens" not in tok:
        return None
    arch = r.architecture if r.architecture in ("llama", "qwen2", "qwen2moe", "qwen3", "qwen3moe") else "llama"
    try:
        fast, extra = convert_gguf_tokenizer(arch, tok)
    except Exception:       # unknown tokenizer model: leave to the caller
        return None
    return PreTrainedTokenizerFast(tokenizer_object=fast, **extra)


def _kquant_linear_targets(r: GGUFReader, arch: str = "llama", cfg=None):
    """GGUF linear tensors stored as k-quants -> (HF module path, qtype)"""
    from .families import TABLES, hf_name
    from .reader import KQUANT_QTYPE
    out = {}
    for name, ti in r.tensors.items():
        if ti.ggml_type not in KQUANT_QTYPE or len(ti.shape) != 2:
            continue
        if arch in TABLES:
            if name == "token_embd.weight":
                continue
            key = hf_name(arch, name, cfg)
            if key is not None and key.endswith(".weight"):
                out[name] = (key[:-len(".weight")], KQUANT_QTYPE[ti.ggml_type])
            continue
        if name == "output.weight":
            out[name] = ("lm_head", KQUANT_QTYPE[ti.ggml_type])
            continue
        m = re.match(r"blk\.(\d+)\.(\w+?)\.weight$", name)
        if m and m.group(2) in _LAYER and not _LAYER[m.group(2)].endswith(".weight"):
            out[name] = (f"model.layers.{m.group(1)}.{_LAYER[m.group(2)]}", KQUANT_QTYPE[ti.ggml_type])
    return out


def _unpermute_rows(raw: np.ndarray, n_rows: int, n_head: int) -> np.ndarray:
    """llama.cpp q/k permutation undone on whole (block-encoded) rows"""
    rows = raw.reshape(n_rows, -1)
    idx = _unpermute(np.arange(n_rows), n_head)
    return np.ascontiguousarray(rows[idx]).reshape(-1)


def load_gguf_model(fpath: str, dtype=torch.float16, low_bit: Optional[str] = None,
                    keep_kquant: bool = False) -> Tuple[torch.nn.Module, object]:
    """GGUF file -> (HF CausalLM with dense ``dtype`` weights, tokenizer).
    ``keep_kquant``: k-quant projections become KQuantLinear modules over the
    file's blocks (everything else stays dense for ``ggml_convert_low_bit``)."""
    from accelerate import init_empty_weights
    from transformers import AutoModelForCausalLM
    from .families import TABLES, family_config, hf_name, qkv_gguf_to_hf
    r = GGUFReader(fpath)
    arch = r.architecture
    fam = family_config(r) if arch in ("bloom", "falcon", "mpt", "baichuan") else None
    yuan = is_yuan(r)
    if yuan:
        cfg, mt = _yuan_config(r), "yuan"
    else:
        cfg, mt = (fam, fam.model_type) if fam is not None else _config(r)
    # llama.cpp's q/k row permutation (Yuan files keep the HF order: the
    # reference's yuan2 loader maps attn_q / attn_k as they are)
    permuted = arch in ("llama", "baichuan") and not yuan
    with init_empty_weights():
        model = AutoModelForCausalLM.from_config(cfg, torch_dtype=dtype)
    n_head, n_kv = cfg.num_attention_heads, getattr(cfg, "num_key_value_heads", cfg.num_attention_heads)
    sd: Dict[str, torch.Tensor] = {}
    experts: Dict[int, Dict[str, np.ndarray]] = {}
    kq_targets = _kquant_linear_targets(r, arch, cfg) if keep_kquant else {}
    kq_blocks = {}
    for name in r.tensors:
        if arch in TABLES and name not in kq_targets:
            key = hf_name(arch, name, cfg)
            if key is None:
                continue
            w = r.tensor(name)
            if ".attn_qkv." in name:
                w = qkv_gguf_to_hf(arch, w, cfg)
            sd[key] = torch.from_numpy(np.ascontiguousarray(w))
            continue
        if name in kq_targets:
            path, qt = kq_targets[name]
            ti = r.tensors[name]
            k, n = ti.shape                                  # GGUF order: ne0 = in_features
            raw = np.asarray(r.raw(name))
            kind = name.split(".")[2] if name.startswith("blk.") else ""
            if kind in ("attn_q", "attn_k") and permuted:
                raw = _unpermute_rows(raw, n, n_head if kind == "attn_q" else n_kv)
            if kind == "attn_qkv":                       # fused families: HF row order, whole block rows
                rows = qkv_gguf_to_hf(arch, np.arange(n), cfg)
                raw = np.ascontiguousarray(raw.reshape(n, -1)[rows]).reshape(-1)
            kq_blocks[path] = (torch.from_numpy(np.array(raw, dtype=np.uint8)), qt, n, k)
            continue
        w = r.tensor(name)
        if name == "token_embd.weight":
            sd["model.embed_tokens.weight"] = torch.from_numpy(w)
            continue
        if name == "output_norm.weight":
            sd["model.norm.weight"] = torch.from_numpy(w)
            continue
        if name == "output.weight":
            sd["lm_head.weight"] = torch.from_numpy(w)
            continue
        m = re.match(r"blk\.(\d+)\.(\w+?)\.(weight|bias)$", name)
        if not m:
            continue
        i, kind, wb = int(m.group(1)), m.group(2), m.group(3)
        if kind in ("ffn_gate_exps", "ffn_up_exps", "ffn_down_exps"):
            experts.setdefault(i, {})[kind] = w
            continue
        target = _LAYER.get(kind)
        if target is None:
            continue
        if kind in ("attn_q", "attn_k") and permuted and wb == "weight":
            w = _unpermute(w, n_head if kind == "attn_q" else n_kv)
        elif kind in ("attn_q", "attn_k") and permuted and wb == "bias":
            w = _unpermute(w[:, None], n_head if kind == "attn_q" else n_kv)[:, 0]
        key = f"model.layers.{i}.{target}"
        if not key.endswith((".weight", ".bias")):
            key += "." + wb
        if kind == "ffn_gate_inp_shexp" and w.ndim == 1:
            w = w[None, :]
        sd[key] = torch.from_numpy(np.ascontiguousarray(w))
    for i, ex in experts.items():
        g, u, d = ex["ffn_gate_exps"], ex["ffn_up_exps"], ex["ffn_down_exps"]    # [E, I, H], [E, I, H], [E, H, I]
        sd[f"model.layers.{i}.mlp.experts.gate_up_proj"] = torch.from_numpy(np.concatenate([g, u], 1))
        sd[f"model.layers.{i}.mlp.experts.down_proj"] = torch.from_numpy(np.ascontiguousarray(d))
    sd = {k: v.to(dtype) for k, v in sd.items()}
    model.load_state_dict(sd, strict=False, assign=True)
    if cfg.tie_word_embeddings:
        model.tie_weights()
    if kq_blocks:
        from ..transformers.low_bit_linear import KQuantLinear
        for path, (blob, qt, n, k) in kq_blocks.items():
            parent_path, leaf = path.rsplit(".", 1) if "." in path else ("", path)
            parent = model.get_submodule(parent_path) if parent_path else model
            old = getattr(parent, leaf)
            bias = old.bias if getattr(old, "bias", None) is not None and old.bias.device.type != "meta" else None
            setattr(parent, leaf, KQuantLinear.from_blocks(blob, qt, n, k, device="cpu", bias=bias))
    from ..transformers.model import _reinit_meta_buffers
    _reinit_meta_buffers(model, cfg)
    missing = [n for n, p in model.named_parameters() if p.device.type == "meta"]
    if missing:
        raise RuntimeError(f"GGUF file lacks tensors for: {missing[:6]}")
    return model.eval(), _tokenizer(r)
