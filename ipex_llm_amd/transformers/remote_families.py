"""Remote-code model families loaded without their remote code.

ChatGLM2 / ChatGLM3 / GLM-4 checkpoints (``model_type: chatglm``, THUDM remote
code) and Qwen v1 (``model_type: qwen``) are not part of ``transformers``;
the reference runs their remote code and patches it per family
(``SRC/transformers/models/chatglm2.py``, ``chatglm4.py:163-205``
(rotary_two / multi-query attention), ``qwen.py``; conversion table
``SRC/transformers/convert.py:1275-2139``).

Both are architectures ``transformers`` ships under another name, so here the
checkpoint is re-expressed, tensor by tensor, as that model and then takes the
normal path (low-bit conversion + the native decoder):

* chatglm -> ``GlmForCausalLM``: fused ``query_key_value`` (MQA: q heads then
  ``multi_query_group_num`` k / v heads) split into q / k / v projections,
  ``dense_h_to_4h`` = [gate; up] = Glm's ``gate_up_proj``, rotary on the first
  half of each head in interleaved pairs (``partial_rotary_factor`` 0.5,
  base 10000 * ``rope_ratio``), RMSNorm, untied ``output_layer``.
* internlm (v1) -> ``LlamaForCausalLM`` with ``attention_bias`` (q/k/v/o
  biases, llama tensor names; reference ``SRC/transformers/models/internlm.py``).
* qwen -> ``Qwen2ForCausalLM``: ``c_attn`` (q|k|v with bias) split, ``c_proj``
  -> o_proj, MLP ``c_proj(w1(x) * silu(w2(x)))`` -> gate = w2, up = w1,
  down = c_proj, full-width NeoX rotary (``rotary_emb_base``).  Qwen v1's
  dynamic-NTK / logn attention scaling only act beyond ``seq_length`` and are
  not reproduced (reference qwen.py applies them on that long-context branch).

Parity of the layouts is pinned against the in-library models (tests build
the chatglm / qwen tensor names from a random Glm / Qwen2 model and compare
logits); against the remote code itself it is unpinned (not importable here).
"""
from __future__ import annotations

import glob
import json
import os
from typing import Dict, Optional

import torch

FAMILIES = ("chatglm", "qwen", "internlm", "yuan")


def family_of(path) -> Optional[str]:
    if not isinstance(path, (str, os.PathLike)) or not os.path.isdir(path):
        return None
    f = os.path.join(path, "config.json")
    if not os.path.exists(f):
        return None
    with open(f) as fh:
        mt = json.load(fh).get("model_type")
    return mt if mt in FAMILIES else None


def _load_state_dict(path) -> Dict[str, torch.Tensor]:
    sd: Dict[str, torch.Tensor] = {}
    st = sorted(glob.glob(os.path.join(path, "*.safetensors")))
    if st:
        from safetensors.torch import load_file
        for f in st:
            sd.update(load_file(f))
        return sd
    for f in sorted(glob.glob(os.path.join(path, "pytorch_model*.bin"))):
        sd.update(torch.load(f, map_location="cpu", weights_only=True))
    if not sd:
        raise FileNotFoundError(f"no safetensors / pytorch_model*.bin weights under {path}")
    return sd


# ---------------------------------------------------------------- chatglm
def chatglm_to_glm_config(c: dict):
    from transformers import GlmConfig
    nh = c["num_attention_heads"]
    nkv = c.get("multi_query_group_num", nh) if c.get("multi_query_attention", False) else nh
    D = c.get("kv_channels", c["hidden_size"] // nh)
    return GlmConfig(
        vocab_size=c.get("padded_vocab_size", c.get("vocab_size")), hidden_size=c["hidden_size"],
        intermediate_size=c["ffn_hidden_size"], num_hidden_layers=c["num_layers"], num_attention_heads=nh,
        num_key_value_heads=nkv, head_dim=D, max_position_embeddings=c.get("seq_length", 8192),
        rms_norm_eps=c.get("layernorm_epsilon", 1e-5), attention_bias=bool(c.get("add_qkv_bias", True)),
        tie_word_embeddings=False, pad_token_id=None, eos_token_id=c.get("eos_token_id"),
        rope_parameters={"rope_type": "default", "rope_theta": 10000.0 * float(c.get("rope_ratio", 1.0)),
                         "partial_rotary_factor": 0.5})


def chatglm_to_glm_weights(sd: Dict[str, torch.Tensor], c: dict) -> Dict[str, torch.Tensor]:
    nh = c["num_attention_heads"]
    nkv = c.get("multi_query_group_num", nh) if c.get("multi_query_attention", False) else nh
    D = c.get("kv_channels", c["hidden_size"] // nh)
    out = {}
    pre = "transformer.encoder.layers."
    for k, v in sd.items():
        if k == "transformer.embedding.word_embeddings.weight":
            out["model.embed_tokens.weight"] = v
        elif k == "transformer.encoder.final_layernorm.weight":
            out["model.norm.weight"] = v
        elif k == "transformer.output_layer.weight":
            out["lm_head.weight"] = v
        elif k.startswith(pre):
            i, rest = k[len(pre):].split(".", 1)
            L = f"model.layers.{i}."
            if rest.startswith("self_attention.query_key_value."):
                kind = rest.rsplit(".", 1)[1]
                q, kk, vv = torch.split(v, [nh * D, nkv * D, nkv * D], 0)
                out[L + f"self_attn.q_proj.{kind}"] = q
                out[L + f"self_attn.k_proj.{kind}"] = kk
                out[L + f"self_attn.v_proj.{kind}"] = vv
            elif rest == "self_attention.dense.weight":
                out[L + "self_attn.o_proj.weight"] = v
            elif rest == "mlp.dense_h_to_4h.weight":
                out[L + "mlp.gate_up_proj.weight"] = v
            elif rest == "mlp.dense_4h_to_h.weight":
                out[L + "mlp.down_proj.weight"] = v
            elif rest in ("input_layernorm.weight", "post_attention_layernorm.weight"):
                out[L + rest] = v
        # rotary_pos_emb.inv_freq and other buffers are recomputed
    return out


# ---------------------------------------------------------------- qwen v1
def qwen_to_qwen2_config(c: dict):
    from transformers import Qwen2Config
    nh = c["num_attention_heads"]
    return Qwen2Config(
        vocab_size=c["vocab_size"], hidden_size=c["hidden_size"], intermediate_size=c["intermediate_size"] // 2,
        num_hidden_layers=c["num_hidden_layers"], num_attention_heads=nh, num_key_value_heads=nh,
        max_position_embeddings=c.get("max_position_embeddings", c.get("seq_length", 8192)),
        rms_norm_eps=c.get("layer_norm_epsilon", 1e-6), tie_word_embeddings=bool(c.get("tie_word_embeddings", False)),
        rope_parameters={"rope_type": "default", "rope_theta": float(c.get("rotary_emb_base", 10000.0))})


def qwen_to_qwen2_weights(sd: Dict[str, torch.Tensor], c: dict) -> Dict[str, torch.Tensor]:
    H = c["hidden_size"]
    out = {}
    for k, v in sd.items():
        if k == "transformer.wte.weight":
            out["model.embed_tokens.weight"] = v
        elif k == "transformer.ln_f.weight":
            out["model.norm.weight"] = v
        elif k == "lm_head.weight":
            out["lm_head.weight"] = v
        elif k.startswith("transformer.h."):
            i, rest = k[len("transformer.h."):].split(".", 1)
            L = f"model.layers.{i}."
            if rest.startswith("attn.c_attn."):
                kind = rest.rsplit(".", 1)[1]
                q, kk, vv = torch.split(v, [H, H, H], 0)
                out[L + f"self_attn.q_proj.{kind}"] = q
                out[L + f"self_attn.k_proj.{kind}"] = kk
                out[L + f"self_attn.v_proj.{kind}"] = vv
            elif rest == "attn.c_proj.weight":
                out[L + "self_attn.o_proj.weight"] = v
            elif rest == "mlp.w1.weight":
                out[L + "mlp.up_proj.weight"] = v
            elif rest == "mlp.w2.weight":
                out[L + "mlp.gate_proj.weight"] = v
            elif rest == "mlp.c_proj.weight":
                out[L + "mlp.down_proj.weight"] = v
            elif rest == "ln_1.weight":
                out[L + "input_layernorm.weight"] = v
            elif rest == "ln_2.weight":
                out[L + "post_attention_layernorm.weight"] = v
    return out


# ---------------------------------------------------------------- internlm v1
def internlm_to_llama_config(c: dict):
    from transformers import LlamaConfig
    rot = c.get("rotary") or {}
    return LlamaConfig(
        vocab_size=c["vocab_size"], hidden_size=c["hidden_size"], intermediate_size=c["intermediate_size"],
        num_hidden_layers=c["num_hidden_layers"], num_attention_heads=c["num_attention_heads"],
        num_key_value_heads=c.get("num_key_value_heads", c["num_attention_heads"]),
        max_position_embeddings=c.get("max_position_embeddings", 2048), rms_norm_eps=c.get("rms_norm_eps", 1e-6),
        attention_bias=bool(c.get("bias", True)), tie_word_embeddings=bool(c.get("tie_word_embeddings", False)),
        rope_parameters={"rope_type": "default", "rope_theta": float(rot.get("base", c.get("rope_theta", 10000.0)))})


def load_remote_family(path, torch_dtype="auto"):
    """HF model of the in-library architecture equivalent to a chatglm / qwen
    checkpoint, with the checkpoint's tensors mapped in (CPU)."""
    fam = family_of(path)
    if fam is None:
        raise ValueError(f"{path}: not a chatglm / qwen checkpoint")
    with open(os.path.join(path, "config.json")) as fh:
        c = json.load(fh)
    sd = _load_state_dict(path)
    if fam == "chatglm":
        from transformers import GlmForCausalLM
        cfg, mapped, cls = chatglm_to_glm_config(c), chatglm_to_glm_weights(sd, c), GlmForCausalLM
    elif fam == "internlm":
        from transformers import LlamaForCausalLM
        cfg, mapped, cls = internlm_to_llama_config(c), dict(sd), LlamaForCausalLM
    elif fam == "yuan":
        # Yuan 2.0 (remote code): the in-library LFA model, same tensor names
        from ..models.yuan import YuanForCausalLM, yuan_config_from_remote
        cfg, cls = yuan_config_from_remote(c), YuanForCausalLM
        mapped = {k: v for k, v in sd.items() if not k.endswith("rotary_emb.inv_freq")}
    else:
        from transformers import Qwen2ForCausalLM
        cfg, mapped, cls = qwen_to_qwen2_config(c), qwen_to_qwen2_weights(sd, c), Qwen2ForCausalLM
    if torch_dtype in (None, "auto"):
        torch_dtype = next(iter(mapped.values())).dtype
    with torch.device("meta"):
        model = cls(cfg)
    missing, unexpected = model.load_state_dict(mapped, strict=False, assign=True)
    missing = [m for m in missing if not m.endswith("rotary_emb.inv_freq")]
    if cfg.tie_word_embeddings and "lm_head.weight" in missing:
        missing.remove("lm_head.weight")
        model.tie_weights()
    if missing or unexpected:
        raise ValueError(f"{fam} checkpoint mapping: missing {missing[:5]}, unexpected {unexpected[:5]}")
    # buffers built on meta (rotary inv_freq) are recomputed on the CPU
    if hasattr(model.model, "rotary_emb"):
        model.model.rotary_emb = type(model.model.rotary_emb)(model.config)
    model = model.to(torch_dtype)
    model.config.illm_source_model_type = fam
    return model.eval()
