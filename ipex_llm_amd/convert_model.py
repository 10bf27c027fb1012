"""``llm_convert``: convert an HF checkpoint to a deployable low-bit artifact.

Reference: ``SRC/convert_model.py:31-144`` / ``ggml/convert_model.py`` (HF
or pth -> ggml f16 -> quantized ``.bin`` through the native ``quantize-*``
binaries; ``llm-convert`` CLI).  MI355X version, no external binaries:
  * ``outtype`` = any low-bit qtype name (``"int4"`` = sym_int4, ``"nf4"``,
    ``"fp8"`` ...) -> a ``save_low_bit`` directory (safetensors, portable
    canonical layout) loadable with ``AutoModelForCausalLM.load_low_bit``;
  * ``outtype`` = ``"gguf_f16" | "gguf_q8_0" | "gguf_q4_0" | "gguf_f32"`` or
    the k-quants ``"gguf_q4_k" | "gguf_q5_k" | "gguf_q6_k" | "gguf_q2_k" |
    "gguf_q4_k_m" | "gguf_q4_k_s"`` -> a GGUF file readable by ``from_gguf``
    and llama.cpp, for the llama-layout families and bloom / falcon / mpt
    (the reference's per-family ``.bin`` conversions: llama, bloom, gptneox,
    starcoder; k-quant blocks are the device layout of ``KQuantLinear``).
"""
from __future__ import annotations

import argparse
import os

import numpy as np
import torch

_OUT_ALIASES = {"int4": "sym_int4", "int8": "sym_int8", "q4_0": "sym_int4", "q4_1": "asym_int4",
                "q5_0": "sym_int5", "q5_1": "asym_int5", "q8_0": "sym_int8"}


def llm_convert(model: str, outfile: str, outtype: str = "int4", model_family: str = "llama",
                model_format: str = "pth", tmp_path: str = None, **kwargs) -> str:
    outtype = outtype.lower()
    if outtype.startswith("gguf"):
        return export_gguf(model, outfile, outtype.split("_", 1)[1] if "_" in outtype else "f16")
    if outtype in ("q4_k", "q5_k", "q6_k", "q2_k", "q4_k_m", "q4_k_s") and str(outfile).endswith(".gguf"):
        return export_gguf(model, outfile, outtype)
    from .transformers import AutoModelForCausalLM
    qtype = _OUT_ALIASES.get(outtype, outtype)
    m = AutoModelForCausalLM.from_pretrained(model, load_in_low_bit=qtype,
                                             torch_dtype=kwargs.get("torch_dtype", torch.float16),
                                             trust_remote_code=kwargs.get("trust_remote_code", False))
    m.save_low_bit(outfile)
    try:
        from transformers import AutoTokenizer
        AutoTokenizer.from_pretrained(model).save_pretrained(outfile)
    except Exception:  # no tokenizer files next to the checkpoint
        pass
    return outfile


def _permute(w: np.ndarray, n_head: int) -> np.ndarray:
    """HF rotate-half rows -> llama.cpp interleaved rows (inverse of gguf.api._unpermute)"""
    out = w.shape[0]
    return w.reshape(n_head, out // n_head // 2, 2, *w.shape[1:]).swapaxes(1, 2).reshape(w.shape)


def export_gguf(model, outfile: str, qtype: str = "f16", tokenizer=None) -> str:
    """Write a llama-family HF model (path or module) as GGUF."""
    from .gguf.reader import F16, F32, Q2_K, Q4_0, Q4_K, Q5_K, Q6_K, Q8_0, GGUFWriter
    if isinstance(model, str):
        from transformers import AutoModelForCausalLM as HF, AutoTokenizer
        src = model
        model = HF.from_pretrained(src, torch_dtype=torch.float32)
        if tokenizer is None:
            try:
                tokenizer = AutoTokenizer.from_pretrained(src)
            except Exception:
                tokenizer = None
    cfg = model.config
    mt = cfg.model_type
    arch = {"llama": "llama", "mistral": "llama", "qwen2": "qwen2", "qwen3": "qwen3"}.get(mt)
    if arch is None and mt not in ("bloom", "falcon", "mpt"):
        raise NotImplementedError(f"GGUF export supports llama/mistral/qwen2/qwen3/bloom/falcon/mpt, not {mt}")
    kq = {"q4_k": Q4_K, "q5_k": Q5_K, "q6_k": Q6_K, "q2_k": Q2_K, "q4_k_m": Q4_K, "q4_k_s": Q4_K}
    tq = {"f32": F32, "f16": F16, "q8_0": Q8_0, "q4_0": Q4_0, **kq}[qtype]

    def mat_type(hf_name, v):
        """k-quants: only rows of 256-multiples; q4_k_m / q4_k_s: llama.cpp's
        mixed policy (quantize/qtypes.mixed_kquant_qtype)"""
        if tq not in kq.values():
            return tq
        if v.shape[-1] % 256:
            return Q8_0 if v.shape[-1] % 32 == 0 else F32
        if qtype in ("q4_k_m", "q4_k_s"):
            from .quantize import qtypes as Qt
            q = Qt.mixed_kquant_qtype("gguf_" + qtype.replace("_k_", "k_"), hf_name, cfg.num_hidden_layers)
            return {Qt.Q6_K: Q6_K, Qt.Q5_K: Q5_K}.get(q, Q4_K)
        return tq
    if arch is None:
        from .gguf.families import export_family_gguf
        emb_t = Q8_0 if tq in kq.values() else tq
        return export_family_gguf(model, outfile, emb_t, mat_type)
    w = GGUFWriter(outfile, arch)
    nh, nkv = cfg.num_attention_heads, getattr(cfg, "num_key_value_heads", cfg.num_attention_heads)
    w.add(f"{arch}.context_length", int(cfg.max_position_embeddings))
    w.add(f"{arch}.embedding_length", int(cfg.hidden_size))
    w.add(f"{arch}.block_count", int(cfg.num_hidden_layers))
    w.add(f"{arch}.feed_forward_length", int(cfg.intermediate_size))
    w.add(f"{arch}.attention.head_count", int(nh))
    w.add(f"{arch}.attention.head_count_kv", int(nkv))
    w.add(f"{arch}.attention.layer_norm_rms_epsilon", float(cfg.rms_norm_eps))
    theta = getattr(cfg, "rope_theta", None) or (getattr(cfg, "rope_parameters", None) or {}).get("rope_theta", 10000.0)
    w.add(f"{arch}.rope.freq_base", float(theta))
    w.add(f"{arch}.vocab_size", int(cfg.vocab_size))
    if tokenizer is not None:
        vocab = tokenizer.get_vocab()
        toks = [""] * len(vocab)
        for t, i in vocab.items():
            if i < len(toks):
                toks[i] = t
        w.add("tokenizer.ggml.model", "gpt2")
        w.add("tokenizer.ggml.tokens", toks)
    sd = {k: v.detach().float().cpu().numpy() for k, v in model.state_dict().items()}
    names = {"input_layernorm": "attn_norm", "post_attention_layernorm": "ffn_norm", "self_attn.q_proj": "attn_q",
             "self_attn.k_proj": "attn_k", "self_attn.v_proj": "attn_v", "self_attn.o_proj": "attn_output",
             "self_attn.q_norm": "attn_q_norm", "self_attn.k_norm": "attn_k_norm", "mlp.gate_proj": "ffn_gate",
             "mlp.up_proj": "ffn_up", "mlp.down_proj": "ffn_down"}
    for k, v in sd.items():
        if k == "model.embed_tokens.weight":
            w.add_tensor("token_embd.weight", v, (Q8_0 if tq in kq.values() else tq) if v.shape[1] % 32 == 0 else F32)
        elif k == "model.norm.weight":
            w.add_tensor("output_norm.weight", v, F32)
        elif k == "lm_head.weight":
            if not getattr(cfg, "tie_word_embeddings", False):
                w.add_tensor("output.weight", v, mat_type("lm_head", v))
        else:
            parts = k.split(".")
            if len(parts) < 5 or parts[1] != "layers":
                continue
            i, rest, wb = parts[2], ".".join(parts[3:-1]), parts[-1]
            g = names.get(rest)
            if g is None:
                continue
            if g in ("attn_q", "attn_k") and arch == "llama":
                v = _permute(v if v.ndim == 2 else v[:, None], nh if g == "attn_q" else nkv)
                v = v if wb == "weight" else v[:, 0]
            is_mat = v.ndim == 2 and v.shape[1] % 32 == 0 and "norm" not in g
            w.add_tensor(f"blk.{i}.{g}.{wb}", v, mat_type(f"model.layers.{i}.{rest}", v) if is_mat else F32)
    w.write()
    return outfile


def main(argv=None):
    ap = argparse.ArgumentParser(description="convert an HF checkpoint to a low-bit directory or GGUF")
    ap.add_argument("model")
    ap.add_argument("--outfile", "-o", required=True)
    ap.add_argument("--outtype", "-t", default="int4")
    ap.add_argument("--model-family", "-x", default="llama")
    a = ap.parse_args(argv)
    print(llm_convert(a.model, a.outfile, a.outtype, a.model_family))


if __name__ == "__main__":
    main()
