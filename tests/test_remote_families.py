"""ChatGLM2/3/4 and Qwen v1 checkpoints (remote-code families) loaded through
the tensor mapping of transformers/remote_families.py: a random in-library
Glm / Qwen2 model is written out under the chatglm / qwen tensor names and
config keys (reference SRC/transformers/models/chatglm4.py, qwen.py layouts),
loaded back, and must reproduce the original logits; the low-bit path then
runs it through the native decoder.  Parity against the remote code itself is
unpinned (not importable offline)."""
import json

import pytest
import torch


def _chatglm_dir(tmp_path, mqa=True):
    from transformers import GlmConfig, GlmForCausalLM
    nh, nkv, D, H = 4, (2 if mqa else 4), 16, 64
    cfg = GlmConfig(vocab_size=96, hidden_size=H, intermediate_size=80, num_hidden_layers=2, num_attention_heads=nh,
                    num_key_value_heads=nkv, head_dim=D, rms_norm_eps=1e-5, attention_bias=True, pad_token_id=None,
                    max_position_embeddings=256,
                    rope_parameters={"rope_type": "default", "rope_theta": 10000.0 * 2.0,
                                     "partial_rotary_factor": 0.5})
    torch.manual_seed(0)
    ref = GlmForCausalLM(cfg).eval()
    sd = {}
    g = ref.state_dict()
    sd["transformer.embedding.word_embeddings.weight"] = g["model.embed_tokens.weight"]
    sd["transformer.encoder.final_layernorm.weight"] = g["model.norm.weight"]
    sd["transformer.output_layer.weight"] = g["lm_head.weight"]
    sd["transformer.rotary_pos_emb.inv_freq"] = torch.zeros(D // 4)
    for i in range(cfg.num_hidden_layers):
        p, L = f"model.layers.{i}.", f"transformer.encoder.layers.{i}."
        for kind in ("weight", "bias"):
            sd[L + f"self_attention.query_key_value.{kind}"] = torch.cat(
                [g[p + f"self_attn.{n}_proj.{kind}"] for n in "qkv"], 0)
        sd[L + "self_attention.dense.weight"] = g[p + "self_attn.o_proj.weight"]
        sd[L + "mlp.dense_h_to_4h.weight"] = g[p + "mlp.gate_up_proj.weight"]
        sd[L + "mlp.dense_4h_to_h.weight"] = g[p + "mlp.down_proj.weight"]
        sd[L + "input_layernorm.weight"] = g[p + "input_layernorm.weight"]
        sd[L + "post_attention_layernorm.weight"] = g[p + "post_attention_layernorm.weight"]
    conf = {"model_type": "chatglm", "architectures": ["ChatGLMModel"], "num_layers": 2, "hidden_size": H,
            "ffn_hidden_size": 80, "kv_channels": D, "num_attention_heads": nh, "multi_query_attention": mqa,
            "multi_query_group_num": nkv, "padded_vocab_size": 96, "seq_length": 256, "layernorm_epsilon": 1e-5,
            "add_qkv_bias": True, "rope_ratio": 2.0, "rmsnorm": True, "torch_dtype": "float32"}
    d = tmp_path / "chatglm"
    d.mkdir()
    from safetensors.torch import save_file
    save_file({k: v.contiguous() for k, v in sd.items()}, str(d / "model.safetensors"))
    (d / "config.json").write_text(json.dumps(conf))
    return ref, d


def _qwen_dir(tmp_path):
    from transformers import Qwen2Config, Qwen2ForCausalLM
    H, nh = 64, 4
    cfg = Qwen2Config(vocab_size=96, hidden_size=H, intermediate_size=88, num_hidden_layers=2, num_attention_heads=nh,
                      num_key_value_heads=nh, rms_norm_eps=1e-6, max_position_embeddings=256,
                      rope_parameters={"rope_type": "default", "rope_theta": 10000.0})
    torch.manual_seed(1)
    ref = Qwen2ForCausalLM(cfg).eval()
    g = ref.state_dict()
    sd = {"transformer.wte.weight": g["model.embed_tokens.weight"], "transformer.ln_f.weight": g["model.norm.weight"],
          "lm_head.weight": g["lm_head.weight"]}
    for i in range(cfg.num_hidden_layers):
        p, L = f"model.layers.{i}.", f"transformer.h.{i}."
        for kind in ("weight", "bias"):
            sd[L + f"attn.c_attn.{kind}"] = torch.cat([g[p + f"self_attn.{n}_proj.{kind}"] for n in "qkv"], 0)
        sd[L + "attn.c_proj.weight"] = g[p + "self_attn.o_proj.weight"]
        sd[L + "mlp.w1.weight"] = g[p + "mlp.up_proj.weight"]
        sd[L + "mlp.w2.weight"] = g[p + "mlp.gate_proj.weight"]
        sd[L + "mlp.c_proj.weight"] = g[p + "mlp.down_proj.weight"]
        sd[L + "ln_1.weight"] = g[p + "input_layernorm.weight"]
        sd[L + "ln_2.weight"] = g[p + "post_attention_layernorm.weight"]
    conf = {"model_type": "qwen", "architectures": ["QWenLMHeadModel"], "num_hidden_layers": 2, "hidden_size": H,
            "intermediate_size": 2 * 88, "num_attention_heads": nh, "vocab_size": 96, "seq_length": 256,
            "max_position_embeddings": 256, "layer_norm_epsilon": 1e-6, "rotary_emb_base": 10000.0,
            "rotary_pct": 1.0, "kv_channels": H // nh, "torch_dtype": "float32"}
    d = tmp_path / "qwen"
    d.mkdir()
    torch.save({k: v.contiguous() for k, v in sd.items()}, str(d / "pytorch_model.bin"))
    (d / "config.json").write_text(json.dumps(conf))
    return ref, d


def _internlm_dir(tmp_path):
    from transformers import LlamaConfig, LlamaForCausalLM
    cfg = LlamaConfig(vocab_size=96, hidden_size=64, intermediate_size=96, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=4, attention_bias=True, max_position_embeddings=256, rms_norm_eps=1e-6,
                      rope_parameters={"rope_type": "default", "rope_theta": 10000.0})
    torch.manual_seed(2)
    ref = LlamaForCausalLM(cfg).eval()
    conf = {"model_type": "internlm", "architectures": ["InternLMForCausalLM"], "vocab_size": 96, "hidden_size": 64,
            "intermediate_size": 96, "num_hidden_layers": 2, "num_attention_heads": 4, "bias": True,
            "max_position_embeddings": 256, "rms_norm_eps": 1e-6, "rotary": {"base": 10000, "type": "dynamic"}}
    d = tmp_path / "internlm"
    d.mkdir()
    from safetensors.torch import save_file
    save_file({k: v.contiguous() for k, v in ref.state_dict().items()}, str(d / "model.safetensors"))
    (d / "config.json").write_text(json.dumps(conf))
    return ref, d


def _family_dir(tmp_path, family, mqa=True):
    if family == "chatglm":
        return _chatglm_dir(tmp_path, mqa)
    return _qwen_dir(tmp_path) if family == "qwen" else _internlm_dir(tmp_path)


@pytest.mark.parametrize("family,mqa", [("chatglm", True), ("chatglm", False), ("qwen", False),
                                        ("internlm", False)])
def test_remote_family_mapping_reproduces_logits(tmp_path, family, mqa):
    from ipex_llm_amd.transformers.remote_families import family_of, load_remote_family
    ref, d = _family_dir(tmp_path, family, mqa)
    assert family_of(str(d)) == family
    m = load_remote_family(str(d), torch.float32)
    ids = torch.randint(0, 96, (2, 12), generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        want = ref(ids).logits
        got = m(ids).logits
    assert torch.allclose(got, want, atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("family", ["chatglm", "qwen", "internlm"])
def test_remote_family_low_bit_native(tmp_path, family):
    """from_pretrained(load_in_low_bit) on a chatglm / qwen directory: native
    decoder over low-bit weights, logits close to the dense original"""
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    ref, d = _family_dir(tmp_path, family)
    m = AutoModelForCausalLM.from_pretrained(str(d), load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    assert getattr(m.config, "illm_source_model_type", None) == family
    ids = torch.randint(0, 96, (1, 10), generator=torch.Generator().manual_seed(4))
    with torch.no_grad():
        want = ref(ids).logits.float()
        got = m(ids).logits.float()
    rel = ((got - want).norm() / want.norm()).item()
    assert rel < 3e-2, rel
    out = m.generate(ids, max_new_tokens=4, do_sample=False)
    assert out.shape[1] == 14
