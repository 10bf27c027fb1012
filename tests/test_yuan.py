"""Yuan 2.0 localized-filtering attention (models/yuan.py).

* the in-library model's convolutions equal the remote-code formulation
  (``gguf/models/model_implement/yuan2/yuan_hf_model.py:66-133``: Conv2d over
  ``[B, H, S, 1]``, padding 1, first S outputs; the decode step over the
  stored last two hidden states);
* converted to low-bit and run on the native decoder (LFA cache in the
  paged-slot layout), the full-sequence logits and an incremental decode
  through the cache match the float model;
* a Yuan GGUF file (architecture "llama", "yuan" in general.name, lf tensors
  as the reference's loader names them, gguf/models/yuan2.py:66-97) loads
  into the same model.  No Yuan checkpoint ships with the reference: random
  weights, parity against the remote-code formulas, not real outputs."""
import numpy as np
import pytest
import torch

H, NH, L, V, I = 256, 4, 2, 512, 512


def _cfg():
    from ipex_llm_amd.models.yuan import YuanConfig
    return YuanConfig(vocab_size=V, hidden_size=H, intermediate_size=I, num_hidden_layers=L, num_attention_heads=NH,
                      max_position_embeddings=512, rms_norm_eps=1e-6)


def _model(seed=0):
    from ipex_llm_amd.models.yuan import YuanForCausalLM
    torch.manual_seed(seed)
    m = YuanForCausalLM(_cfg()).eval()
    with torch.no_grad():
        for n, p in m.named_parameters():
            if p.dim() == 1:
                p.add_(torch.randn_like(p) * 0.1)
            elif "conv" in n:
                p.mul_(4.0)                       # make the filter matter
    return m


def _remote_lf(lf, x, before=None):
    """the remote code's LocalizedFiltering (train / inference forward), [B, S, H]"""
    inputs = x.transpose(0, 1)
    S, B, E = inputs.shape
    res = inputs
    if before is None:
        t = inputs.view(S, 1, B, E).permute(2, 3, 0, 1)
        o1 = lf.conv1(t)[:, :, :S, :]
        o2 = lf.conv2(o1)[:, :, :S, :].permute(2, 3, 0, 1).contiguous().view(S, B, E)
    else:
        t = torch.cat((before.transpose(0, 1), inputs), 0).view(3, 1, B, E).permute(2, 3, 0, 1)
        o1 = lf.conv1(t)
        o2 = lf.conv2(o1[:, :, 1:-1, :])[:, :, 1:-1, :].view(1, B, E)
    return lf.output_layernorm(o2 + res).transpose(0, 1)


def test_lf_matches_remote_formulation():
    m = _model()
    lf = m.model.layers[0].self_attn.lf_gate
    x = torch.randn(2, 9, H)
    with torch.no_grad():
        torch.testing.assert_close(lf(x), _remote_lf(lf, x), rtol=1e-5, atol=1e-5)
        # decode step: memory = the previous two inputs
        full = lf(x)[:, -1:]
        step = _remote_lf(lf, x[:, -1:], x[:, -3:-1])
        torch.testing.assert_close(full, step, rtol=1e-5, atol=1e-5)


def test_yuan_native_matches_float(tmp_path):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    ref = _model()
    p = str(tmp_path / "yuan")
    ref.save_pretrained(p)
    ids = torch.randint(0, V, (1, 12))
    with torch.no_grad():
        want = ref(ids).logits.float()
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32).eval()
    assert getattr(m, "_illm_native_attached", False), "native decoder not attached"
    from ipex_llm_amd.models.builder import native_from_hf
    nm = native_from_hf(m)
    assert all(L.self_attn.lf is not None for L in nm.layers)
    with torch.no_grad():
        out = m(ids[:, :8], use_cache=True)
        got = out.logits.float()
        rel = ((got - want[:, :8]).norm() / want[:, :8].norm()).item()
        assert rel < 3e-2, rel
        cache = out.past_key_values
        for t in range(8, 12):                  # one token at a time: the filter reads the cached h / o1
            step = m(ids[:, t:t + 1], past_key_values=cache).logits.float()
            r = ((step[:, -1] - want[:, t]).norm() / want[:, t].norm()).item()
            assert r < 3e-2, (t, r)


def test_yuan_native_greedy_equals_chunked(tmp_path):
    """generation through the engine: prompt in one chunk vs the same tokens
    fed one by one give the same greedy continuation (cache addressing)"""
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    ref = _model(1)
    p = str(tmp_path / "y2")
    ref.save_pretrained(p)
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="bf16", torch_dtype=torch.float32).eval()
    ids = torch.randint(0, V, (1, 6))
    with torch.no_grad():
        a = m.generate(ids, max_new_tokens=5, do_sample=False)
        lg = ref(a[:, :-1]).logits.float()
    assert (lg[0, 5:].argmax(-1) == a[0, 6:]).float().mean().item() >= 0.8


def test_yuan_gguf_loads(tmp_path):
    from ipex_llm_amd.gguf import reader as G
    from ipex_llm_amd.gguf.api import load_gguf_model
    ref = _model(2)
    sd = {k: v.float().numpy() for k, v in ref.state_dict().items()}
    f = str(tmp_path / "yuan.gguf")
    w = G.GGUFWriter(f, "llama")
    w.add("general.name", "Yuan2-2B-test")
    for k, v in (("embedding_length", H), ("feed_forward_length", I), ("block_count", L),
                 ("attention.head_count", NH), ("attention.head_count_kv", NH), ("context_length", 512)):
        w.add(f"llama.{k}", v)
    w.add("llama.attention.layer_norm_rms_epsilon", 1e-6)
    w.add("tokenizer.ggml.tokens", [f"t{i}" for i in range(V)])
    w.add_tensor("token_embd.weight", sd["model.embed_tokens.weight"])
    w.add_tensor("output_norm.weight", sd["model.norm.weight"])
    w.add_tensor("output.weight", sd["lm_head.weight"])
    names = {"attn_q": "self_attn.q_proj.weight", "attn_k": "self_attn.k_proj.weight",
             "attn_v": "self_attn.v_proj.weight", "attn_output": "self_attn.o_proj.weight",
             "ffn_gate": "mlp.gate_proj.weight", "ffn_up": "mlp.up_proj.weight", "ffn_down": "mlp.down_proj.weight",
             "attn_norm": "input_layernorm.weight", "ffn_norm": "post_attention_layernorm.weight",
             "lf_output_norm": "self_attn.lf_gate.output_layernorm.weight",
             "conv1.weight": "self_attn.lf_gate.conv1.weight", "conv2.weight": "self_attn.lf_gate.conv2.weight",
             "conv1.bias": "self_attn.lf_gate.conv1.bias", "conv2.bias": "self_attn.lf_gate.conv2.bias"}
    for i in range(L):
        for g, hf in names.items():
            gn = f"blk.{i}.{g}" if "." in g else f"blk.{i}.{g}.weight"
            w.add_tensor(gn, sd[f"model.layers.{i}.{hf}"])
    w.write()
    m, _ = load_gguf_model(f, dtype=torch.float32)
    assert type(m).__name__ == "YuanForCausalLM"
    ids = torch.randint(0, V, (2, 9))
    with torch.no_grad():
        a, b = ref(ids).logits, m(ids).logits
    assert ((a - b).norm() / a.norm()).item() < 1e-5
