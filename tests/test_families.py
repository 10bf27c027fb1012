"""Model-family coverage on CPU: every architecture the reference optimises
 loads through ``from_pretrained(load_in_low_bit=...)``, its
logits stay close to the dense HF model, and ``generate`` runs.

Families the native decoder covers run natively; the rest keep the HF forward
over low-bit linears (the reference's per-arch forward swap,
``SRC/transformers/convert.py:1275-2139``).  Random tiny configs, no
checkpoints (no network)."""
import pytest
import torch

H, I, L, V = 64, 128, 2, 256

FAMILIES = {
    "gpt2": dict(n_embd=H, n_layer=L, n_head=4, vocab_size=V, n_positions=128),
    "gpt_neox": dict(hidden_size=H, intermediate_size=I, num_hidden_layers=L, num_attention_heads=4,
                     vocab_size=V, max_position_embeddings=128),
    "bloom": dict(hidden_size=H, n_layer=L, n_head=4, vocab_size=V),
    "falcon": dict(hidden_size=H, num_hidden_layers=L, num_attention_heads=4, vocab_size=V,
                   new_decoder_architecture=False, multi_query=True),
    "phi": dict(hidden_size=H, intermediate_size=I, num_hidden_layers=L, num_attention_heads=4, vocab_size=V,
                max_position_embeddings=128),
    "mpt": dict(d_model=H, n_layers=L, n_heads=4, vocab_size=V, max_seq_len=128),
    "gpt_bigcode": dict(n_embd=H, n_layer=L, n_head=4, vocab_size=V, n_positions=128),
    "starcoder2": dict(hidden_size=H, intermediate_size=I, num_hidden_layers=L, num_attention_heads=4,
                       num_key_value_heads=2, vocab_size=V, max_position_embeddings=128),
    "stablelm": dict(hidden_size=H, intermediate_size=I, num_hidden_layers=L, num_attention_heads=4,
                     num_key_value_heads=2, vocab_size=V, max_position_embeddings=128),
    "gptj": dict(n_embd=H, n_layer=L, n_head=4, vocab_size=V, n_positions=128, rotary_dim=8),
    "opt": dict(hidden_size=H, ffn_dim=I, num_hidden_layers=L, num_attention_heads=4, vocab_size=V,
                word_embed_proj_dim=H, max_position_embeddings=128),
    "codegen": dict(n_embd=H, n_layer=L, n_head=4, vocab_size=V, n_positions=128, rotary_dim=8),
    "olmo": dict(hidden_size=H, intermediate_size=I, num_hidden_layers=L, num_attention_heads=4, vocab_size=V,
                 max_position_embeddings=128),
    "granite": dict(hidden_size=H, intermediate_size=I, num_hidden_layers=L, num_attention_heads=4,
                    num_key_value_heads=2, vocab_size=V, max_position_embeddings=128,
                    embedding_multiplier=2.0, residual_multiplier=0.5, logits_scaling=2.0,
                    attention_multiplier=0.1),
    "cohere": dict(hidden_size=H, intermediate_size=I, num_hidden_layers=L, num_attention_heads=4,
                   num_key_value_heads=2, vocab_size=V, max_position_embeddings=128),
    "mixtral": dict(hidden_size=H, intermediate_size=I, num_hidden_layers=L, num_attention_heads=4,
                    num_key_value_heads=2, vocab_size=V, max_position_embeddings=128, num_local_experts=4,
                    num_experts_per_tok=2),
    "rwkv": dict(hidden_size=H, num_hidden_layers=L, attention_hidden_size=H, intermediate_size=I, vocab_size=V,
                 context_length=128, rescale_every=1),
    "deepseek_v3": dict(hidden_size=H, intermediate_size=I, moe_intermediate_size=32, num_hidden_layers=L,
                        num_attention_heads=4, num_key_value_heads=4, vocab_size=V, max_position_embeddings=128,
                        n_routed_experts=8, num_experts_per_tok=2, n_group=4, topk_group=2, n_shared_experts=1,
                        first_k_dense_replace=1, q_lora_rank=32, kv_lora_rank=32, qk_rope_head_dim=16,
                        qk_nope_head_dim=16, v_head_dim=16, rope_interleave=True),
    "qwen2_moe": dict(hidden_size=H, intermediate_size=I, moe_intermediate_size=64,
                      shared_expert_intermediate_size=I, num_hidden_layers=L, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=V, max_position_embeddings=128, num_experts=4,
                      num_experts_per_tok=2),
}


def _build(mt, path):
    from transformers import AutoConfig, AutoModelForCausalLM
    cfg = AutoConfig.for_model(mt, **FAMILIES[mt])
    torch.manual_seed(0)
    m = AutoModelForCausalLM.from_config(cfg).eval()
    with torch.no_grad():
        for n, p in m.named_parameters():
            if p.dim() >= 2 and "embed" not in n and "wte" not in n and "wpe" not in n:
                p.normal_(0, 0.05)
            if n.endswith(".gate.weight"):
                p.normal_(0, 1.0)          # decisive routing: quantization noise must not flip experts
    m.save_pretrained(path)
    return m


@pytest.mark.parametrize("mt", sorted(FAMILIES))
def test_family_lowbit_logits_and_generate(mt, tmp_path):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    p = str(tmp_path / mt)
    try:
        ref = _build(mt, p)
    except (ValueError, KeyError, ImportError) as e:      # family absent from this transformers
        pytest.skip(f"{mt}: {e}")
    ids = torch.randint(3, V, (1, 10), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        want = ref(ids).logits.float()
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    with torch.no_grad():
        got = m(ids).logits.float()
    rel = ((got - want).norm() / want.norm()).item()
    assert rel < 6e-2, (mt, rel)
    out = m.generate(ids, max_new_tokens=4, min_new_tokens=4, do_sample=False)
    assert out.shape == (1, 14), (mt, out.shape)
