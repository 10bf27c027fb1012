"""Hook-parity tests for the non-llama families on the native decoder
(models/generic.py): a tiny random-init HF model of each layout is saved,
loaded through ``AutoModelForCausalLM.from_pretrained(load_in_low_bit=...)``
and its full-sequence logits (native forward) plus an incremental decode
step through the paged cache are compared with the HF forward of the same
weights -- the reference's ``test/inference_gpu/test_transformers_api_attention.py``
pattern (optimized forward vs original forward on the same input).

sym_int8 weights: a wrong QKV row order / residual wiring / position scheme
gives O(1) errors, int8 rounding stays at ~1e-2."""
import pytest
import torch
import transformers as T

from ipex_llm_amd.models.generic import alibi_slopes

H, NH, L, V = 128, 4, 2, 256


def _mk(kind):
    c = dict(vocab_size=V)
    if kind == "bloom":
        return T.BloomConfig(hidden_size=H, n_layer=L, n_head=NH, **c)
    if kind == "bloom6":                    # non-power-of-two heads: extra ALiBi slopes
        return T.BloomConfig(hidden_size=192, n_layer=L, n_head=6, **c)
    if kind == "mpt":
        return T.MptConfig(d_model=H, n_layers=L, n_heads=NH, max_seq_len=256, **c)
    if kind == "gpt_bigcode":
        return T.GPTBigCodeConfig(n_embd=H, n_layer=L, n_head=NH, n_positions=256, **c)
    if kind == "gpt_bigcode_mha":
        return T.GPTBigCodeConfig(n_embd=H, n_layer=L, n_head=NH, n_positions=256, multi_query=False, **c)
    if kind == "gpt2":
        return T.GPT2Config(n_embd=H, n_layer=L, n_head=NH, n_positions=256, **c)
    if kind == "starcoder2":
        return T.Starcoder2Config(hidden_size=H, num_hidden_layers=L, num_attention_heads=NH, num_key_value_heads=2,
                                  intermediate_size=256, max_position_embeddings=256, **c)
    if kind == "gpt_neox":
        return T.GPTNeoXConfig(hidden_size=H, num_hidden_layers=L, num_attention_heads=NH, intermediate_size=256,
                               max_position_embeddings=256, **c)
    if kind == "gpt_neox_seq":
        return T.GPTNeoXConfig(hidden_size=H, num_hidden_layers=L, num_attention_heads=NH, intermediate_size=256,
                               max_position_embeddings=256, use_parallel_residual=False, **c)
    if kind == "phi":
        return T.PhiConfig(hidden_size=H, num_hidden_layers=L, num_attention_heads=NH, intermediate_size=256,
                           max_position_embeddings=256, **c)
    if kind == "falcon":                    # falcon-7b: multi-query, one shared norm
        return T.FalconConfig(hidden_size=H, num_hidden_layers=L, num_attention_heads=NH, **c)
    if kind == "falcon_new":                # falcon-40b/180b: grouped KV, two norms
        return T.FalconConfig(hidden_size=H, num_hidden_layers=L, num_attention_heads=NH, num_kv_heads=2,
                              new_decoder_architecture=True, **c)
    if kind == "falcon_seq":
        return T.FalconConfig(hidden_size=H, num_hidden_layers=L, num_attention_heads=NH, multi_query=False,
                              parallel_attn=False, bias=True, **c)
    if kind == "gptj":
        return T.GPTJConfig(n_embd=H, n_layer=L, n_head=NH, rotary_dim=16, n_positions=256, **c)
    if kind == "stablelm":
        return T.StableLmConfig(hidden_size=H, num_hidden_layers=L, num_attention_heads=NH, num_key_value_heads=2,
                                intermediate_size=256, max_position_embeddings=256, use_qkv_bias=True, **c)
    raise KeyError(kind)


KINDS = ["bloom", "bloom6", "mpt", "gpt_bigcode", "gpt_bigcode_mha", "gpt2", "starcoder2", "gpt_neox",
         "gpt_neox_seq", "phi", "falcon", "falcon_new", "falcon_seq", "gptj", "stablelm"]


def _hf(kind, path):
    torch.manual_seed(0)
    m = T.AutoModelForCausalLM.from_config(_mk(kind)).eval()
    with torch.no_grad():                   # LayerNorm params off their 1/0 init so the wiring matters
        for n, p in m.named_parameters():
            if p.dim() == 1:
                p.add_(torch.randn_like(p) * 0.1)
    m.save_pretrained(path)
    return m


@pytest.mark.parametrize("kind", KINDS)
def test_family_native_matches_hf(kind, tmp_path):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    p = str(tmp_path / kind)
    ref = _hf(kind, p)
    ids = torch.randint(0, V, (1, 12))
    with torch.no_grad():
        want = ref(ids).logits.float()
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32).eval()
    assert getattr(m, "_illm_native_attached", False), f"{kind}: native decoder not attached"
    from ipex_llm_amd.models.builder import native_from_hf
    assert type(native_from_hf(m)).__name__ == "GenericCausalLM"
    with torch.no_grad():
        out = m(ids[:, :8], use_cache=True)
        got = out.logits.float()
        rel = ((got - want[:, :8]).norm() / want[:, :8].norm()).item()
        assert rel < 3e-2, (kind, rel)
        # 4 more tokens one at a time through the paged cache (decode path)
        cache = out.past_key_values
        for t in range(8, 12):
            step = m(ids[:, t:t + 1], past_key_values=cache).logits.float()
            r = ((step[:, -1] - want[:, t]).norm() / want[:, t].norm()).item()
            assert r < 3e-2, (kind, t, r)


def test_generate_matches_hf_greedy(tmp_path):
    """bloom (ALiBi) greedy generation through the engine == HF generate"""
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    p = str(tmp_path / "b")
    ref = _hf("bloom", p)
    ids = torch.randint(0, V, (1, 10))
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="bf16", torch_dtype=torch.float32).eval()
    m16 = T.AutoModelForCausalLM.from_pretrained(p, torch_dtype=torch.bfloat16).eval()
    with torch.no_grad():
        a = m.generate(ids, max_new_tokens=6, do_sample=False)
        lg = m(a[:, :-1]).logits.float()
        b = m16(a[:, :-1]).logits.float()
    # our greedy tokens are the argmax of the HF (bf16 weights) logits at each step
    assert (lg[0, 9:].argmax(-1) == a[0, 10:]).all()
    assert ((lg - b).norm() / b.norm()).item() < 3e-2


def test_alibi_slopes_match_hf():
    from transformers.models.bloom.modeling_bloom import build_alibi_tensor
    for n in (4, 6, 12, 16):
        mask = torch.ones(1, 5)
        a = build_alibi_tensor(mask, n, torch.float32).view(n, 5)
        torch.testing.assert_close(a[:, 1], alibi_slopes(n))
    from transformers.models.mpt.modeling_mpt import build_mpt_alibi_tensor
    for n in (4, 6, 8):
        a = build_mpt_alibi_tensor(n, 5).view(n, 5)      # (k - 4) * slope
        torch.testing.assert_close(a[:, -1] - a[:, -2], alibi_slopes(n, "mpt"))


def test_unsupported_variant_keeps_hf_forward(tmp_path):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    p = str(tmp_path / "phiqk")
    torch.manual_seed(0)
    cfg = T.PhiConfig(hidden_size=H, num_hidden_layers=1, num_attention_heads=NH, intermediate_size=256,
                      vocab_size=V, qk_layernorm=True)
    ref = T.AutoModelForCausalLM.from_config(cfg).eval()
    ref.save_pretrained(p)
    ids = torch.randint(0, V, (1, 7))
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32).eval()
    assert not getattr(m, "_illm_native_attached", False)
    with torch.no_grad():
        a, b = m(ids).logits, ref(ids).logits
    assert ((a - b).norm() / b.norm()).item() < 3e-2


@pytest.mark.parametrize("kind", ["bloom", "falcon_new", "gpt_neox"])
def test_family_low_bit_round_trip(kind, tmp_path):
    """save_low_bit / load_low_bit of a rewritten (re-ordered QKV) model"""
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    p = str(tmp_path / kind)
    _hf(kind, p)
    ids = torch.randint(0, V, (1, 9))
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int4", torch_dtype=torch.float32).eval()
    with torch.no_grad():
        a = m(ids).logits
    sd = str(tmp_path / "saved")
    m.save_low_bit(sd)
    m2 = AutoModelForCausalLM.load_low_bit(sd, torch_dtype=torch.float32).eval()
    assert getattr(m2, "_illm_native_attached", False)
    with torch.no_grad():
        assert torch.allclose(m2(ids).logits, a, atol=1e-5)


@pytest.mark.parametrize("kind", ["glm", "glm4"])
def test_glm_native_matches_hf(kind, tmp_path):
    """GLM / GLM-4 (ChatGLM-4 layout): interleaved partial RoPE, qkv bias,
    fused [gate; up], GLM-4 sandwich norms -- on the llama-native decoder"""
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    C = T.GlmConfig if kind == "glm" else T.Glm4Config
    cfg = C(vocab_size=V, hidden_size=H, num_hidden_layers=L, num_attention_heads=NH, num_key_value_heads=2,
            head_dim=32, intermediate_size=256, max_position_embeddings=256, pad_token_id=0, eos_token_id=1,
            bos_token_id=1)
    torch.manual_seed(0)
    ref = T.AutoModelForCausalLM.from_config(cfg).eval()
    with torch.no_grad():
        for n, p_ in ref.named_parameters():
            if p_.dim() == 1:
                p_.add_(torch.randn_like(p_) * 0.1)
    p = str(tmp_path / kind)
    ref.save_pretrained(p)
    ids = torch.randint(0, V, (1, 12))
    with torch.no_grad():
        want = ref(ids).logits.float()
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32).eval()
    assert getattr(m, "_illm_native_attached", False)
    with torch.no_grad():
        out = m(ids[:, :8], use_cache=True)
        rel = ((out.logits.float() - want[:, :8]).norm() / want[:, :8].norm()).item()
        assert rel < 3e-2, rel
        cache = out.past_key_values
        for t in range(8, 12):
            step = m(ids[:, t:t + 1], past_key_values=cache).logits.float()
            r = ((step[:, -1] - want[:, t]).norm() / want[:, t].norm()).item()
            assert r < 3e-2, (t, r)


def _mla_cfg(kind):
    if kind == "deepseek_v3":
        return T.AutoConfig.for_model("deepseek_v3", hidden_size=128, intermediate_size=256, moe_intermediate_size=64,
                                      num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=4,
                                      vocab_size=V, max_position_embeddings=256, n_routed_experts=8,
                                      num_experts_per_tok=2, n_group=2, topk_group=1, n_shared_experts=1,
                                      first_k_dense_replace=1, q_lora_rank=64, kv_lora_rank=64, qk_rope_head_dim=16,
                                      qk_nope_head_dim=32, v_head_dim=32)
    if kind == "deepseek_v3_noq":            # q_lora_rank None (V2-Lite style q_proj)
        return T.AutoConfig.for_model("deepseek_v3", hidden_size=128, intermediate_size=256, moe_intermediate_size=64,
                                      num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=4,
                                      vocab_size=V, max_position_embeddings=256, n_routed_experts=8,
                                      num_experts_per_tok=2, n_group=2, topk_group=1, n_shared_experts=1,
                                      first_k_dense_replace=1, q_lora_rank=None, kv_lora_rank=64,
                                      qk_rope_head_dim=16, qk_nope_head_dim=32, v_head_dim=32, rope_interleave=False)
    if kind == "minicpm3":
        return T.AutoConfig.for_model("minicpm3", hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                                      num_attention_heads=4, num_key_value_heads=4, vocab_size=V,
                                      max_position_embeddings=256, q_lora_rank=64, kv_lora_rank=64,
                                      qk_rope_head_dim=16, qk_nope_head_dim=32, v_head_dim=32)
    raise KeyError(kind)


@pytest.mark.parametrize("kind", ["deepseek_v3", "deepseek_v3_noq", "minicpm3"])
def test_mla_native_matches_hf(kind, tmp_path):
    """absorbed-weight MLA over the paged latent cache vs the HF forward"""
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from ipex_llm_amd.models.builder import native_from_hf
    torch.manual_seed(0)
    ref = T.AutoModelForCausalLM.from_config(_mla_cfg(kind)).eval()
    with torch.no_grad():
        for n, p_ in ref.named_parameters():
            if p_.dim() == 1 and "norm" in n:
                p_.add_(torch.randn_like(p_) * 0.1)
            if n.endswith("mlp.gate.weight"):
                p_.normal_(0, 1.0)
    p = str(tmp_path / kind)
    ref.save_pretrained(p)
    ids = torch.randint(0, V, (1, 12))
    with torch.no_grad():
        want = ref(ids).logits.float()
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32).eval()
    assert getattr(m, "_illm_native_attached", False)
    nm = native_from_hf(m)
    assert type(nm).__name__ == "MLACausalLM"
    with torch.no_grad():
        out = m(ids[:, :8], use_cache=True)
        rel = ((out.logits.float() - want[:, :8]).norm() / want[:, :8].norm()).item()
        assert rel < 3e-2, rel
        cache = out.past_key_values
        # the paged cache holds the latent rows only: [c_kv | k_pe]
        assert cache.engine.cache.k[0].shape[-1] == 64 + 16 and cache.engine.cache.k[0].shape[1] == 1
        for t in range(8, 12):
            step = m(ids[:, t:t + 1], past_key_values=cache).logits.float()
            r = ((step[:, -1] - want[:, t]).norm() / want[:, t].norm()).item()
            assert r < 3e-2, (t, r)
        g = m.generate(ids[:, :6], max_new_tokens=5, do_sample=False)
    # greedy continuation agrees with the HF argmax of the same prefix
    with torch.no_grad():
        lg = ref(g[:, :-1]).logits
    assert (lg[0, 5:].argmax(-1) == g[0, 6:]).float().mean() >= 0.8


def _qwen2vl(tmp_path):
    vc = dict(depth=1, embed_dim=64, hidden_size=128, num_heads=4, in_channels=3, patch_size=4, spatial_merge_size=2,
              temporal_patch_size=2, mlp_ratio=2)
    tc = dict(vocab_size=V, hidden_size=H, intermediate_size=256, num_hidden_layers=L, num_attention_heads=NH,
              num_key_value_heads=2, max_position_embeddings=512,
              rope_parameters={"rope_type": "default", "rope_theta": 10000.0, "mrope_section": [4, 6, 6]})
    cfg = T.Qwen2VLConfig(vision_config=vc, text_config=tc, image_token_id=250, video_token_id=251,
                          vision_start_token_id=252, vision_end_token_id=253)
    torch.manual_seed(0)
    m = T.Qwen2VLForConditionalGeneration(cfg).eval()
    p = str(tmp_path / "qwen2vl")
    m.save_pretrained(p)
    ids = torch.tensor([[5, 6, 252] + [250] * 4 + [253, 7, 8, 9]])
    pix = torch.randn(16, 3 * 2 * 4 * 4)
    thw = torch.tensor([[1, 4, 4]])
    return m, p, ids, pix, thw


def test_qwen2_vl_native_mrope_matches_hf(tmp_path):
    """Qwen2-VL: HF vision tower + native language model with M-RoPE rows;
    prompt logits match HF, and decoding continues at cache_len + rope_delta"""
    from ipex_llm_amd.transformers import AutoModelForVision2Seq
    ref, p, ids, pix, thw = _qwen2vl(tmp_path)
    mm = (ids == 250).int()
    with torch.no_grad():
        want = ref(input_ids=ids, pixel_values=pix, image_grid_thw=thw, mm_token_type_ids=mm).logits.float()
    m = AutoModelForVision2Seq.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32).eval()
    assert getattr(m, "_illm_native_attached", False)
    got = m.vl_forward(input_ids=ids, pixel_values=pix, image_grid_thw=thw, mm_token_type_ids=mm).logits.float()
    rel = ((got - want).norm() / want.norm()).item()
    assert rel < 3e-2, rel
    out = m.generate(input_ids=ids, pixel_values=pix, image_grid_thw=thw, mm_token_type_ids=mm, max_new_tokens=6)
    # each generated token is the argmax of the HF model over the growing sequence
    seq = out[0].tolist()
    for t in range(ids.shape[1], len(seq)):
        x = torch.tensor([seq[:t]])
        with torch.no_grad():
            lg = ref(input_ids=x, pixel_values=pix, image_grid_thw=thw,
                     mm_token_type_ids=(x == 250).int()).logits[0, -1]
        top2 = lg.topk(2).values
        assert seq[t] == int(lg.argmax()) or (top2[0] - top2[1]).abs() < 1e-2, t
    # text-only prompts: plain native generate (M-RoPE == RoPE)
    txt = torch.tensor([[5, 6, 7, 8]])
    assert m.generate(txt, max_new_tokens=3).shape == (1, 7)


def test_qwen2_5_vl_native_matches_hf(tmp_path):
    from ipex_llm_amd.transformers import AutoModelForVision2Seq
    vc = dict(depth=2, hidden_size=64, intermediate_size=128, num_heads=4, in_channels=3, patch_size=4,
              spatial_merge_size=2, temporal_patch_size=2, window_size=16, out_hidden_size=H,
              fullatt_block_indexes=[1])
    tc = dict(vocab_size=V, hidden_size=H, intermediate_size=256, num_hidden_layers=L, num_attention_heads=NH,
              num_key_value_heads=2, max_position_embeddings=512,
              rope_parameters={"rope_type": "default", "rope_theta": 10000.0, "mrope_section": [4, 6, 6]})
    cfg = T.Qwen2_5_VLConfig(vision_config=vc, text_config=tc, image_token_id=250, video_token_id=251,
                             vision_start_token_id=252, vision_end_token_id=253)
    torch.manual_seed(0)
    ref = T.Qwen2_5_VLForConditionalGeneration(cfg).eval()
    p = str(tmp_path / "q25vl")
    ref.save_pretrained(p)
    ids = torch.tensor([[5, 6, 252] + [250] * 4 + [253, 7, 8, 9]])
    pix, thw, mm = torch.randn(16, 3 * 2 * 4 * 4), torch.tensor([[1, 4, 4]]), (ids == 250).int()
    with torch.no_grad():
        want = ref(input_ids=ids, pixel_values=pix, image_grid_thw=thw, mm_token_type_ids=mm).logits.float()
    m = AutoModelForVision2Seq.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32).eval()
    got = m.vl_forward(input_ids=ids, pixel_values=pix, image_grid_thw=thw, mm_token_type_ids=mm).logits.float()
    assert ((got - want).norm() / want.norm()).item() < 3e-2
