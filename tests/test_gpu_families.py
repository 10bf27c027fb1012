"""Non-llama families on the GPU (models/generic.py): LayerNorm kernel,
ALiBi slopes inside the flash-decoding kernel, identity-table rope_kv for
learned positions, partial / interleaved RoPE -- native logits vs the HF
forward (fp32, CPU) of the same weights, and hipGraph decode == eager."""
import pytest
import torch
import transformers as T

pytestmark = pytest.mark.gpu

H, NH, L, V = 256, 4, 2, 512        # head_dim 64: the native decode / prefill kernels


def _cfg(kind):
    if kind == "bloom":
        return T.BloomConfig(hidden_size=H, n_layer=L, n_head=NH, vocab_size=V)
    if kind == "mpt":
        return T.MptConfig(d_model=H, n_layers=L, n_heads=NH, max_seq_len=512, vocab_size=V)
    if kind == "starcoder2":
        return T.Starcoder2Config(hidden_size=H, num_hidden_layers=L, num_attention_heads=NH, num_key_value_heads=2,
                                  intermediate_size=512, max_position_embeddings=512, vocab_size=V)
    if kind == "gpt_neox":
        return T.GPTNeoXConfig(hidden_size=H, num_hidden_layers=L, num_attention_heads=NH, intermediate_size=512,
                               max_position_embeddings=512, vocab_size=V)
    if kind == "gptj":
        return T.GPTJConfig(n_embd=H, n_layer=L, n_head=NH, rotary_dim=32, n_positions=512, vocab_size=V)
    if kind == "gpt_bigcode":
        return T.GPTBigCodeConfig(n_embd=H, n_layer=L, n_head=NH, n_positions=512, vocab_size=V)
    if kind == "falcon_new":
        return T.FalconConfig(hidden_size=H, num_hidden_layers=L, num_attention_heads=NH, num_kv_heads=2,
                              new_decoder_architecture=True, vocab_size=V)
    raise KeyError(kind)


@pytest.mark.parametrize("kind", ["bloom", "mpt", "starcoder2", "gpt_neox", "gptj", "gpt_bigcode", "falcon_new"])
def test_family_gpu_matches_hf(kind, tmp_path):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    torch.manual_seed(0)
    ref = T.AutoModelForCausalLM.from_config(_cfg(kind)).eval()
    with torch.no_grad():
        for n, p in ref.named_parameters():
            if p.dim() == 1:
                p.add_(torch.randn_like(p) * 0.1)
    path = str(tmp_path / kind)
    ref.save_pretrained(path)
    ids = torch.randint(0, V, (1, 40))
    with torch.no_grad():
        want = ref(ids).logits.float()
    m = AutoModelForCausalLM.from_pretrained(path, load_in_low_bit="sym_int8", torch_dtype=torch.bfloat16)
    m = m.to("cuda").eval()
    assert getattr(m, "_illm_native_attached", False)
    with torch.no_grad():
        out = m(ids[:, :32].cuda(), use_cache=True)
        got = out.logits.float().cpu()
        rel = ((got - want[:, :32]).norm() / want[:, :32].norm()).item()
        assert rel < 5e-2, (kind, rel)
        cache = out.past_key_values
        for t in range(32, 40):                 # single-token decode steps (flash-decoding kernel)
            step = m(ids[:, t:t + 1].cuda(), past_key_values=cache).logits.float().cpu()
            r = ((step[:, -1] - want[:, t]).norm() / want[:, t].norm()).item()
            assert r < 5e-2, (kind, t, r)
        g = m.generate(ids[:, :16].cuda(), max_new_tokens=12, do_sample=False, use_graph=True)
        e = m.generate(ids[:, :16].cuda(), max_new_tokens=12, do_sample=False, use_graph=False)
    assert torch.equal(g.cpu(), e.cpu()), kind


def test_mla_deepseek_v3_gpu(tmp_path):
    """absorbed MLA over the paged latent cache on the GPU (bf16): prompt
    logits and decode steps vs the HF fp32 forward, hipGraph decode == eager"""
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    cfg = T.AutoConfig.for_model("deepseek_v3", hidden_size=256, intermediate_size=512, moe_intermediate_size=128,
                                 num_hidden_layers=2, num_attention_heads=8, num_key_value_heads=8, vocab_size=V,
                                 max_position_embeddings=512, n_routed_experts=8, num_experts_per_tok=2, n_group=2,
                                 topk_group=1, n_shared_experts=1, first_k_dense_replace=1, q_lora_rank=128,
                                 kv_lora_rank=128, qk_rope_head_dim=32, qk_nope_head_dim=64, v_head_dim=64)
    torch.manual_seed(0)
    ref = T.AutoModelForCausalLM.from_config(cfg).eval()
    with torch.no_grad():
        for n, p in ref.named_parameters():
            if n.endswith("mlp.gate.weight"):
                p.normal_(0, 1.0)
    path = str(tmp_path / "ds3")
    ref.save_pretrained(path)
    ids = torch.randint(0, V, (1, 40))
    with torch.no_grad():
        want = ref(ids).logits.float()
    m = AutoModelForCausalLM.from_pretrained(path, load_in_low_bit="sym_int8", torch_dtype=torch.bfloat16)
    m = m.to("cuda").eval()
    assert getattr(m, "_illm_native_attached", False)
    with torch.no_grad():
        out = m(ids[:, :32].cuda(), use_cache=True)
        rel = ((out.logits.float().cpu() - want[:, :32]).norm() / want[:, :32].norm()).item()
        assert rel < 6e-2, rel
        cache = out.past_key_values
        for t in range(32, 40):
            step = m(ids[:, t:t + 1].cuda(), past_key_values=cache).logits.float().cpu()
            r = ((step[:, -1] - want[:, t]).norm() / want[:, t].norm()).item()
            assert r < 6e-2, (t, r)
        g = m.generate(ids[:, :16].cuda(), max_new_tokens=12, do_sample=False, use_graph=True)
        e = m.generate(ids[:, :16].cuda(), max_new_tokens=12, do_sample=False, use_graph=False)
    assert torch.equal(g.cpu(), e.cpu())


def test_qwen2_vl_gpu(tmp_path):
    """Qwen2-VL on the GPU: native language model (bf16, head_dim 64) with
    M-RoPE rows for the image prompt, hipGraph decode at cache_len + delta"""
    from ipex_llm_amd.transformers import AutoModelForVision2Seq
    vc = dict(depth=1, embed_dim=64, hidden_size=256, num_heads=4, in_channels=3, patch_size=4, spatial_merge_size=2,
              temporal_patch_size=2, mlp_ratio=2)
    tc = dict(vocab_size=V, hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
              num_key_value_heads=2, max_position_embeddings=1024,
              rope_parameters={"rope_type": "default", "rope_theta": 10000.0, "mrope_section": [8, 12, 12]})
    cfg = T.Qwen2VLConfig(vision_config=vc, text_config=tc, image_token_id=500, video_token_id=501,
                          vision_start_token_id=502, vision_end_token_id=503)
    torch.manual_seed(0)
    ref = T.Qwen2VLForConditionalGeneration(cfg).eval()
    path = str(tmp_path / "qvl")
    ref.save_pretrained(path)
    ids = torch.tensor([[5, 6, 502] + [500] * 16 + [503] + list(range(10, 40))])
    pix, thw = torch.randn(64, 3 * 2 * 4 * 4), torch.tensor([[1, 8, 8]])
    mm = (ids == 500).int()
    with torch.no_grad():
        want = ref(input_ids=ids, pixel_values=pix, image_grid_thw=thw, mm_token_type_ids=mm).logits.float()
    m = AutoModelForVision2Seq.from_pretrained(path, load_in_low_bit="sym_int8", torch_dtype=torch.bfloat16)
    m = m.to("cuda").eval()
    got = m.vl_forward(input_ids=ids.cuda(), pixel_values=pix.cuda(), image_grid_thw=thw.cuda(),
                       mm_token_type_ids=mm.cuda()).logits.float().cpu()
    assert ((got - want).norm() / want.norm()).item() < 5e-2
    g = m.generate(input_ids=ids.cuda(), pixel_values=pix.cuda(), image_grid_thw=thw.cuda(), mm_token_type_ids=mm.cuda(),
                   max_new_tokens=8, use_graph=True)
    e = m.generate(input_ids=ids.cuda(), pixel_values=pix.cuda(), image_grid_thw=thw.cuda(), mm_token_type_ids=mm.cuda(),
                   max_new_tokens=8, use_graph=False)
    assert torch.equal(g.cpu(), e.cpu())


def test_yuan_lfa_gpu(tmp_path):
    """Yuan 2.0 LFA on the native decoder (models/yuan.py): prefill, cached
    single-token steps (the filter reads the slot-addressed h / conv cache)
    and hipGraph decode == eager decode"""
    from ipex_llm_amd.models.yuan import YuanConfig, YuanForCausalLM
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    torch.manual_seed(0)
    ref = YuanForCausalLM(YuanConfig(vocab_size=V, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                                     num_attention_heads=4, max_position_embeddings=512)).eval()
    with torch.no_grad():
        for n, p in ref.named_parameters():
            if p.dim() == 1:
                p.add_(torch.randn_like(p) * 0.1)
            elif "conv" in n:
                p.mul_(4.0)
    path = str(tmp_path / "yuan")
    ref.save_pretrained(path)
    ids = torch.randint(0, V, (1, 40))
    with torch.no_grad():
        want = ref(ids).logits.float()
    m = AutoModelForCausalLM.from_pretrained(path, load_in_low_bit="sym_int8", torch_dtype=torch.bfloat16)
    m = m.to("cuda").eval()
    assert getattr(m, "_illm_native_attached", False)
    with torch.no_grad():
        out = m(ids[:, :32].cuda(), use_cache=True)
        got = out.logits.float().cpu()
        assert ((got - want[:, :32]).norm() / want[:, :32].norm()).item() < 5e-2
        cache = out.past_key_values
        for t in range(32, 40):
            step = m(ids[:, t:t + 1].cuda(), past_key_values=cache).logits.float().cpu()
            r = ((step[:, -1] - want[:, t]).norm() / want[:, t].norm()).item()
            assert r < 5e-2, (t, r)
        g = m.generate(ids[:, :16].cuda(), max_new_tokens=12, do_sample=False, use_graph=True)
        e = m.generate(ids[:, :16].cuda(), max_new_tokens=12, do_sample=False, use_graph=False)
    assert torch.equal(g.cpu(), e.cpu())
