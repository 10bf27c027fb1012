"""Prompt-lookup and self-speculative decoding produce exactly the greedy
output of the target model (reference: lookup.py / speculative.py)."""
import torch


def _tiny(tmp_path):
    from transformers import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=64, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512)
    m = LlamaForCausalLM(cfg).eval()
    p = str(tmp_path / "m")
    m.save_pretrained(p)
    return p


def test_lookup_matches_greedy(tmp_path):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    p = _tiny(tmp_path)
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    # repetitive prompt: n-gram candidates exist
    ids = torch.tensor([[5, 6, 7, 8, 9, 5, 6, 7, 8, 9, 5, 6, 7, 8, 9, 5, 6]])
    ref = m.generate(ids, max_new_tokens=20)
    out = m.generate(ids, max_new_tokens=20, prompt_lookup_num_tokens=4)
    assert torch.equal(out, ref)
    from ipex_llm_amd.transformers.hf_native import get_native
    st = get_native(m)[1].lookup_stats
    assert st["drafted"] > 0


def test_candidate_table():
    from ipex_llm_amd.generation.lookup import PromptLookupCandidates
    g = PromptLookupCandidates(num_output_tokens=3, max_matching_ngram_size=2)
    g.init([1, 2, 3, 4, 1, 2])
    assert g.candidates() == [3, 4, 1]
    g.extend([9])
    assert g.candidates() == []


def test_candidate_count_policy_matches_reference():
    """reference update_candidate_strategy (lookup.py:253-270): +1 capped at 9
    on full acceptance, never below 0, re-enabled from 0 by the acceptance rate"""
    from ipex_llm_amd.generation.lookup import PromptLookupCandidates
    g = PromptLookupCandidates(num_output_tokens=8, seed=0)
    g.update(8, 8)
    assert g.num_output_tokens == 9
    g.update(9, 9)
    assert g.num_output_tokens == 9                  # max_candidates
    assert g.accept_rate == 1.0
    # many rejections with a low acceptance rate walk it down to 0 (min_candidates)
    for _ in range(40):
        g.update(g.num_output_tokens, 0)
    assert g.num_output_tokens == 0 and g.candidates() == []
    assert 0.0 < g.accept_rate < 0.5
    # at 0 drafts the re-enable probability is accept_rate + 0.15
    hits = 0
    for i in range(400):
        h = PromptLookupCandidates(num_output_tokens=0, seed=i)
        h.update(0, 0, accept_rate=0.35)
        hits += h.num_output_tokens == 1
    assert 0.35 < hits / 400 < 0.65


def test_self_speculative_matches_target_greedy(tmp_path):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    p = _tiny(tmp_path)
    tgt = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="bf16", torch_dtype=torch.float32)
    ids = torch.randint(0, 64, (1, 9), generator=torch.Generator().manual_seed(2))
    ref = tgt.generate(ids, max_new_tokens=24)
    spec = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="bf16", torch_dtype=torch.float32,
                                                speculative=True)
    out = spec.generate(ids, max_new_tokens=24)
    assert torch.equal(out, ref)
    assert spec.n_drafted > 0 and spec.n_matched > 0


def test_graph_speculator_eager_matches_target_greedy(tmp_path):
    """the device-resident round (generation/spec_graph.py) run eagerly on the
    host: same tokens as the target's plain greedy decoding, for several
    draft lengths, adaptive or not"""
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from ipex_llm_amd.transformers.hf_native import get_native
    from ipex_llm_amd.generation.spec_graph import GraphSpeculator
    p = _tiny(tmp_path)
    tgt = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="bf16", torch_dtype=torch.float32)
    dft = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int4", torch_dtype=torch.float32)
    ids = torch.randint(0, 64, (1, 9), generator=torch.Generator().manual_seed(2))
    ref = tgt.generate(ids, max_new_tokens=24)[0].tolist()
    te, de = get_native(tgt)[1], get_native(dft)[1]
    for k, adaptive in ((1, False), (3, False), (2, True)):
        sp = GraphSpeculator(te, de, k, 128, use_graph=False, k_max=5 if adaptive else k, adaptive=adaptive)
        out = sp.generate(ids[0].tolist(), 24)
        assert out == ref, (k, adaptive)
        assert sp.rounds > 0 and 0.0 <= sp.acceptance <= 1.0
        # a second call reuses the speculator (graph keys / buffers)
        assert sp.generate(ids[0].tolist(), 10) == ref[:9 + 10]
