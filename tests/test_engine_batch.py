"""Batched prefill (one [B*n, K] forward) == per-sequence prefill (CPU)."""
import torch
from transformers import LlamaConfig

from ipex_llm_amd.engine.runner import Engine
from ipex_llm_amd.models.builder import random_native_model
from ipex_llm_amd.models.cache import SequenceState


def test_prefill_batch_matches_sequential():
    cfg = LlamaConfig(vocab_size=256, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512)
    m = random_native_model(cfg, "sym_int8", "cpu", torch.float32, seed=0, std=0.2)
    B, n = 3, 21
    ids = torch.randint(0, 256, (B, n), generator=torch.Generator().manual_seed(1))
    e1 = Engine(m)
    e1._ensure_cache(B, 64)
    s1 = [SequenceState(e1.cache.allocator.alloc(1)) for _ in range(B)]
    ref = torch.cat([e1.prefill(s1[b], ids[b]) for b in range(B)])
    e2 = Engine(m)
    e2._ensure_cache(B, 64)
    s2 = [SequenceState(e2.cache.allocator.alloc(1)) for _ in range(B)]
    out = e2.prefill_batch(s2, ids)
    assert out.shape == ref.shape
    assert torch.allclose(out, ref, atol=1e-4, rtol=1e-4)
    assert all(s.length == n for s in s2)
    # the KV written by both paths is identical
    for li in range(len(m.layers)):
        for b in range(B):
            kb1 = e1.cache.k[li][s1[b].blocks[0]]
            kb2 = e2.cache.k[li][s2[b].blocks[0]]
            assert torch.allclose(kb1[:, :n], kb2[:, :n], atol=1e-5)


def test_trace_ranges_recorded_by_torch_profiler():
    """IPEX_LLM_TRACE ranges (roctx + record_function) around prefill / decode
    steps and per decoder layer show up in a torch.profiler trace (CPU run)"""
    import torch
    from transformers import LlamaConfig
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.utils import trace
    cfg = LlamaConfig(vocab_size=128, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=256)
    m = random_native_model(cfg, "sym_int8", "cpu", torch.float32, seed=0)
    trace.enable(True)
    try:
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
            Engine(m).generate([[1, 2, 3, 4]], max_new_tokens=3, use_graph=False)
    finally:
        trace.enable(False)
    names = {e.name for e in prof.events()}
    assert "decode_step" in names and "prefill[4]" in names and "layer1" in names
