"""End-to-end native decoder on the GPU: eager vs hipGraph decode parity and
GPU vs host (C++ CPU GEMM) logits parity on the same quantized weights."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cfg(layers=2):
    from transformers import LlamaConfig
    return LlamaConfig(vocab_size=1024, hidden_size=512, intermediate_size=1024, num_hidden_layers=layers,
                       num_attention_heads=8, num_key_value_heads=2, max_position_embeddings=4096)


def test_graph_vs_eager_decode(cuda):
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.engine.runner import Engine
    m = random_native_model(_cfg(), "sym_int4", cuda, torch.bfloat16, seed=3)
    e = Engine(m)
    prompts = [list(range(1, 40)), list(range(5, 90))]
    a = e.generate(prompts, max_new_tokens=24, use_graph=False)
    b = e.generate(prompts, max_new_tokens=24, use_graph=True)
    assert a == b


def test_gpu_vs_cpu_logits(cuda):
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.engine.runner import Engine
    m = random_native_model(_cfg(), "sym_int4", cuda, torch.bfloat16, seed=5)
    ids = torch.arange(3, 70)
    eg = Engine(m)
    from ipex_llm_amd.models.cache import SequenceState
    eg._ensure_cache(1, 128)
    s = SequenceState(eg.cache.allocator.alloc(2))
    lg = eg.prefill(s, ids).float().cpu()
    mc = m.to("cpu")
    ec = Engine(mc)
    ec._ensure_cache(1, 128)
    s2 = SequenceState(ec.cache.allocator.alloc(2))
    lc = ec.prefill(s2, ids).float()
    rel = ((lg - lc).norm() / lc.norm()).item()
    assert rel < 3e-2, rel
