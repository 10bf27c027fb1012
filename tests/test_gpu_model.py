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


@pytest.mark.gpu
def test_compress_kv_graph_decode_on_gpu(cuda):
    """compressed KV (pos_offset) through the fused RoPE + decode_advance kernels"""
    from transformers import LlamaConfig
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.models.builder import random_native_model
    cfg = LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=4096)
    m = random_native_model(cfg, "sym_int4", cuda, torch.bfloat16, seed=0)
    prompt = [list(range(1, 400))]
    eager = Engine(m).generate(prompt, max_new_tokens=12, use_graph=False, compress_kv=True,
                               compress_capacity=192, compress_window=32)
    graph = Engine(m).generate(prompt, max_new_tokens=12, use_graph=True, compress_kv=True,
                               compress_capacity=192, compress_window=32)
    assert eager == graph and len(graph[0]) == 399 + 12
