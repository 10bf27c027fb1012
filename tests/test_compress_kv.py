"""SnapKV compress-KV (reference kv.py compress_kv): with capacity >= prompt
length nothing changes; with a small capacity generation still runs and the
kept tokens follow the observation window's attention."""
import torch


def _model():
    from transformers import LlamaConfig
    from ipex_llm_amd.models.builder import random_native_model
    cfg = LlamaConfig(vocab_size=128, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=2048)
    return random_native_model(cfg, "sym_int8", "cpu", torch.float32, seed=0, std=0.2)


def test_compress_kv_generation():
    from ipex_llm_amd.engine.runner import Engine
    m = _model()
    prompt = [list(torch.randint(1, 128, (300,), generator=torch.Generator().manual_seed(0)).tolist())]
    ref = Engine(m).generate(prompt, max_new_tokens=8, use_graph=False)
    same = Engine(m).generate(prompt, max_new_tokens=8, use_graph=False, compress_kv=True,
                              compress_capacity=512, compress_window=32)
    assert same == ref                              # prompt shorter than the capacity: untouched
    comp = Engine(m).generate(prompt, max_new_tokens=8, use_graph=False, compress_kv=True,
                              compress_capacity=128, compress_window=32)
    assert len(comp[0]) == 308
    # the first token is produced before compression: identical
    assert comp[0][300] == ref[0][300]
