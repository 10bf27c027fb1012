"""Self-speculative decoding on the GPU as captured hipGraph rounds
(generation/spec_graph.py): bf16 target (dequantized INT4 weights) + INT4
draft; the output follows the target's greedy decoding and the rounds ran
from captured graphs."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_graph_speculative_matches_target():
    from transformers import LlamaConfig
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.generation.spec_graph import GraphSpeculator
    from ipex_llm_amd.models.builder import dense_copy, random_native_model
    cfg = LlamaConfig(vocab_size=2048, hidden_size=512, intermediate_size=1024, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=2048)
    dev = torch.device("cuda")
    draft = random_native_model(cfg, "sym_int4", dev, torch.bfloat16, seed=0)
    target = dense_copy(draft)
    te, de = Engine(target), Engine(draft)
    prompt = list(range(3, 60))
    ref = te.generate([prompt], max_new_tokens=40, use_graph=True)[0]
    for k, adaptive in ((2, False), (4, True)):
        sp = GraphSpeculator(te, de, k, 256, k_max=6 if adaptive else k, adaptive=adaptive)
        out = sp.generate(prompt, 40)
        assert len(out) == len(ref)
        agree = sum(int(a == b) for a, b in zip(out, ref)) / len(ref)
        assert agree >= 0.9, (k, agree)
        assert sp.graphs, "no round ran from a captured graph"
        assert sp.acceptance > 0.3, sp.acceptance
