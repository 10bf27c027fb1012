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


@pytest.mark.parametrize("B,n", [(1, 200), (4, 520)])
def test_graph_prefill_matches_eager(cuda, B, n):
    """Engine.prefill_batch(use_graph=True): captured once per shape (first
    call: warm-up + capture + replay), later calls replay with new prompts /
    slots / block tables -- logits and the written KV (via the following
    graph decode) equal the eager prefill's"""
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.models.cache import SequenceState
    m = random_native_model(_cfg(), "sym_int4", cuda, torch.bfloat16, seed=11)
    e = Engine(m)
    max_len = n + 32
    e._ensure_cache(2 * B, max_len)
    nblk = (max_len + e.block_size - 1) // e.block_size
    g = torch.Generator().manual_seed(1)
    res = {}
    for trial in range(3):                       # trial 0 captures, 1-2 replay (new prompts on trial 2)
        prompts = torch.randint(0, 1024, (B, n), generator=g if trial == 2 else torch.Generator().manual_seed(0))
        for mode in (False, True):
            e.cache.allocator = type(e.cache.allocator)(e.cache.num_blocks)
            seqs = [SequenceState(e.cache.allocator.alloc(nblk)) for _ in range(B)]
            if mode:                             # different blocks than the eager run: the table is an input
                seqs = [SequenceState(e.cache.allocator.alloc(nblk)) for _ in range(B)]
            lg = e.prefill_batch(seqs, prompts, use_graph=mode).float()
            st = e.decode_step_obj(seqs, max_len, greedy=True, use_graph=True)
            st.set_state(lg.argmax(-1), torch.tensor([s.length for s in seqs], device=cuda))
            toks = [st.step().clone() for _ in range(6)]
            res[mode] = (lg, torch.stack(toks).cpu())
        assert e._pf_graphs, "prefill graph not captured"
        torch.testing.assert_close(res[True][0], res[False][0], rtol=1e-3, atol=1e-3)
        assert torch.equal(res[True][1], res[False][1]), trial


def test_prefill_dense_shadow_matches_transient(cuda):
    """the resident dequantized prefill shadow (ops/gemm.py _dense_weight,
    auto-enabled by Engine on a >= 128 GiB device) gives the transient-dequant
    logits exactly, eager and graph-captured; entries die with their blob, and
    a new model whose blobs reuse freed addresses never sees stale weights"""
    import gc
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.models.cache import SequenceState
    from ipex_llm_amd.ops import gemm as G
    old = G._DENSE_BUDGET

    def run(seed, budget, mode):
        G.set_dense_budget(budget)
        m = random_native_model(_cfg(), "sym_int4", cuda, torch.bfloat16, seed=seed)
        e = Engine(m)
        G.set_dense_budget(budget)             # the engine's auto rule must not override the test's choice
        e._ensure_cache(2, 640)
        out = []
        for _ in range(2):                     # 2nd call: cache hit (eager) / graph replay
            e.cache.allocator = type(e.cache.allocator)(e.cache.num_blocks)
            seqs = [SequenceState(e.cache.allocator.alloc(10)) for _ in range(2)]
            ids = torch.randint(0, 1024, (2, 300), generator=torch.Generator().manual_seed(7))
            out.append(e.prefill_batch(seqs, ids, use_graph=mode).float().cpu())
        n_cached = len(G._dense_cache)
        del e, m
        gc.collect()
        return out, n_cached

    try:
        for mode in (False, True):
            ref, _ = run(1, 0.0, mode)
            got, n_cached = run(1, 1.0, mode)
            assert n_cached > 0
            for a, b in zip(ref, got):
                assert torch.equal(a, b)
            assert len(G._dense_cache) == 0        # dropped with the model
            other, _ = run(2, 1.0, mode)           # same shapes, other weights
            ref2, _ = run(2, 0.0, mode)
            assert all(torch.equal(a, b) for a, b in zip(other, ref2))
    finally:
        G.set_dense_budget(old / 2 ** 30)
