"""Serving: C++ continuous-batching scheduler, LLMEngine (batched decode,
preemption/recompute) vs the static engine, and the OpenAI/TGI HTTP API
(reference: serving/fastapi/api_server.py, openai_protocol.py)."""
import json

import pytest
import torch


@pytest.fixture(scope="module")
def native():
    from transformers import LlamaConfig
    from ipex_llm_amd.models.builder import random_native_model
    cfg = LlamaConfig(vocab_size=128, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=1024)
    return random_native_model(cfg, "fp8_e4m3", "cpu", torch.float32, seed=0, std=0.2)


def _sched(nb=4, bs=64, mb=8, mp=4096):
    import ipex_llm_amd.ops as ops
    ops.require()
    return torch.classes.ipex_llm_amd.Scheduler(nb, bs, mb, mp)


def _split(plan):
    i1 = plan.index(-1); i2 = plan.index(-1, i1 + 1); i3 = plan.index(-1, i2 + 1)
    return plan[:i1], plan[i1 + 1:i2], plan[i2 + 1:i3], plan[i3 + 1:]


def test_scheduler_admission_preemption_failure():
    s = _sched(nb=4, bs=64)
    s.add(1, 100)          # 2 blocks (room for 101 tokens)
    s.add(2, 60)           # 1 block
    s.add(3, 300)          # can never fit in 4 blocks -> failed, queue continues
    s.add(4, 63)           # 1 block
    p, d, pre, f = _split(list(s.schedule()))
    assert p == [1, 2, 4] and d == [] and f == [3] and s.num_free_blocks() == 0
    for rid, n in ((1, 100), (2, 60), (4, 63)):
        s.advance(rid, n); s.grow(rid)
    p, d, pre, f = _split(list(s.schedule()))
    assert d == [1, 2, 4] and pre == [] and p == []
    for rid in (1, 2, 4):
        s.advance(rid, 1); s.grow(rid)
    # request 4 now needs a second block, the pool is empty: preempt the latest admitted (4)
    p, d, pre, f = _split(list(s.schedule()))
    assert pre == [4] and d == [1, 2]
    assert s.state(4) == 0 and s.context(4) == 65 and s.cached(4) == 0
    s.finish(1)
    p, d, pre, f = _split(list(s.schedule()))
    assert p == [4] and d == [2]


def test_engine_matches_static_generate(native):
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.serving.engine import LLMEngine, SamplingParams
    prompts = [[1, 2, 3, 4, 5], [9, 8, 7], list(range(10, 40))]
    ref = Engine(native).generate(prompts, max_new_tokens=12, use_graph=False)
    eng = LLMEngine(native, max_batch=8, max_model_len=256)
    out = eng.generate(prompts, SamplingParams(max_new_tokens=12))
    assert [p + o for p, o in zip(prompts, out)] == ref


def test_engine_preemption_recompute(native):
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.serving.engine import LLMEngine, SamplingParams
    prompts = [list(range(1, 60)), list(range(3, 62)), list(range(5, 64))]
    ref = Engine(native).generate(prompts, max_new_tokens=10, use_graph=False)
    # 4 blocks of 64: three 60-token prompts fit, but growing past 64 forces preemption
    eng = LLMEngine(native, max_batch=8, max_model_len=256, num_blocks=4)
    out = eng.generate(prompts, SamplingParams(max_new_tokens=10))
    assert eng.stats["preemptions"] > 0
    assert [p + o for p, o in zip(prompts, out)] == ref


def test_scheduler_prefix_cache_reuse_and_eviction():
    s = _sched(nb=6, bs=64)
    s.enable_prefix_caching(True)
    pa = list(range(1, 150))                    # 149 tokens: 2 full blocks + 21
    s.add_tokens(1, pa)
    p, d, pre, f = _split(list(s.schedule()))
    assert p == [1] and s.cached(1) == 0
    s.advance(1, len(pa))
    assert s.num_cached_blocks() == 2           # the two full blocks are indexed
    # same 128-token prefix, different tail: reuses both full blocks
    s.add_tokens(2, pa[:128] + [7, 8, 9])
    p, d, pre, f = _split(list(s.schedule()))
    assert p == [2] and s.cached(2) == 128
    assert list(s.blocks(2))[:2] == list(s.blocks(1))[:2]
    assert s.prefix_hit_tokens() == 128
    # a prompt that IS exactly the 2 cached blocks recomputes its last token
    s.add_tokens(3, pa[:128])
    p, d, pre, f = _split(list(s.schedule()))
    assert p == [3] and s.cached(3) == 64
    # finishing keeps content: blocks become idle-but-cached (counted as free)
    for r in (1, 2, 3):
        s.finish(r)
    assert s.num_free_blocks() == 6 and s.num_cached_blocks() == 2
    s.add_tokens(4, pa[:64] + [1] * 70)          # hits block 0 after all holders left
    p, d, pre, f = _split(list(s.schedule()))
    assert p == [4] and s.cached(4) == 64
    s.finish(4)
    # a request needing every block evicts the idle cached ones
    s.add_tokens(5, [3] * 380)
    p, d, pre, f = _split(list(s.schedule()))
    assert p == [5] and s.cached(5) == 0 and s.num_free_blocks() == 0
    s.advance(5, 380)
    assert s.num_cached_blocks() == 5


def test_scheduler_evicts_idle_cached_before_preempting():
    """free list empty but idle cached blocks available: a running sequence
    crossing a block boundary takes an evicted block, nobody is preempted"""
    s = _sched(nb=4, bs=64)
    s.enable_prefix_caching(True)
    s.add_tokens(1, list(range(1, 129)))        # 2 full blocks -> cached after finish
    _split(list(s.schedule()))
    s.advance(1, 128)
    s.finish(1)
    assert s.num_cached_blocks() == 2 and s.num_free_blocks() == 4
    s.add_tokens(2, [7] * 64)                   # 1 fresh block + 1 for the next token later
    s.add_tokens(3, [9] * 63)
    p, d, pre, f = _split(list(s.schedule()))
    assert p == [2, 3]
    s.advance(2, 64); s.grow(2)
    s.advance(3, 63); s.grow(3)
    # request 2 needs a 2nd block: the free list holds 0 or 1 blocks, the rest are idle cached
    for _ in range(3):
        p, d, pre, f = _split(list(s.schedule()))
        assert pre == [], "preempted although idle cached blocks were available"
        for r in d:
            s.advance(r, 1); s.grow(r)


def test_engine_prefix_cache_matches_uncached(native):
    """shared system prompt: later requests prefill only their suffix and
    produce the tokens of the uncached engine"""
    from ipex_llm_amd.serving.engine import LLMEngine, SamplingParams
    sys_p = [3 + (i * 7) % 120 for i in range(130)]
    prompts = [sys_p + [5, 6, 7], sys_p + [9], sys_p + list(range(40, 70)), sys_p[:64] + [1, 2]]
    ref = LLMEngine(native, max_batch=8, max_model_len=512, enable_prefix_caching=False)
    want = [ref.generate([p], SamplingParams(max_new_tokens=8))[0] for p in prompts]
    eng = LLMEngine(native, max_batch=8, max_model_len=512)
    got = [eng.generate([p], SamplingParams(max_new_tokens=8))[0] for p in prompts]
    assert got == want
    # requests 2..4 reuse 128, 128 and 64 cached prompt tokens
    assert eng.stats["prefix_hit_tokens"] == 128 + 128 + 64
    # a multi-turn continuation reuses the blocks of the previous turn's answer too
    turn2 = prompts[2] + got[2] + [11, 12]
    again = eng.generate([turn2], SamplingParams(max_new_tokens=4))[0]
    assert again == ref.generate([turn2], SamplingParams(max_new_tokens=4))[0]
    assert eng.stats["prefix_hit_tokens"] >= 128 + 128 + 64 + 128


def _tokenizer():
    from tokenizers import Tokenizer, models, pre_tokenizers
    from transformers import PreTrainedTokenizerFast
    vocab = {"<unk>": 0, "<s>": 1, "</s>": 2}
    for i in range(3, 128):
        vocab[f"w{i}"] = i
    tk = Tokenizer(models.WordLevel(vocab, unk_token="<unk>"))
    tk.pre_tokenizer = pre_tokenizers.WhitespaceSplit()
    from tokenizers import decoders
    tk.decoder = decoders.WordPiece(prefix="##")
    return PreTrainedTokenizerFast(tokenizer_object=tk, unk_token="<unk>", bos_token="<s>", eos_token="</s>")


def test_http_api(native):
    from fastapi.testclient import TestClient
    from ipex_llm_amd.serving.api_server import build_app
    from ipex_llm_amd.serving.engine import LLMEngine
    tok = _tokenizer()
    eng = LLMEngine(native, max_batch=4, max_model_len=256, eos_token_id=None)
    app = build_app(eng, tok, "tiny")
    with TestClient(app) as c:
        assert c.get("/health").json()["status"] == "ok"
        assert c.get("/v1/models").json()["data"][0]["id"] == "tiny"
        r = c.post("/v1/completions", json={"prompt": "w5 w6 w7", "max_tokens": 5}).json()
        assert r["object"] == "text_completion" and r["usage"]["completion_tokens"] == 5
        assert len(r["choices"][0]["text"].split()) >= 1
        r2 = c.post("/v1/chat/completions", json={"messages": [{"role": "user", "content": "w9 w10"}],
                                                   "max_tokens": 4}).json()
        assert r2["choices"][0]["message"]["role"] == "assistant"
        with c.stream("POST", "/v1/chat/completions", json={"messages": "w9 w10", "max_tokens": 4,
                                                              "stream": True}) as s:
            lines = [l for l in s.iter_lines() if l]
        assert lines[-1] == "data: [DONE]"
        chunks = [json.loads(l[6:]) for l in lines[:-1]]
        assert chunks[-1]["choices"][0]["finish_reason"] == "length"
        g = c.post("/generate", json={"inputs": "w5 w6 w7", "parameters": {"max_new_tokens": 5}}).json()
        assert g[1] == r["choices"][0]["text"]      # same greedy continuation
        with c.stream("POST", "/generate_stream", json={"inputs": "w5 w6 w7",
                                                         "parameters": {"max_new_tokens": 3}}) as s:
            ev = [json.loads(l[6:]) for l in s.iter_lines() if l]
        assert ev[-1]["details"]["generated_tokens"] == 3
        # Prometheus metrics: request / token counters, TTFT + TPOT histograms, KV usage
        import time as _time
        for _ in range(40):    # the last streamed request's counters land just after its final event
            m = c.get("/metrics").text
            gen = [l for l in m.splitlines() if l.startswith("ipex_llm_generation_tokens_total")]
            if gen and float(gen[0].split()[-1]) >= 5 + 4 + 4 + 5 + 3:
                break
            _time.sleep(0.05)
        assert "ipex_llm_requests_total" in m and "ipex_llm_time_to_first_token_seconds_bucket" in m
        assert gen and float(gen[0].split()[-1]) >= 5 + 4 + 4 + 5 + 3
        assert "ipex_llm_kv_cache_usage_ratio" in m and "ipex_llm_time_per_output_token_seconds_count" in m


@pytest.mark.gpu
def test_engine_graph_decode_matches_eager_on_gpu(cuda):
    """hipGraph-captured continuous-batching decode (padded batch buckets,
    scratch block) == the eager decode path, with requests joining / finishing
    at different steps"""
    from transformers import LlamaConfig
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.serving.engine import LLMEngine, SamplingParams
    cfg = LlamaConfig(vocab_size=512, hidden_size=512, intermediate_size=1024, num_hidden_layers=2,
                      num_attention_heads=8, num_key_value_heads=2, max_position_embeddings=2048)
    m = random_native_model(cfg, "sym_int4", cuda, torch.bfloat16, seed=3, std=0.2)
    prompts = [list(range(1, 70)), [5, 6, 7], list(range(100, 230)), list(range(9, 20))]
    lens = [20, 33, 7, 64]
    outs = {}
    for graph in (False, True):
        eng = LLMEngine(m, max_batch=8, max_model_len=512, use_graph=graph)
        rids = [eng.add_request(p, SamplingParams(max_new_tokens=n)) for p, n in zip(prompts, lens)]
        while eng.has_work():
            eng.step()
        outs[graph] = [eng.requests[r].generated for r in rids]
        assert (len(eng._graphs) > 0) == graph
    a, b = sum(outs[False], []), sum(outs[True], [])
    assert [len(x) for x in outs[True]] == lens
    assert sum(x == y for x, y in zip(a, b)) >= 0.97 * len(a)


@pytest.mark.gpu
def test_engine_prefix_cache_on_gpu(cuda, monkeypatch):
    """prefix-cached suffix prefill (HIP chunked-prefill attention over cached
    blocks) + graph decode gives the uncached engine's tokens.  The prefills
    run the fused GEMM (each row's dot products are independent of M); the
    library GEMM picks M-dependent kernels, so a 46-row suffix and a 302-row
    prompt round differently and a random model's near-tied logits can split."""
    import ipex_llm_amd.ops.gemm as G
    monkeypatch.setattr(G, "_USE_FUSED", True)
    monkeypatch.setattr(G, "_USE_LIB", False)
    from transformers import LlamaConfig
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.serving.engine import LLMEngine, SamplingParams
    cfg = LlamaConfig(vocab_size=1024, hidden_size=512, intermediate_size=1024, num_hidden_layers=2,
                      num_attention_heads=8, num_key_value_heads=2, max_position_embeddings=2048)
    m = random_native_model(cfg, "sym_int4", cuda, torch.bfloat16, seed=11)
    table = [(i * 37) % 1000 + 3 for i in range(300)]
    prompts = [table + [5, 6, 7], table + [9, 10], table[:200] + [4]]
    ref = LLMEngine(m, max_batch=4, max_model_len=512, enable_prefix_caching=False)
    want = [ref.generate([p], SamplingParams(max_new_tokens=8))[0] for p in prompts]
    eng = LLMEngine(m, max_batch=4, max_model_len=512)
    got = [eng.generate([p], SamplingParams(max_new_tokens=8))[0] for p in prompts]
    assert got == want
    assert eng.stats["prefix_hit_tokens"] == 256 + 192
