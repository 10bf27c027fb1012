"""Embedding variants (reference embedding.py), settings/env aliases,
BenchmarkWrapper timing, batched streamer."""
import torch


def _tiny(tmp_path):
    from transformers import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=192, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2)
    p = str(tmp_path / "m")
    LlamaForCausalLM(cfg).save_pretrained(p)
    return p


def test_embedding_variants_match(tmp_path):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from ipex_llm_amd.transformers.embedding import CPUEmbedding, DiskEmbedding, LowBitEmbedding
    p = _tiny(tmp_path)
    ids = torch.randint(0, 192, (2, 8))
    base = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    with torch.no_grad():
        ref = base(ids).logits
    # disk embeddings are fp16: the ~5e-4 input change moves some codes of the
    # CPU GEMM's per-token int8 activations by one step (csrc/cpu/gemm_q4.cpp)
    for kw, cls, tol in (({"cpu_embedding": True}, CPUEmbedding, 1e-5), ({"disk_embedding": True}, DiskEmbedding, 3e-2),
                         ({"embedding_qtype": "sym_int8"}, LowBitEmbedding, 5e-2)):
        m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32, **kw)
        assert isinstance(m.model.embed_tokens, cls)
        with torch.no_grad():
            out = m(ids).logits
        assert ((out - ref).norm() / ref.norm()).item() < tol, cls


def test_settings_env_aliases(monkeypatch):
    from ipex_llm_amd.utils.settings import get_settings
    monkeypatch.setenv("IPEX_LLM_QUANTIZE_KV_CACHE", "1")
    monkeypatch.setenv("BIGDL_LLM_LINEAR_THRESHOLD", "128")
    s = get_settings(refresh=True)
    assert s.quantize_kv_cache and s.linear_threshold == 128
    monkeypatch.delenv("IPEX_LLM_QUANTIZE_KV_CACHE")
    assert not get_settings(refresh=True).quantize_kv_cache


def test_benchmark_wrapper(tmp_path):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from ipex_llm_amd.utils import BenchmarkWrapper
    m = AutoModelForCausalLM.from_pretrained(_tiny(tmp_path), load_in_4bit=True, torch_dtype=torch.float32)
    bw = BenchmarkWrapper(m)
    out = bw.generate(torch.randint(0, 192, (1, 12)), max_new_tokens=6, min_new_tokens=6)
    assert out.shape == (1, 18) and bw.first_cost > 0 and bw.rest_cost_mean > 0


def test_batch_streamer():
    from ipex_llm_amd.transformers.streamer import BatchTextIteratorStreamer

    class Tok:
        def decode(self, ids, **kw):
            return " ".join(f"t{i}" for i in ids)

    s = BatchTextIteratorStreamer(Tok(), 2, skip_prompt=True)
    s.put(torch.tensor([[1, 2], [3, 4]]))      # prompt: skipped
    s.put(torch.tensor([5, 6]))
    s.put(torch.tensor([7, 8]))
    s.end()
    got = [x for x in s]
    assert "".join(g[0] for g in got).strip() == "t5 t7"
