"""llama.cpp-python-style API (reference SRC/ggml/model/llama/llama.py):
tokenize/eval/sample/generate, completions (plain, streamed, stop strings,
prefix-state cache), chat, embeddings, state save/load -- on the native
decoder (llama) and on the HF-forward fallback (gpt2)."""
import pytest
import torch


def _tokenizer():
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers
    from transformers import PreTrainedTokenizerFast
    vocab = {"<unk>": 0, "<s>": 1, "</s>": 2}
    for i in range(3, 320):
        vocab[f"w{i}"] = i
    tk = Tokenizer(models.WordLevel(vocab, unk_token="<unk>"))
    tk.pre_tokenizer = pre_tokenizers.WhitespaceSplit()
    tk.decoder = decoders.WordPiece(prefix="##")
    return PreTrainedTokenizerFast(tokenizer_object=tk, unk_token="<unk>", bos_token="<s>", eos_token="</s>")


@pytest.fixture(scope="module")
def llama_dir(tmp_path_factory):
    from transformers import LlamaConfig, LlamaForCausalLM
    p = str(tmp_path_factory.mktemp("ggml") / "llama")
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=320, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512,
                      eos_token_id=2, bos_token_id=1)
    m = LlamaForCausalLM(cfg).eval()
    with torch.no_grad():
        for n, q in m.named_parameters():
            if q.dim() == 2:
                q.normal_(0, 0.2)
    m.save_pretrained(p)
    _tokenizer().save_pretrained(p)
    return p


def test_llama_api_native(llama_dir):
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.ggml import Llama, LlamaCache
    from ipex_llm_amd.transformers.hf_native import get_native
    llm = Llama(llama_dir, n_ctx=128, low_bit="sym_int8", device="cpu", seed=0)
    assert llm.ctx._eng is not None                       # native decoder path
    toks = llm.tokenize(b"w5 w6 w7 w8")
    assert llm.detokenize(toks) == b"w5 w6 w7 w8" and llm.token_bos() == 1
    ref = Engine(get_native(llm.model)[0]).generate([toks], max_new_tokens=8, use_graph=False)[0][len(toks):]
    ref = ref[:ref.index(2)] if 2 in ref else ref
    got = llm.generate(toks, max_new_tokens=8, temperature=0, repetition_penalty=1.0)
    assert got == ref
    # completions: plain == streamed; prefix reuse after a longer context
    r = llm("w5 w6 w7 w8", max_tokens=6, temperature=0, repeat_penalty=1.0)
    assert r["object"] == "text_completion" and r["usage"]["prompt_tokens"] == len(toks)
    s = "".join(c["choices"][0]["text"] for c in llm("w5 w6 w7 w8", max_tokens=6, temperature=0,
                                                       repeat_penalty=1.0, stream=True))
    assert s == r["choices"][0]["text"]
    # stop string cuts the text
    words = r["choices"][0]["text"].split()
    if len(words) >= 2:
        r2 = llm("w5 w6 w7 w8", max_tokens=6, temperature=0, repeat_penalty=1.0, stop=[words[1]])
        assert words[1] not in r2["choices"][0]["text"] and r2["choices"][0]["finish_reason"] == "stop"
    # state save / load reproduces the continuation; the cache restores a prefix
    llm.reset()
    llm.eval(toks)
    st = llm.save_state()
    a = llm.sample(temp=0, repeat_penalty=1.0)
    llm.eval([5, 9, 11])
    llm.load_state(st)
    assert llm.sample(temp=0, repeat_penalty=1.0) == a
    llm.set_cache(LlamaCache())
    c1 = llm("w5 w6 w7 w8", max_tokens=4, temperature=0, repeat_penalty=1.0)
    llm.reset()
    c2 = llm("w5 w6 w7 w8", max_tokens=4, temperature=0, repeat_penalty=1.0)
    assert c1["choices"][0]["text"] == c2["choices"][0]["text"]
    # chat + embeddings
    ch = llm.create_chat_completion([{"role": "user", "content": "w9 w10"}], max_tokens=3, temperature=0)
    assert ch["choices"][0]["message"]["role"] == "assistant"
    e = llm.create_embedding(["w5 w6", "w7"])
    assert len(e["data"]) == 2 and len(e["data"][0]["embedding"]) == llm.n_embd()
    assert llm.n_vocab() == 320 and llm.n_ctx() == 128


@pytest.mark.parametrize("native", [False, True])
def test_llama_api_hf_fallback(tmp_path, native):
    """gpt2 runs on the native generic decoder; a variant it does not cover
    (scale_attn_by_inverse_layer_idx) keeps the HF forward + its KV cache"""
    from transformers import GPT2Config, GPT2LMHeadModel
    from ipex_llm_amd.ggml import AutoModelForCausalLM as GgmlAuto
    p = str(tmp_path / "gpt2")
    torch.manual_seed(0)
    GPT2LMHeadModel(GPT2Config(n_embd=64, n_layer=2, n_head=4, vocab_size=320, n_positions=128,
                               eos_token_id=2, bos_token_id=1,
                               scale_attn_by_inverse_layer_idx=not native)).save_pretrained(p)
    _tokenizer().save_pretrained(p)
    llm = GgmlAuto.from_pretrained(p, model_family="starcoder", n_ctx=64, low_bit="sym_int8", device="cpu")
    assert (llm.ctx._eng is not None) == native
    toks = llm.tokenize("w5 w6 w7")
    with torch.no_grad():
        hf = llm.model.generate(torch.tensor([toks]), max_new_tokens=6, do_sample=False, eos_token_id=None,
                                pad_token_id=0)
    got = llm.generate(toks, max_new_tokens=6, temperature=0, repetition_penalty=1.0)
    want = hf[0, len(toks):].tolist()
    assert got == want[:len(got)] and (len(got) == 6 or want[len(got)] == 2)
    # prefix reuse through the HF cache (crop) gives the same continuation
    again = llm.generate(toks, max_new_tokens=6, temperature=0, repetition_penalty=1.0)
    assert again == got


def test_langchain_native_llm_and_embeddings(llama_dir):
    """reference langchain/llms/bigdlllm.py + embeddings/bigdlllm.py over the
    native Llama: _call streams the completion chunks and concatenates them
    (== the client's own completion), get_num_tokens tokenizes with the client,
    the family classes pick their ggml class, embeddings are client.embed"""
    from ipex_llm_amd.langchain import BigdlNativeLLM, LlamaEmbeddings, LlamaLLM, BigdlNativeEmbeddings
    llm = LlamaLLM(llama_dir, n_ctx=128, low_bit="sym_int8", seed=0, temperature=0.0, max_tokens=6,
                   repeat_penalty=1.0)
    assert type(llm.client).__name__ == "Llama" and llm._llm_type == "BigDL"
    text = llm.invoke("w5 w6 w7")
    ref = llm.client(prompt="w5 w6 w7", max_tokens=6, temperature=0.0, repeat_penalty=1.0, top_k=40,
                     top_p=0.95)["choices"][0]["text"]
    assert text == ref and len(text) > 0
    chunks = list(llm.stream("w5 w6 w7"))
    assert "".join(c["choices"][0]["text"] for c in chunks) == ref
    assert llm.get_num_tokens("w5 w6 w7") == len(llm.client.tokenize(b"w5 w6 w7"))
    with pytest.raises(ValueError):
        BigdlNativeLLM(llama_dir, model_family="nosuch")
    llm.stop = ["w9"]
    with pytest.raises(ValueError):
        llm._get_parameters(["x"])
    emb = LlamaEmbeddings(llama_dir, low_bit="sym_int8", n_ctx=128)
    q = emb.embed_query("w5 w6")
    assert q == llm.client.embed("w5 w6") and len(q) == 128
    assert emb.embed_documents(["w5 w6", "w7"])[0] == q
    assert BigdlNativeEmbeddings(client=emb.client).embed_query("w5 w6") == q


def test_langchain_vllm_wrapper_batches_on_engine(llama_dir):
    """reference langchain/vllm/vllm.py VLLM: prompts through the continuous-
    batching engine, greedy == the engine's own generate"""
    from transformers import AutoTokenizer
    from ipex_llm_amd.langchain import VLLM
    from ipex_llm_amd.serving.engine import LLMEngine, SamplingParams
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from ipex_llm_amd.transformers.hf_native import get_native
    hf = AutoModelForCausalLM.from_pretrained(llama_dir, load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    tok = AutoTokenizer.from_pretrained(llama_dir)
    eng = LLMEngine(get_native(hf)[0], max_batch=4)
    llm = VLLM(client=eng, tokenizer=tok, temperature=0.0, max_new_tokens=5, ignore_eos=True)
    outs = llm.generate_texts(["w5 w6 w7", "w9 w10"])
    ids = [tok.encode("w5 w6 w7"), tok.encode("w9 w10")]
    ref = eng.generate(ids, SamplingParams(max_new_tokens=5))
    assert outs == [tok.decode(r, skip_special_tokens=True) for r in ref]
    assert llm.invoke("w5 w6 w7") == outs[0]
