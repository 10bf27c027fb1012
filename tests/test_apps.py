"""App-level components: CLI, loader, llm_patch, JSON-constrained decoding
(xgrammar equivalent), LangChain / LlamaIndex wrappers (reference test
strategy: langchain/llamaindex integration tests, CLI smoke)."""
import json
import string

import pytest
import torch


def _char_tokenizer():
    from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers
    from transformers import PreTrainedTokenizerFast
    chars = ["<unk>", "<s>", "</s>"] + list(string.ascii_lowercase + string.digits + "{}[]\":, .-")
    tk = Tokenizer(models.WordLevel({c: i for i, c in enumerate(chars)}, unk_token="<unk>"))
    tk.pre_tokenizer = pre_tokenizers.Split(Regex("."), behavior="isolated")
    tk.decoder = decoders.Fuse()
    return PreTrainedTokenizerFast(tokenizer_object=tk, unk_token="<unk>", bos_token="<s>", eos_token="</s>")


@pytest.fixture(scope="module")
def tiny(tmp_path_factory):
    from transformers import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(0)
    tok = _char_tokenizer()
    cfg = LlamaConfig(vocab_size=len(tok), hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, eos_token_id=2, bos_token_id=1)
    p = str(tmp_path_factory.mktemp("m") / "tiny")
    LlamaForCausalLM(cfg).save_pretrained(p)
    tok.save_pretrained(p)
    return p, tok


def test_cli_generate_and_env_check(tiny, capsys):
    from ipex_llm_amd.cli.main import main
    p, _ = tiny
    main(["generate", "-m", p, "--device", "cpu", "-p", "ab1", "-n", "5", "--low-bit", "sym_int8"])
    info = main(["env-check"])
    assert "torch" in info and "native_extension" in info


def test_loader(tiny):
    from ipex_llm_amd.transformers.loader import load_model, try_run_test_generation
    p, _ = tiny
    m, tok = load_model(p, device="cpu", low_bit="sym_int4")
    assert getattr(m, "_illm_native_attached", False)
    assert try_run_test_generation("", p, "cpu", "sym_int4") == "success"


def test_llm_patch():
    import transformers
    from ipex_llm_amd import llm_patching
    from ipex_llm_amd.transformers import AutoModelForCausalLM as Ours
    orig = transformers.AutoModelForCausalLM
    llm_patching.llm_patch(train=True)
    try:
        assert transformers.AutoModelForCausalLM is Ours
        from ipex_llm_amd.training.args import TrainingArguments
        assert transformers.TrainingArguments is TrainingArguments
    finally:
        llm_patching.llm_unpatch()
    assert transformers.AutoModelForCausalLM is orig


def test_json_constrained_generation(tiny):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from ipex_llm_amd.transformers.xgrammar import _JsonState, create_json_logits_processor
    st = _JsonState()
    assert all(st.feed(c) for c in '{"a": [1, 2.5, "x"], "b": {"c": null}}') and st.done
    assert not _JsonState().feed("}")
    p, tok = tiny
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    proc = create_json_logits_processor(tok, len(tok), schema={"type": "object"})
    ids = tok("ab", return_tensors="pt").input_ids
    out = m.generate(ids, max_new_tokens=24, logits_processor=[proc])
    text = tok.decode(out[0][ids.shape[1]:], skip_special_tokens=True)
    chk = _JsonState("object")
    assert text.startswith("{") and all(chk.feed(c) for c in text), text


def test_langchain_and_llamaindex_wrappers(tiny):
    from ipex_llm_amd.langchain import TransformersEmbeddings, TransformersLLM
    from ipex_llm_amd.llamaindex import IpexLLM
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    p, tok = tiny
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    llm = TransformersLLM(model=m, tokenizer=tok, generate_kwargs={"max_new_tokens": 6})
    out = llm.invoke("abc")
    assert isinstance(out, str)
    assert "".join(llm.stream("abc", max_new_tokens=4)) is not None
    li = IpexLLM(m, tok, max_new_tokens=5)
    assert isinstance(li.complete("ab").text, str)
    assert li.chat([{"role": "user", "content": "hi"}]).text is not None
    from transformers import LlamaModel
    enc = LlamaModel.from_pretrained(p)
    emb = TransformersEmbeddings(enc, tok, normalize=True)
    v = emb.embed_documents(["abc", "xyz"])
    assert len(v) == 2 and abs(sum(x * x for x in v[0]) - 1.0) < 1e-4
