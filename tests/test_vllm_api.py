"""vLLM-style surface on the native engine (reference SRC/vllm/xpu/engine/
engine.py IPEXLLMClass / IPEXLLMLLMEngine / IPEXLLMAsyncLLMEngine and the
OpenAI entry point): same greedy tokens as the serving engine, request
lifecycle, async streaming, the vLLM command line and the served routes.
vLLM itself is not importable here: parity with it is unpinned."""
import asyncio

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
    p = str(tmp_path_factory.mktemp("vllm") / "llama")
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


@pytest.fixture(scope="module")
def llm(llama_dir):
    from ipex_llm_amd.vllm import IPEXLLMClass
    return IPEXLLMClass(model=llama_dir, load_in_low_bit="sym_int4", device="cpu", max_model_len=256,
                        max_num_seqs=8, enforce_eager=True)


def test_offline_generate_matches_serving_engine(llm):
    from ipex_llm_amd.serving.engine import SamplingParams as NSP
    from ipex_llm_amd.vllm import RequestOutput, SamplingParams
    prompts = ["w5 w6 w7", "w10 w11 w12 w13 w14", "w100"]
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    outs = llm.generate(prompts, sp)
    assert len(outs) == 3 and all(isinstance(o, RequestOutput) and o.finished for o in outs)
    tok = llm.get_tokenizer()
    ids = [tok(p)["input_ids"] for p in prompts]
    ref = llm.llm_engine.engine.generate(ids, NSP(max_new_tokens=6, ignore_eos=True))
    for o, r, i in zip(outs, ref, ids):
        assert o.outputs[0].token_ids == r and o.prompt_token_ids == i
        assert o.outputs[0].finish_reason == "length" and len(r) == 6
        assert o.outputs[0].text == tok.decode(r, skip_special_tokens=True)
    # token-id prompts, per-request sampling params
    outs2 = llm.generate(prompt_token_ids=ids, sampling_params=[sp, SamplingParams(max_tokens=2, temperature=0.0,
                                                                                  ignore_eos=True), sp])
    assert outs2[0].outputs[0].token_ids == ref[0] and outs2[1].outputs[0].token_ids == ref[1][:2]
    with pytest.raises(ValueError):
        llm.generate(["w5"], SamplingParams(n=2))


def test_engine_step_loop_and_abort(llm):
    from ipex_llm_amd.vllm import SamplingParams
    eng = llm.llm_engine
    eng.add_request("a", "w5 w6", SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True))
    eng.add_request("b", None, SamplingParams(max_tokens=50, temperature=0.0, ignore_eos=True),
                    prompt_token_ids=[1, 7, 8])
    seen, steps = {}, 0
    while eng.has_unfinished_requests() and steps < 200:
        for o in eng.step():
            seen[o.request_id] = o
        if "a" in seen and seen["a"].finished:
            eng.abort_request("b")
        steps += 1
    assert seen["a"].finished and len(seen["a"].outputs[0].token_ids) == 4
    assert not seen["b"].finished and len(seen["b"].outputs[0].token_ids) < 50     # aborted mid-way
    assert not eng.has_unfinished_requests() and eng.step() == []


def test_async_engine_streams(llama_dir, llm):
    from ipex_llm_amd.vllm import IPEXLLMAsyncLLMEngine, SamplingParams
    eng = IPEXLLMAsyncLLMEngine(llm.llm_engine)
    sp = SamplingParams(max_tokens=5, temperature=0.0, ignore_eos=True)

    async def run():
        outs = []
        async for o in eng.generate("w5 w6 w7", sp, "r1"):
            outs.append(o)
        return outs

    try:
        outs = asyncio.run(run())
    finally:
        eng.shutdown()
    assert outs[-1].finished and len(outs[-1].outputs[0].token_ids) == 5
    lens = [len(o.outputs[0].token_ids) for o in outs]
    assert lens == sorted(lens)
    ref = llm.generate(["w5 w6 w7"], sp)[0].outputs[0].token_ids
    assert outs[-1].outputs[0].token_ids == ref


def test_openai_entrypoint_cli_and_routes(llama_dir):
    from fastapi.testclient import TestClient
    from ipex_llm_amd.vllm.entrypoints.openai.api_server import build_app_from_args
    from ipex_llm_amd.vllm.entrypoints.openai.cli_args import make_arg_parser, unsupported
    args = make_arg_parser().parse_args(["--model", llama_dir, "--load-in-low-bit", "sym_int4", "--device", "cpu",
                                         "--max-model-len", "256", "--max-num-seqs", "4", "--enforce-eager",
                                         "--served-model-name", "tiny", "--api-key", "k1", "--swap-space", "4",
                                         "--disable-log-requests"])
    assert unsupported(args) == ["--swap-space", "--disable-log-requests"]
    app, _ = build_app_from_args(args)
    with TestClient(app) as c:
        assert c.get("/v1/models").status_code == 401
        h = {"Authorization": "Bearer k1"}
        ms = c.get("/v1/models", headers=h).json()
        assert ms["data"][0]["id"] == "tiny"
        r = c.post("/v1/completions", headers=h, json={"model": "tiny", "prompt": "w5 w6 w7", "max_tokens": 4})
        assert r.status_code == 200 and r.json()["usage"]["completion_tokens"] >= 1
    with pytest.raises(ValueError):
        build_app_from_args(make_arg_parser().parse_args(["--model", llama_dir, "--device", "cpu", "-tp", "2"]))
