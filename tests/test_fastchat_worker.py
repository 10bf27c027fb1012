"""FastChat-protocol worker (reference serving/fastchat/ipex_llm_worker.py):
NUL-delimited streaming, stop strings, status/count/conv/details endpoints,
embeddings and controller registration + heartbeat (requests mocked)."""
import json

import pytest
import torch


@pytest.fixture(scope="module")
def native():
    from transformers import LlamaConfig
    from ipex_llm_amd.models.builder import random_native_model
    cfg = LlamaConfig(vocab_size=128, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=1024)
    return random_native_model(cfg, "sym_int8", "cpu", torch.float32, seed=0, std=0.2)


def _tokenizer():
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers
    from transformers import PreTrainedTokenizerFast
    vocab = {"<unk>": 0, "<s>": 1, "</s>": 2}
    for i in range(3, 128):
        vocab[f"w{i}"] = i
    tk = Tokenizer(models.WordLevel(vocab, unk_token="<unk>"))
    tk.pre_tokenizer = pre_tokenizers.WhitespaceSplit()
    tk.decoder = decoders.WordPiece(prefix="##")
    return PreTrainedTokenizerFast(tokenizer_object=tk, unk_token="<unk>", bos_token="<s>", eos_token="</s>")


def test_fastchat_worker_endpoints(native):
    from fastapi.testclient import TestClient
    from ipex_llm_amd.serving.engine import LLMEngine
    from ipex_llm_amd.serving.fastchat_worker import IPEXLLMWorker, build_worker_app, is_partial_stop
    tok = _tokenizer()
    eng = LLMEngine(native, max_batch=4, max_model_len=256)
    w = IPEXLLMWorker(eng, tok, ["tiny"], conv_template="vicuna_v1.1", stream_interval=1)
    with TestClient(build_worker_app(w)) as c:
        assert c.post("/worker_get_status").json()["model_names"] == ["tiny"]
        assert c.post("/count_token", json={"prompt": "w5 w6 w7"}).json()["count"] == 3
        assert c.post("/worker_get_conv_template").json()["conv"] == "vicuna_v1.1"
        assert c.post("/model_details").json()["context_length"] == 256
        g = c.post("/worker_generate", json={"prompt": "w5 w6 w7", "max_new_tokens": 5, "temperature": 0,
                                             "echo": False}).json()
        assert g["error_code"] == 0 and g["usage"]["completion_tokens"] == 5 and g["finish_reason"] == "length"
        with c.stream("POST", "/worker_generate_stream",
                      json={"prompt": "w5 w6 w7", "max_new_tokens": 5, "temperature": 0, "echo": False}) as s:
            body = b"".join(s.iter_bytes())
        chunks = [json.loads(x) for x in body.split(b"\0") if x]
        assert len(chunks) >= 2 and chunks[-1]["text"] == g["text"]
        assert all(chunks[i]["text"] == chunks[-1]["text"][:len(chunks[i]["text"])] for i in range(len(chunks)))
        words = g["text"].split()
        if len(words) >= 3:
            st = c.post("/worker_generate", json={"prompt": "w5 w6 w7", "max_new_tokens": 5, "temperature": 0,
                                                  "echo": False, "stop": words[2]}).json()
            assert words[2] not in st["text"] and st["finish_reason"] == "stop"
        e = c.post("/worker_get_embeddings", json={"input": ["w5 w6", "w9"]}).json()
        assert len(e["embedding"]) == 2 and e["token_num"] == 3
        assert abs(sum(v * v for v in e["embedding"][0]) - 1.0) < 1e-4
        big = c.post("/worker_generate", json={"prompt": " ".join(["w5"] * 300), "max_new_tokens": 4}).json()
        assert big["error_code"] != 0
    assert is_partial_stop("abc</", "</s>") and not is_partial_stop("abc", "</s>")
    assert not eng.has_work()


def test_fastchat_worker_controller(native, monkeypatch):
    import requests
    from ipex_llm_amd.serving.engine import LLMEngine
    from ipex_llm_amd.serving.fastchat_worker import IPEXLLMWorker
    calls = []

    class R:
        def __init__(self, d):
            self.d = d

        def json(self):
            return self.d

        def raise_for_status(self):
            pass

    def post(url, json=None, timeout=None):
        calls.append((url, json))
        return R({"exist": False})

    monkeypatch.setattr(requests, "post", post)
    eng = LLMEngine(native, max_batch=2, max_model_len=128)
    w = IPEXLLMWorker(eng, _tokenizer(), ["tiny"], "http://ctl", "http://me", no_register=False)
    w._stop_hb.set()
    assert calls[0][0] == "http://ctl/register_worker" and calls[0][1]["worker_name"] == "http://me"
    w.send_heart_beat()                     # controller forgot us -> re-register
    assert [u for u, _ in calls] == ["http://ctl/register_worker", "http://ctl/receive_heart_beat",
                                     "http://ctl/register_worker"]
