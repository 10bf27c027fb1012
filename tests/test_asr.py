"""/v1/audio/transcriptions (serving/asr.py, reference
SRC/serving/fastapi/api_server.py:404-428 + model_worker.py:97-114).

A tiny random Whisper (the real checkpoints are not available offline) is
converted to low-bit linears; the transcriber's cached greedy decoder loop
must produce the same tokens as an uncached greedy loop over the full
decoder prefix, and the HTTP route must accept a multipart WAV upload (any
sample rate, stereo) and answer in the OpenAI formats."""
import io

import numpy as np
import pytest
import torch


class _Tok:
    special = {"<|startoftranscript|>": 50, "<|en|>": 51, "<|zh|>": 52, "<|transcribe|>": 53,
               "<|notimestamps|>": 54, "<|startofprev|>": 55}
    unk_token_id = 0
    eos_token_id = 49

    def convert_tokens_to_ids(self, t):
        return self.special.get(t, 0)

    def encode(self, text, add_special_tokens=False):
        return [1 + (ord(c) % 40) for c in text]

    def decode(self, ids, skip_special_tokens=True):
        return " ".join(f"t{i}" for i in ids if i < 49)


@pytest.fixture(scope="module")
def whisper():
    from transformers import WhisperConfig, WhisperFeatureExtractor, WhisperForConditionalGeneration
    torch.manual_seed(0)
    cfg = WhisperConfig(vocab_size=64, num_mel_bins=80, encoder_layers=1, decoder_layers=2, d_model=64,
                        encoder_attention_heads=2, decoder_attention_heads=2, encoder_ffn_dim=128,
                        decoder_ffn_dim=128, max_source_positions=1500, max_target_positions=64,
                        eos_token_id=49, pad_token_id=48, bos_token_id=50, decoder_start_token_id=50)
    m = WhisperForConditionalGeneration(cfg).eval()
    from ipex_llm_amd import optimize_model
    m = optimize_model(m, low_bit="sym_int8")
    return m, WhisperFeatureExtractor(feature_size=80)


def _wav(x, sr):
    from scipy.io import wavfile
    b = io.BytesIO()
    wavfile.write(b, sr, x)
    return b.getvalue()


def _naive(model, feats, prompt, n):
    ids = list(prompt)
    out = []
    with torch.no_grad():
        for _ in range(n):
            lg = model(input_features=feats, decoder_input_ids=torch.tensor([ids])).logits[0, -1]
            t = int(lg.float().argmax())
            if t == 49:
                break
            out.append(t)
            ids.append(t)
    return out


def test_transcriber_cached_loop_matches_uncached(whisper):
    from ipex_llm_amd.serving.asr import WhisperTranscriber
    from ipex_llm_amd.transformers.low_bit_linear import LowBitLinear
    model, fe = whisper
    assert any(isinstance(mod, LowBitLinear) for mod in model.modules())
    tr = WhisperTranscriber(model, fe, _Tok(), max_new_tokens=12)
    sr = 8000
    t = np.arange(sr) / sr
    audio = (0.3 * np.sin(2 * np.pi * 440 * t)).astype(np.float32)
    feats = tr.features(audio, sr)
    assert feats.shape == (1, 80, 3000)
    prompt = tr.prompt_ids("en")
    assert prompt == [50, 51, 53, 54]
    assert tr.generate_ids(feats, prompt) == _naive(model, feats, prompt, 12)
    with pytest.raises(ValueError):
        tr.prompt_ids("xx")


def test_transcription_route(whisper, tmp_path):
    from fastapi.testclient import TestClient
    from ipex_llm_amd.serving.api_server import build_app
    from ipex_llm_amd.serving.asr import WhisperTranscriber, decode_wav
    from ipex_llm_amd.serving.engine import LLMEngine
    from ipex_llm_amd.models.builder import random_native_model
    from transformers import LlamaConfig
    model, fe = whisper
    tr = WhisperTranscriber(model, fe, _Tok(), max_new_tokens=8)
    lm = random_native_model(LlamaConfig(vocab_size=64, hidden_size=64, intermediate_size=128, num_hidden_layers=1,
                                         num_attention_heads=2, num_key_value_heads=2), "sym_int8", "cpu",
                             torch.float32)
    eng = LLMEngine(lm, max_batch=2, max_model_len=64)
    rng = np.random.default_rng(0)
    stereo = (rng.standard_normal((22050, 2)) * 3000).astype(np.int16)        # 1 s, 22.05 kHz, PCM16 stereo
    wav = _wav(stereo, 22050)
    x, sr = decode_wav(wav)
    assert sr == 22050 and x.shape == (22050,) and np.abs(x).max() <= 1.0
    want = tr.transcribe(x, sr, "en")
    app = build_app(eng, _Tok(), "tiny", asr=tr)
    with TestClient(app) as c:
        r = c.post("/v1/audio/transcriptions", files={"file": ("a.wav", wav, "audio/wav")},
                   data={"model": "whisper", "language": "en"})
        assert r.status_code == 200, r.text
        assert r.json() == {"text": want}
        r = c.post("/v1/audio/transcriptions", files={"file": ("a.wav", wav, "audio/wav")},
                   data={"language": "en", "response_format": "text"})
        assert r.status_code == 200 and r.text == want
        r = c.post("/v1/audio/transcriptions", files={"file": ("a.wav", wav, "audio/wav")},
                   data={"language": "en", "response_format": "srt"})
        assert r.text.startswith("1\n00:00:00,000 --> 00:00:01,000\n")
        r = c.post("/v1/audio/transcriptions", data={"language": "en"})
        assert r.status_code == 400
        r = c.post("/v1/audio/transcriptions", files={"file": ("a.wav", wav, "audio/wav")},
                   data={"language": "klingon"})
        assert r.status_code == 400
    app2 = build_app(eng, _Tok(), "tiny")
    with TestClient(app2) as c:
        r = c.post("/v1/audio/transcriptions", files={"file": ("a.wav", wav, "audio/wav")})
        assert r.status_code == 501
