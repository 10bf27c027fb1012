"""Speech transcription for the OpenAI-compatible server
(``POST /v1/audio/transcriptions``).

Reference: ``SRC/serving/fastapi/api_server.py:404-428`` (the route: an
uploaded audio file plus ``model`` / ``language`` / ``response_format`` form
fields, answered with ``{"text": ...}``) and
``SRC/serving/fastapi/model_worker.py:97-114`` (load the audio at the
feature extractor's sampling rate, log-mel features, ``generate`` with the
language / transcribe forced decoder prompt).

Here:
  * the multipart body is parsed with the standard library (``email``), so
    the route needs no ``python-multipart``; the upload is decoded in memory
    (WAV: PCM 8/16/24/32-bit or IEEE float, any channel count -- mono mix)
    and resampled to the extractor's rate with a polyphase filter
    (``scipy.signal.resample_poly``) instead of writing it to ``./filename``
    and calling librosa;
  * :class:`WhisperTranscriber` runs the encoder once and a greedy cached
    decoder loop (``<|startoftranscript|><|lang|><|transcribe|>
    <|notimestamps|>`` prompt, stop at EOS / ``max_new_tokens``) on the
    model as loaded -- low-bit linears when it came through
    ``AutoModelForSpeechSeq2Seq.from_pretrained(..., load_in_low_bit=...)``.
    Requests run one at a time on a worker thread (the reference's worker
    serves one ASR request per step as well).
"""
from __future__ import annotations

import io
import math
import threading
from email.parser import BytesParser
from email.policy import HTTP
from typing import Dict, List, Optional, Tuple, Union

import numpy as np
import torch

FormValue = Union[str, Tuple[str, bytes]]


def parse_multipart(body: bytes, content_type: str) -> Dict[str, FormValue]:
    """multipart/form-data -> {field: str | (filename, bytes)}"""
    if "multipart/form-data" not in (content_type or ""):
        raise ValueError("expected a multipart/form-data body")
    msg = BytesParser(policy=HTTP).parsebytes(b"Content-Type: " + content_type.encode() + b"\r\n\r\n" + body)
    if not msg.is_multipart():
        raise ValueError("malformed multipart body")
    out: Dict[str, FormValue] = {}
    for part in msg.iter_parts():
        name = part.get_param("name", header="content-disposition")
        if not name:
            continue
        payload = part.get_payload(decode=True) or b""
        fname = part.get_filename()
        out[name] = (fname, payload) if fname is not None else payload.decode("utf-8", "replace")
    return out


def decode_wav(data: bytes) -> Tuple[np.ndarray, int]:
    """WAV bytes -> (mono float32 in [-1, 1], sample rate)"""
    from scipy.io import wavfile
    sr, x = wavfile.read(io.BytesIO(data))
    if x.dtype == np.uint8:
        x = (x.astype(np.float32) - 128.0) / 128.0
    elif x.dtype == np.int16:
        x = x.astype(np.float32) / 32768.0
    elif x.dtype == np.int32:                    # 24-bit PCM is returned left-aligned in int32
        x = x.astype(np.float32) / 2147483648.0
    else:
        x = x.astype(np.float32)
    if x.ndim == 2:
        x = x.mean(axis=1)
    return np.ascontiguousarray(x, dtype=np.float32), int(sr)


def resample(x: np.ndarray, sr: int, target: int) -> np.ndarray:
    if sr == target:
        return x
    from scipy.signal import resample_poly
    g = math.gcd(int(sr), int(target))
    return resample_poly(x, target // g, sr // g).astype(np.float32)


class WhisperTranscriber:
    """Greedy Whisper transcription with an encoder pass and a cached
    decoder loop.  ``tokenizer`` needs ``convert_tokens_to_ids`` and
    ``decode`` (a WhisperTokenizer / WhisperProcessor.tokenizer)."""

    def __init__(self, model, feature_extractor, tokenizer, max_new_tokens: int = 440):
        self.model = model.eval()
        self.fe = feature_extractor
        self.tok = tokenizer
        self.max_new_tokens = max_new_tokens
        self.lock = threading.Lock()
        gc = getattr(model, "generation_config", None)
        eos = getattr(gc, "eos_token_id", None) if gc is not None else None
        if eos is None:
            eos = getattr(tokenizer, "eos_token_id", None)
        if eos is None:
            eos = model.config.eos_token_id
        self.eos = set(eos if isinstance(eos, (list, tuple)) else [eos])

    @property
    def sampling_rate(self) -> int:
        return int(getattr(self.fe, "sampling_rate", 16000))

    def _tid(self, token: str) -> Optional[int]:
        i = self.tok.convert_tokens_to_ids(token)
        unk = getattr(self.tok, "unk_token_id", None)
        return None if i is None or (unk is not None and i == unk) else int(i)

    def prompt_ids(self, language: Optional[str] = None, task: str = "transcribe",
                   timestamps: bool = False) -> List[int]:
        """<|startoftranscript|> [<|lang|>] <|task|> [<|notimestamps|>]"""
        ids = [self._tid("<|startoftranscript|>")]
        if language:
            lang = language.lower()
            lid = self._tid(f"<|{lang}|>")
            if lid is None:
                raise ValueError(f"unsupported language {language!r}")
            ids.append(lid)
        ids.append(self._tid(f"<|{task}|>"))
        if not timestamps:
            ids.append(self._tid("<|notimestamps|>"))
        if any(i is None for i in ids):
            raise ValueError("tokenizer lacks the Whisper special tokens")
        return ids

    def features(self, audio: np.ndarray, sr: int) -> torch.Tensor:
        audio = resample(audio, sr, self.sampling_rate)
        f = self.fe(audio, sampling_rate=self.sampling_rate, return_tensors="pt").input_features
        p = next(self.model.parameters())
        return f.to(p.device, p.dtype if p.dtype in (torch.float16, torch.bfloat16, torch.float32) else torch.float32)

    @torch.no_grad()
    def generate_ids(self, features: torch.Tensor, prompt: List[int]) -> List[int]:
        m = self.model
        enc = m.get_encoder()(features)
        dev = features.device
        ids = torch.tensor([prompt], device=dev)
        past, out = None, []
        cur = ids
        for _ in range(self.max_new_tokens):
            o = m(encoder_outputs=enc, decoder_input_ids=cur, past_key_values=past, use_cache=True)
            past = o.past_key_values
            nxt = int(o.logits[0, -1].float().argmax())
            if nxt in self.eos:
                break
            out.append(nxt)
            cur = torch.tensor([[nxt]], device=dev)
        return out

    def transcribe(self, audio: np.ndarray, sr: int, language: Optional[str] = None,
                   prompt: Optional[str] = None) -> str:
        with self.lock:
            ids = self.prompt_ids(language)
            if prompt:                               # OpenAI "prompt": previous-context tokens
                prev = self._tid("<|startofprev|>")
                if prev is not None:
                    ids = [prev] + list(self.tok.encode(" " + prompt.strip(), add_special_tokens=False)) + ids
            toks = self.generate_ids(self.features(audio, sr), ids)
            return self.tok.decode(toks, skip_special_tokens=True).strip()

    @classmethod
    def from_pretrained(cls, path: str, low_bit: Optional[str] = "sym_int4", device: Optional[str] = None, **kw):
        from transformers import WhisperProcessor
        from ..transformers import AutoModelForSpeechSeq2Seq
        proc = WhisperProcessor.from_pretrained(path)
        args = {"load_in_low_bit": low_bit} if low_bit else {}
        model = AutoModelForSpeechSeq2Seq.from_pretrained(path, **args)
        if device:
            model = model.to(device)
        return cls(model, proc.feature_extractor, proc.tokenizer, **kw)


def srt_or_vtt(text: str, fmt: str, duration: float) -> str:
    """one cue spanning the clip (no timestamp tokens are generated)"""
    def ts(t, sep):
        h, r = divmod(t, 3600)
        mi, s = divmod(r, 60)
        return f"{int(h):02d}:{int(mi):02d}:{int(s):02d}{sep}{int(round((s % 1) * 1000)):03d}"
    if fmt == "srt":
        return f"1\n{ts(0, ',')} --> {ts(duration, ',')}\n{text}\n"
    return f"WEBVTT\n\n{ts(0, '.')} --> {ts(duration, '.')}\n{text}\n"
