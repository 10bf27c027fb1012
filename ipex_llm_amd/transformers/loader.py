"""Model loading helpers for tests / benchmarks (reference
``SRC/transformers/loader.py:30-172``: ``load_model`` picks the AutoModel
class, low-bit dtype and speculative flags; ``run_test_generation``)."""
from __future__ import annotations

import os
import time

import torch


def load_model(model_path: str, device: str = "cuda", low_bit: str = "sym_int4", trust_remote_code: bool = True,
               speculative: bool = False, load_low_bit_model: bool = False, **kwargs):
    from transformers import AutoTokenizer
    from .model import AutoModelForCausalLM
    kw = dict(trust_remote_code=trust_remote_code, **kwargs)
    if speculative and low_bit not in ("fp16", "bf16"):
        raise ValueError("self-speculative decoding needs low_bit fp16 or bf16 (the draft is sym_int4)")
    if load_low_bit_model:
        model = AutoModelForCausalLM.load_low_bit(model_path)
    else:
        dt = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(low_bit, "auto")
        model = AutoModelForCausalLM.from_pretrained(model_path, load_in_low_bit=low_bit, torch_dtype=dt,
                                                     speculative=speculative, **kw)
    model = model.to(device).eval()
    tok = AutoTokenizer.from_pretrained(model_path, trust_remote_code=trust_remote_code)
    return model, tok


def run_test_generation(model_path: str, device: str = "cuda", low_bit: str = "sym_int4",
                        load_low_bit_model: bool = False, prompt: str = "What is AI?", max_new_tokens: int = 32):
    model, tok = load_model(model_path, device, low_bit, load_low_bit_model=load_low_bit_model)
    ids = tok(prompt, return_tensors="pt").input_ids.to(device)
    t0 = time.perf_counter()
    out = model.generate(ids, max_new_tokens=max_new_tokens)
    dt = time.perf_counter() - t0
    text = tok.decode(out[0], skip_special_tokens=True)
    print(f"[{os.path.basename(model_path)} {low_bit}] {dt:.2f}s\n{text}")
    return text


def try_run_test_generation(local_model_hub, model_path, device, low_bit, load_low_bit_model=False):
    path = os.path.join(local_model_hub, model_path) if local_model_hub else model_path
    try:
        run_test_generation(path, device, low_bit, load_low_bit_model)
        return "success"
    except Exception as e:  # reported, not raised (reference behaviour)
        return f"failed: {e}"
