"""Perplexity harness (sliding window over one token stream).

Reference: ``python/llm/dev/benchmark/perplexity/run_wikitext.py`` (HF's
strided perplexity recipe: windows of ``max_length`` tokens advanced by
``stride``, only the tokens not seen by the previous window are scored) and
``ppl.py`` (per-sample perplexity of an optimized model).  No dataset
download here: the token stream comes from a local text file (tokenized with
the model's tokenizer) or from ids the caller already has.

    python -m ipex_llm_amd.cli ppl --model_path DIR --data_path wiki.test.raw --precision sym_int4
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F


@torch.no_grad()
def strided_perplexity(model, ids: torch.Tensor, max_length: int = 512, stride: Optional[int] = None,
                       device=None) -> Dict:
    """ids: [1, N] or [N] token ids.  Returns {"ppl", "nll", "tokens", "windows"}.
    With stride == max_length the windows are disjoint; a smaller stride
    gives every scored token up to max_length - stride tokens of context."""
    ids = ids.reshape(1, -1)
    stride = stride or max_length
    assert 0 < stride <= max_length
    dev = device or next(model.parameters()).device
    N = ids.shape[1]
    nll, count, windows, prev_end = 0.0, 0, 0, 0
    for begin in range(0, N, stride):
        end = min(begin + max_length, N)
        trg_len = end - prev_end                  # tokens not scored by the previous window
        x = ids[:, begin:end].to(dev)
        logits = model(x).logits.float()
        # score positions [end - trg_len, end) -> predicted from the position before
        first = max(1, x.shape[1] - trg_len)
        lg = logits[0, first - 1:-1]
        tgt = x[0, first:]
        nll += F.cross_entropy(lg, tgt, reduction="sum").item()
        count += tgt.numel()
        windows += 1
        prev_end = end
        if end == N:
            break
    mean = nll / max(1, count)
    return {"ppl": math.exp(mean), "nll": mean, "tokens": count, "windows": windows}


def text_ids(tokenizer, path: str, max_tokens: Optional[int] = None) -> torch.Tensor:
    """a local text file -> one token stream (wikitext is joined with blank lines)"""
    with open(path, encoding="utf-8") as f:
        text = f.read()
    ids = tokenizer(text, return_tensors="pt").input_ids
    return ids[:, :max_tokens] if max_tokens else ids


__all__ = ["strided_perplexity", "text_ids"]
