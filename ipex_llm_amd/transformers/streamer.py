"""Batched text streaming (reference ``SRC/transformers/streamer.py:26-114``,
``BatchTextIteratorStreamer``): ``put`` receives one token per sequence per
step; every sequence gets its own incrementally-decoded text queue."""
from __future__ import annotations

from queue import Queue
from typing import List, Optional

import torch


class BatchTextIteratorStreamer:
    def __init__(self, tokenizer, batch_size: int, skip_prompt: bool = True, timeout: Optional[float] = None,
                 **decode_kwargs):
        self.tokenizer, self.batch_size = tokenizer, batch_size
        self.skip_prompt, self.timeout, self.decode_kwargs = skip_prompt, timeout, decode_kwargs
        self.token_cache: List[List[int]] = [[] for _ in range(batch_size)]
        self.print_len = [0] * batch_size
        self.text_queues = [Queue() for _ in range(batch_size)]
        self.stop_signal = None
        self.next_tokens_are_prompt = True

    def put(self, value):
        if isinstance(value, torch.Tensor):
            value = value.tolist()
        if not isinstance(value, list):
            value = [value]
        if self.skip_prompt and self.next_tokens_are_prompt and value and isinstance(value[0], list):
            self.next_tokens_are_prompt = False
            return
        self.next_tokens_are_prompt = False
        for b, tok in enumerate(value[:self.batch_size]):
            toks = tok if isinstance(tok, list) else [tok]
            self.token_cache[b].extend(int(t) for t in toks)
            text = self.tokenizer.decode(self.token_cache[b], **self.decode_kwargs)
            if text.endswith("\n"):
                out, self.token_cache[b], self.print_len[b] = text[self.print_len[b]:], [], 0
            elif text.endswith("�"):
                continue
            else:
                out = text[self.print_len[b]:]
                self.print_len[b] += len(out)
            if out:
                self.text_queues[b].put(out, timeout=self.timeout)

    def end(self):
        for b in range(self.batch_size):
            if self.token_cache[b]:
                text = self.tokenizer.decode(self.token_cache[b], **self.decode_kwargs)
                rest = text[self.print_len[b]:]
                if rest:
                    self.text_queues[b].put(rest, timeout=self.timeout)
            self.text_queues[b].put(self.stop_signal, timeout=self.timeout)

    def __iter__(self):
        return self

    def __next__(self):
        """one string per sequence per call; finished sequences yield ''"""
        outs, alive = [], False
        for q in self.text_queues:
            v = q.get(timeout=self.timeout) if not getattr(q, "_done", False) else None
            if v is None:
                q._done = True
                outs.append("")
            else:
                alive = True
                outs.append(v)
        if not alive:
            raise StopIteration
        return outs
