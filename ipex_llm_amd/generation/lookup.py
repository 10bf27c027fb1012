"""Prompt-lookup decoding (n-gram candidates verified in one forward).

Reference: ``SRC/transformers/lookup.py`` -- ``PromptLookupCandidateGenerator``
(145-272: n-gram lookup table over prompt + output, adaptive candidate
count) and ``lookup_generate`` (274-457); ``IPEX_LLM_PERFORMANCE_MODE=1``
turns it on for prompts of >= 100 tokens (50-135).

Here verification is one native forward over ``[last] + candidates`` on the
paged KV cache; rejected positions need no cache crop (the cache is
position-addressed: ``seq.length`` is rewound and later writes overwrite
them).  With GQA group * (1 + candidates) <= 16 the verify step runs on the
flash-decoding kernel, i.e. it costs about one decode step.
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

import torch

PERFORMANCE_MODE_LOOKUP_INPUT_THRESHOLD = 100


def performance_mode_lookahead(prompt_len: int) -> Optional[int]:
    """Reference behaviour: IPEX_LLM_PERFORMANCE_MODE=1 -> lookahead 2 for long prompts."""
    if os.environ.get("IPEX_LLM_PERFORMANCE_MODE") == "1" and prompt_len >= PERFORMANCE_MODE_LOOKUP_INPUT_THRESHOLD:
        return 2
    return None


class PromptLookupCandidates:
    """n-gram -> earliest position table, updated as tokens are generated, and
    the reference's adaptive candidate count
    (``PromptLookupCandidateGenerator.update_candidate_strategy``,
    SRC/transformers/lookup.py:163-175, 253-270): +1 (capped at
    ``max_candidates`` = 9) when every candidate was accepted; otherwise -1 with
    probability that grows with the number of rejected candidates and falls with
    the running acceptance rate; from 0 candidates (plain decoding) the count is
    re-enabled at 1 with probability ~ the acceptance rate + 0.15."""

    def __init__(self, num_output_tokens: int = 10, max_matching_ngram_size: int = 2, min_candidates: int = 0,
                 max_candidates: int = 9, seed: Optional[int] = None):
        import random
        self.num_output_tokens = num_output_tokens
        self.max_n = max(1, max_matching_ngram_size)
        self.min_c, self.max_c = min_candidates, max_candidates
        self.table: Dict[Tuple[int, ...], int] = {}
        self.tokens: List[int] = []
        self.n_drafted = 0
        self.n_matched = 0
        self._rng = random.Random(seed)

    def init(self, tokens: Sequence[int]):
        self.tokens = list(tokens)
        for n in range(1, self.max_n + 1):
            for i in range(len(self.tokens) - n + 1):
                self.table.setdefault(tuple(self.tokens[i:i + n]), i)

    def extend(self, new: Sequence[int]):
        start = len(self.tokens)
        self.tokens.extend(new)
        for n in range(1, self.max_n + 1):
            for i in range(max(0, start - n + 1), len(self.tokens) - n + 1):
                self.table.setdefault(tuple(self.tokens[i:i + n]), i)

    def candidates(self) -> List[int]:
        if self.num_output_tokens == 0:
            return []
        L = len(self.tokens)
        for n in range(min(self.max_n, L - 1), 0, -1):
            key = tuple(self.tokens[L - n:])
            i = self.table.get(key)
            if i is not None and i + n < L:
                return self.tokens[i + n:i + n + self.num_output_tokens]
        return []

    @property
    def accept_rate(self) -> float:
        return self.n_matched / self.n_drafted if self.n_drafted > 0 else 1.0

    def update(self, n_cand: int, n_accepted: int, accept_rate: Optional[float] = None):
        """one verify step: ``n_cand`` candidates drafted, ``n_accepted`` matched"""
        self.n_drafted += n_cand
        self.n_matched += n_accepted
        rate = self.accept_rate if accept_rate is None else accept_rate
        if self.num_output_tokens == 0:
            if self._rng.random() - 0.15 <= rate:
                self.num_output_tokens = 1
        elif n_accepted == self.num_output_tokens:
            self.num_output_tokens = min(self.num_output_tokens + 1, self.max_c)
        elif n_cand > n_accepted:
            if self._rng.random() + 0.1 * (n_cand - n_accepted) > rate:
                self.num_output_tokens = max(self.num_output_tokens - 1, self.min_c)


@torch.no_grad()
def lookup_generate(engine, prompts: Sequence[Sequence[int]], num_output_tokens: int = 10, max_new_tokens: int = 32,
                    eos_token_id=None, timing=None, streamer=None, max_matching_ngram_size: int = 2,
                    min_new_tokens: int = 0, **_) -> List[List[int]]:
    """Greedy generation with prompt-lookup speculation (one sequence at a
    time, like the reference).  Output tokens equal plain greedy decoding."""
    eos = set([eos_token_id] if isinstance(eos_token_id, int) else (eos_token_id or []))
    outs = []
    sync = torch.cuda.synchronize if engine.model.device.type == "cuda" else (lambda: None)
    engine.lookup_stats = {"drafted": 0, "accepted": 0, "steps": 0}
    for p in prompts:
        p = list(p)
        max_len = len(p) + max_new_tokens + num_output_tokens + 16
        engine._ensure_cache(1, max_len)
        seq = engine.new_sequence(max_len)
        t0 = time.perf_counter()
        lg = engine.forward_chunk(seq, p, 0)
        last = int(torch.argmax(lg[-1]))
        out = p + [last]
        sync()
        if timing is not None:
            timing.first_cost = time.perf_counter() - t0
        if streamer is not None:
            streamer.put(torch.tensor([last]))
        gen = PromptLookupCandidates(num_output_tokens, max_matching_ngram_size)
        gen.init(out)
        new = 1
        while new < max_new_tokens and not (last in eos and new >= min_new_tokens):
            t1 = time.perf_counter()
            cand = gen.candidates()[:max(0, max_new_tokens - new - 1)]
            lg = engine.forward_chunk(seq, [last] + cand, seq.length)
            pred = torch.argmax(lg, -1).tolist()
            m = 0
            while m < len(cand) and cand[m] == pred[m]:
                m += 1
            accepted = cand[:m] + [pred[m]]
            seq.length -= len(cand) - m               # rewind past the rejected candidates
            stop = False
            emitted = []
            for t in accepted:
                emitted.append(t)
                new += 1
                if (t in eos and new >= min_new_tokens) or new >= max_new_tokens:
                    stop = True
                    break
            out.extend(emitted)
            gen.extend(emitted)
            gen.update(len(cand), m)
            engine.lookup_stats["drafted"] += len(cand)
            engine.lookup_stats["accepted"] += m
            engine.lookup_stats["steps"] += 1
            last = emitted[-1]
            sync()
            if timing is not None:
                dt = time.perf_counter() - t1
                timing.rest_costs.extend([dt / len(emitted)] * len(emitted))
            if streamer is not None:
                streamer.put(torch.tensor(emitted))
            if stop:
                break
        engine.cache.allocator.release(seq.blocks)
        outs.append(out)
    if streamer is not None:
        streamer.end()
    return outs
