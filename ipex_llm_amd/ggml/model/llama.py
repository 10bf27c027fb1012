"""llama.cpp-python-style model API over the native engine.

Reference: ``SRC/ggml/model/llama/llama.py`` -- ``Llama`` (123-1419:
tokenize / eval / sample / generate / completion / chat / embeddings / state
save+load), ``LlamaCache`` (63-106, prefix-keyed LRU of states) and
``LlamaState`` (109-120); the family wrappers ``Gptneox`` / ``Bloom`` /
``Starcoder`` and the HF-like ``GenerationMixin``
(``SRC/ggml/model/generation/utils.py``).  The reference drives the ggml C
library through ctypes; here the same API drives the low-bit model (native
MI355X decoder with a paged KV cache when the architecture is native, its HF
forward with a KV cache otherwise).  Model files: a HF directory, a
``save_low_bit`` directory or a ``.gguf`` file.
"""
from __future__ import annotations

import os
import time
from collections import OrderedDict, deque
from typing import Deque, List, Optional, Sequence

import torch

from ...engine.runner import Engine


class LlamaState:
    """Snapshot of one context: evaluated tokens, last logits and the KV
    contents (host copies)."""

    def __init__(self, eval_tokens: Deque[int], eval_logits: Deque[List[float]], llama_state,
                 llama_state_size: int):
        self.eval_tokens = eval_tokens
        self.eval_logits = eval_logits
        self.llama_state = llama_state
        self.llama_state_size = llama_state_size


def longest_token_prefix(a: Sequence[int], b: Sequence[int]) -> int:
    n = 0
    for x, y in zip(a, b):
        if x != y:
            break
        n += 1
    return n


class LlamaCache:
    """Prefix cache of states: lookup returns the state whose token key shares
    the longest prefix with the query (LRU eviction by total bytes)."""

    def __init__(self, capacity_bytes: int = (2 << 30)):
        self.cache_state: "OrderedDict[tuple, LlamaState]" = OrderedDict()
        self.capacity_bytes = capacity_bytes

    @property
    def cache_size(self) -> int:
        return sum(s.llama_state_size for s in self.cache_state.values())

    def _find_longest_prefix_key(self, key: Sequence[int]) -> Optional[tuple]:
        best, best_len = None, 0
        for k in self.cache_state:
            n = longest_token_prefix(k, key)
            if n > best_len:
                best, best_len = k, n
        return best

    def __getitem__(self, key: Sequence[int]) -> LlamaState:
        k = self._find_longest_prefix_key(tuple(key))
        if k is None:
            raise KeyError("no cached prefix")
        self.cache_state.move_to_end(k)
        return self.cache_state[k]

    def __contains__(self, key: Sequence[int]) -> bool:
        return self._find_longest_prefix_key(tuple(key)) is not None

    def __setitem__(self, key: Sequence[int], value: LlamaState):
        key = tuple(key)
        if key in self.cache_state:
            del self.cache_state[key]
        self.cache_state[key] = value
        while self.cache_size > self.capacity_bytes and len(self.cache_state) > 1:
            self.cache_state.popitem(last=False)


def load_model_and_tokenizer(model_path: str, low_bit: str, device):
    from ...transformers import AutoModelForCausalLM
    from ...transformers.model import LOW_BIT_META
    if model_path.endswith(".gguf"):
        model, tok = AutoModelForCausalLM.from_gguf(model_path, low_bit=low_bit)
    else:
        from transformers import AutoTokenizer
        if os.path.exists(os.path.join(model_path, LOW_BIT_META)):
            model = AutoModelForCausalLM.load_low_bit(model_path)
        else:
            model = AutoModelForCausalLM.from_pretrained(model_path, load_in_low_bit=low_bit)
        tok = AutoTokenizer.from_pretrained(model_path)
    return model.to(device).eval(), tok


class LlamaContext:
    """Token context over the model: ``eval`` extends it chunk by chunk and
    keeps the last logits; ``rewind`` keeps a prefix (the paged cache is
    position-addressed, later positions are overwritten)."""

    def __init__(self, model, n_ctx: int, n_batch: int, logits_all: bool):
        self.model = model
        self._n_ctx, self.n_batch, self.logits_all = n_ctx, min(n_ctx, n_batch), logits_all
        self.eval_tokens: Deque[int] = deque(maxlen=n_ctx)
        self.eval_logits: Deque[List[float]] = deque(maxlen=n_ctx if logits_all else 1)
        self._scores: Optional[torch.Tensor] = None          # last-token logits (f32, host)
        self._eng, self._seq, self._past = None, None, None
        try:
            from ...transformers.hf_native import get_native
            nm, _ = get_native(model)
            self._eng = Engine(nm)
            self._eng._ensure_cache(1, n_ctx + 1)
            self._seq = self._eng.new_sequence(n_ctx + 1)
        except (RuntimeError, AttributeError):
            self._eng = None
        self._device = next(model.parameters()).device

    def reset(self):
        self.eval_tokens.clear()
        self.eval_logits.clear()
        self._scores = None
        self._past = None
        if self._seq is not None:
            self._seq.length = 0

    def rewind(self, n: int):
        toks = list(self.eval_tokens)[:n]
        self.eval_tokens.clear()
        self.eval_tokens.extend(toks)
        if self._seq is not None:
            self._seq.length = n
        elif self._past is not None:
            if hasattr(self._past, "crop"):
                self._past.crop(n)
            else:
                self._past = None
                self.eval_tokens.clear()
                self.eval(toks)

    @torch.no_grad()
    def eval(self, tokens: Sequence[int]):
        toks = [int(t) for t in tokens]
        for i in range(0, len(toks), self.n_batch):
            chunk = toks[i:i + self.n_batch]
            n_past = len(self.eval_tokens)
            if n_past + len(chunk) > self._n_ctx:
                raise ValueError(f"Requested tokens exceed context window of {self._n_ctx}")
            if self._eng is not None:
                if self.logits_all:
                    lg = self._eng.forward_chunk(self._seq, chunk, n_past)
                else:
                    lg = self._eng.prefill(self._seq, torch.tensor(chunk, dtype=torch.long), n_past)
            else:
                ids = torch.tensor([chunk], dtype=torch.long, device=self._device)
                out = self.model(input_ids=ids, past_key_values=self._past, use_cache=True)
                self._past = out.past_key_values
                lg = out.logits[0].float()
                if not self.logits_all:
                    lg = lg[-1:]
            lg = lg.float().cpu()
            self.eval_tokens.extend(chunk)
            if self.logits_all:
                self.eval_logits.extend(lg.tolist())
            else:
                self.eval_logits.append(lg[-1].tolist())
            self._scores = lg[-1]

    def save(self) -> LlamaState:
        n = len(self.eval_tokens)
        kv, size = None, 0
        if self._eng is not None:
            c = self._eng.cache
            nb = (n + c.bs - 1) // c.bs
            blocks = torch.tensor(self._seq.blocks[:nb], dtype=torch.long, device=c.k[0].device)
            kv = ([k.index_select(0, blocks).cpu() for k in c.k], [v.index_select(0, blocks).cpu() for v in c.v])
            size = sum(t.numel() * t.element_size() for t in kv[0] + kv[1])
        elif self._past is not None:
            import copy
            kv = copy.deepcopy(self._past)
            size = n * 1024
        nlog = 4 * len(self.eval_logits) * (len(self.eval_logits[-1]) if self.eval_logits else 0)
        return LlamaState(deque(self.eval_tokens, maxlen=self._n_ctx),
                          deque(self.eval_logits, maxlen=self.eval_logits.maxlen), kv, size + nlog)

    def load(self, state: LlamaState) -> None:
        self.eval_tokens = deque(state.eval_tokens, maxlen=self._n_ctx)
        self.eval_logits = deque(state.eval_logits, maxlen=state.eval_logits.maxlen)
        self._scores = torch.tensor(self.eval_logits[-1]) if self.eval_logits else None
        if self._eng is not None:
            c = self._eng.cache
            if state.llama_state is not None:
                ks, vs = state.llama_state
                blocks = torch.tensor(self._seq.blocks[:ks[0].shape[0]], dtype=torch.long, device=c.k[0].device)
                for li in range(len(c.k)):
                    c.k[li].index_copy_(0, blocks, ks[li].to(c.k[li].device))
                    c.v[li].index_copy_(0, blocks, vs[li].to(c.v[li].device))
            self._seq.length = len(self.eval_tokens)
        else:
            import copy
            self._past = copy.deepcopy(state.llama_state)

    @torch.no_grad()
    def hidden(self, toks: List[int]) -> torch.Tensor:
        """final hidden states [n, H] of toks from position 0 (resets)"""
        self.reset()
        if self._eng is not None:
            from ...engine.runner import nsplit_for
            from ...models.cache import make_block_table, slots_for
            from ...models.decoder import AttnMeta
            nm, c, dev = self._eng.model, self._eng.cache, self._eng.model.device
            n = len(toks)
            meta = AttnMeta(1, n, make_block_table([self._seq], len(self._seq.blocks), dev),
                            torch.tensor([n], dtype=torch.int32, device=dev), nsplit_for(n), [n])
            h = nm.forward_tokens(torch.tensor(toks, device=dev), torch.arange(n, device=dev),
                                  slots_for(self._seq, 0, n, c.bs).to(dev), meta, c, return_hidden=True)
        else:
            out = self.model(input_ids=torch.tensor([toks], device=self._device), output_hidden_states=True)
            h = out.hidden_states[-1][0]
        self.reset()
        return h
