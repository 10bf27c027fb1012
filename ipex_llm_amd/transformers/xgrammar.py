"""Structured (JSON) output as a logits processor.

Reference: ``SRC/transformers/xgrammar.py`` (wraps the ``xgrammar`` package:
``create_json_logits_processor(tokenizer, vocab_size, schema)`` /
``reset_json_logits_processor``).  ``xgrammar`` is not available in this
image, so the processor is native: an incremental JSON pushdown recognizer
over the decoded text; each step the highest-scoring candidates (top
``max_candidates``) are checked in order and every token that would make the
output an invalid JSON prefix is masked.  ``schema`` only constrains the
top-level type (object/array); full JSON-schema validation is parity
unpinned.
"""
from __future__ import annotations

from typing import List, Optional

import torch

_WS = " \t\n\r"


class _JsonState:
    """character-level JSON prefix recognizer (returns False on the first invalid char)"""

    def __init__(self, top: Optional[str] = None):
        self.stack: List[str] = []          # 'o' object, 'a' array
        self.mode = "value"                 # what is expected next
        self.top = top
        self.in_str = self.esc = False
        self.str_is_key = False
        self.lit = ""                       # pending literal / number chars
        self.done = False
        self.started = False
        self.ws_run = 0                     # consecutive whitespace (capped: generation must progress)

    def copy(self):
        c = _JsonState.__new__(_JsonState)
        c.__dict__ = {**self.__dict__, "stack": list(self.stack)}
        return c

    def _end_value(self):
        if not self.stack:
            self.done = True
            self.mode = "end"
        else:
            self.mode = "comma_or_close"

    def feed(self, ch: str) -> bool:
        if self.in_str:
            if self.esc:
                self.esc = False
            elif ch == "\\":
                self.esc = True
            elif ch == '"':
                self.in_str = False
                if self.str_is_key:
                    self.mode = "colon"
                else:
                    self._end_value()
            return True
        if self.lit:
            if ch.isalnum() or ch in ".+-eE":
                self.lit += ch
                return self._lit_ok(partial=True)
            if not self._lit_ok(partial=False):
                return False
            self.lit = ""
            self._end_value()
        if ch in _WS:
            if not self.started or self.ws_run >= 1 or self.done:
                return False
            self.ws_run += 1
            return True
        self.ws_run = 0
        self.started = True
        if self.mode == "end":
            return False
        if self.mode == "key_or_close":
            if ch == "}":
                return self._close("o")
            if ch == '"':
                self.in_str, self.str_is_key = True, True
                return True
            return False
        if self.mode == "key":
            if ch == '"':
                self.in_str, self.str_is_key = True, True
                return True
            return False
        if self.mode == "colon":
            if ch == ":":
                self.mode = "value"
                return True
            return False
        if self.mode == "comma_or_close":
            top = self.stack[-1]
            if ch == ",":
                self.mode = "key" if top == "o" else "value"
                return True
            return self._close(top) if ch in "}]" and {"}": "o", "]": "a"}[ch] == top else False
        if self.mode in ("value", "value_or_close"):
            if self.mode == "value_or_close" and ch == "]":
                return self._close("a")
            if not self.stack and self.top is not None and ch != {"object": "{", "array": "["}.get(self.top, ch):
                return False
            if ch == "{":
                self.stack.append("o")
                self.mode = "key_or_close"
                return True
            if ch == "[":
                self.stack.append("a")
                self.mode = "value_or_close"
                return True
            if ch == '"':
                self.in_str, self.str_is_key = True, False
                return True
            if ch in "-0123456789tfn":
                self.lit = ch
                return self._lit_ok(partial=True)
        return False

    def _close(self, kind):
        if not self.stack or self.stack[-1] != kind:
            return False
        self.stack.pop()
        self._end_value()
        return True

    def _lit_ok(self, partial: bool) -> bool:
        s = self.lit
        for word in ("true", "false", "null"):
            if word.startswith(s) or s == word:
                return True if partial else s == word
        try:
            float(s)
            return True
        except ValueError:
            return partial and s in ("-",) or (partial and s[-1] in "eE+-." and _num_prefix(s))


def _num_prefix(s: str) -> bool:
    try:
        float(s + "0")
        return True
    except ValueError:
        return False


class JsonLogitsProcessor:
    def __init__(self, tokenizer, vocab_size: int, schema=None, max_candidates: int = 64):
        self.tok, self.V = tokenizer, vocab_size
        self.top = (schema or {}).get("type") if isinstance(schema, dict) else None
        self.max_candidates = max_candidates
        self.schema = schema
        self.prompt_len: Optional[int] = None
        self.states: List[_JsonState] = []

    def _state_for(self, b: int, gen: List[int]) -> _JsonState:
        st = _JsonState(self.top)
        for ch in self.tok.decode(gen, skip_special_tokens=True):
            st.feed(ch)
        return st

    def __call__(self, input_ids: torch.Tensor, scores: torch.Tensor) -> torch.Tensor:
        if self.prompt_len is None:
            self.prompt_len = input_ids.shape[1]
        out = torch.full_like(scores, float("-inf"))
        eos = getattr(self.tok, "eos_token_id", None)
        for b in range(scores.shape[0]):
            gen = input_ids[b, self.prompt_len:].tolist()
            st = self._state_for(b, gen)
            order = torch.argsort(scores[b], descending=True)[: self.max_candidates].tolist()
            allowed = []
            for t in order:
                if t == eos:
                    if st.done:
                        allowed.append(t)
                    continue
                text = self.tok.decode([t], skip_special_tokens=True)
                if not text:
                    continue
                c = st.copy()
                if all(c.feed(ch) for ch in text):
                    allowed.append(t)
            if not allowed and eos is not None:
                allowed = [eos]
            out[b, allowed] = scores[b, allowed]
        return out


def create_json_logits_processor(tokenizer, vocab_size: int, schema=None):
    return JsonLogitsProcessor(tokenizer, vocab_size, schema)


def reset_json_logits_processor(processor: JsonLogitsProcessor) -> JsonLogitsProcessor:
    return JsonLogitsProcessor(processor.tok, processor.V, processor.schema, processor.max_candidates)
