"""Structured (JSON / JSON-schema) output as a logits processor.

Reference: ``SRC/transformers/xgrammar.py`` (wraps the ``xgrammar`` package:
``create_json_logits_processor(tokenizer, vocab_size, schema)`` /
``reset_json_logits_processor``; xgrammar compiles the schema to a grammar
and masks tokens with a bitmask every step).  ``xgrammar`` is not available
in this image, so the processor is native:

* no schema: an incremental JSON pushdown recognizer (any JSON value);
* a JSON schema: compiled to a regular expression over the output text
  (objects with declared properties in declared order, required / optional
  properties, arrays with min/maxItems, string length / pattern, enum,
  const, integer / number / boolean / null, anyOf / oneOf, type lists,
  local ``$ref``), matched incrementally with partial matching
  (``regex.fullmatch(..., partial=True)``): a token is allowed iff the
  output extended by it can still complete to a schema-valid document, EOS
  iff the document is complete.

Each step the highest-scoring candidates are checked first and the search
widens until at least one token passes.  Parity with xgrammar's exact
whitespace rules is unpinned (here: at most one space between tokens).
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


# ----------------------------------------------------------------- schema -> regex
_WSP = r" ?"
_STR_CHAR = r'(?:[^"\\\x00-\x1f]|\\["\\/bfnrt]|\\u[0-9a-fA-F]{4})'
_INT = r"-?(?:0|[1-9][0-9]{0,15})"
_NUM = _INT + r"(?:\.[0-9]{1,16})?(?:[eE][+-]?[0-9]{1,3})?"


def _lit(v) -> str:
    import json
    import regex
    return regex.escape(json.dumps(v, separators=(", ", ": ")))


def _generic(depth: int) -> str:
    """any JSON value, nesting limited to ``depth`` (regular)"""
    scalar = "(?:" + "|".join(['"' + _STR_CHAR + '*"', _NUM, "true", "false", "null"]) + ")"
    if depth <= 0:
        return scalar
    inner = _generic(depth - 1)
    obj = r"\{(?:" + _WSP + '"' + _STR_CHAR + '*"' + _WSP + ":" + _WSP + inner + "(?:" + _WSP + "," + _WSP + \
        '"' + _STR_CHAR + '*"' + _WSP + ":" + _WSP + inner + ")*)?" + _WSP + r"\}"
    arr = r"\[(?:" + _WSP + inner + "(?:" + _WSP + "," + _WSP + inner + ")*)?" + _WSP + r"\]"
    return "(?:" + "|".join([scalar, obj, arr]) + ")"


def schema_to_regex(schema, root=None, depth: int = 0) -> str:
    """JSON schema -> regular expression of its valid documents (compact:
    at most one space around ``:`` / ``,`` / brackets)"""
    import regex
    root = schema if root is None else root
    if depth > 24:
        raise ValueError("JSON schema nests too deeply (recursive $ref?)")
    if schema is True or schema == {}:
        return _generic(3)
    if "$ref" in schema:
        ref = schema["$ref"]
        if not ref.startswith("#/"):
            raise ValueError(f"only local $ref is supported, got {ref}")
        node = root
        for part in ref[2:].split("/"):
            node = node[part]
        return schema_to_regex(node, root, depth + 1)
    if "const" in schema:
        return _lit(schema["const"])
    if "enum" in schema:
        return "(?:" + "|".join(_lit(v) for v in schema["enum"]) + ")"
    for key in ("anyOf", "oneOf"):
        if key in schema:
            return "(?:" + "|".join(schema_to_regex(s, root, depth + 1) for s in schema[key]) + ")"
    if "allOf" in schema and len(schema["allOf"]) == 1:
        return schema_to_regex(schema["allOf"][0], root, depth + 1)
    t = schema.get("type")
    if isinstance(t, list):
        return "(?:" + "|".join(schema_to_regex({**schema, "type": x}, root, depth + 1) for x in t) + ")"
    if t == "object" or (t is None and "properties" in schema):
        props = schema.get("properties", {})
        if not props:
            return _generic(3) if t is None else r"\{(?:" + _WSP + '"' + _STR_CHAR + '*"' + _WSP + ":" + \
                _WSP + _generic(2) + "(?:" + _WSP + "," + _WSP + '"' + _STR_CHAR + '*"' + _WSP + ":" + _WSP + \
                _generic(2) + ")*)?" + _WSP + r"\}"
        req = set(schema.get("required", []))
        names = list(props)
        items = [regex.escape('"' + n + '"') + _WSP + ":" + _WSP + schema_to_regex(props[n], root, depth + 1)
                 for n in names]
        sep = _WSP + "," + _WSP
        alts = []
        for f in range(len(names)):
            if any(n in req for n in names[:f]):
                break                            # a required property cannot be skipped
            pat = items[f]
            for j in range(f + 1, len(names)):
                pat += (sep + items[j]) if names[j] in req else "(?:" + sep + items[j] + ")?"
            alts.append(pat)
        body = "(?:" + _WSP + "(?:" + "|".join(alts) + "))"
        if not req:
            body += "?"
        return r"\{" + body + _WSP + r"\}"
    if t == "array":
        item = schema_to_regex(schema.get("items", {}), root, depth + 1)
        lo, hi = int(schema.get("minItems", 0)), schema.get("maxItems")
        sep = _WSP + "," + _WSP
        if hi is not None and int(hi) == 0:
            return r"\[" + _WSP + r"\]"
        rest = "{%d,%s}" % (max(lo - 1, 0), "" if hi is None else int(hi) - 1)
        body = "(?:" + _WSP + item + "(?:" + sep + item + ")" + rest + ")"
        if lo == 0:
            body += "?"
        return r"\[" + body + _WSP + r"\]"
    if t == "string":
        if "pattern" in schema:
            p = schema["pattern"]
            p = p[1:] if p.startswith("^") else p
            p = p[:-1] if p.endswith("$") else p
            return '"' + "(?:" + p + ")" + '"'
        lo, hi = int(schema.get("minLength", 0)), schema.get("maxLength")
        return '"' + _STR_CHAR + "{%d,%s}" % (lo, "" if hi is None else int(hi)) + '"'
    if t == "integer":
        return _INT
    if t == "number":
        return _NUM
    if t == "boolean":
        return "(?:true|false)"
    if t == "null":
        return "null"
    return _generic(3)


class _RegexState:
    """incremental matcher over the decoded output (prefix check = partial match)"""

    def __init__(self, pattern):
        self.pat = pattern

    def viable(self, text: str) -> bool:
        return self.pat.fullmatch(text, partial=True) is not None

    def complete(self, text: str) -> bool:
        return self.pat.fullmatch(text) is not None


class JsonLogitsProcessor:
    def __init__(self, tokenizer, vocab_size: int, schema=None, max_candidates: int = 64):
        self.tok, self.V = tokenizer, vocab_size
        if isinstance(schema, str):
            import json
            schema = json.loads(schema)
        self.top = (schema or {}).get("type") if isinstance(schema, dict) else None
        self.max_candidates = max_candidates
        self.schema = schema
        self.prompt_len: Optional[int] = None
        self.states: List[_JsonState] = []
        self.rx = None
        if isinstance(schema, dict) and schema:
            import regex
            self.rx = _RegexState(regex.compile(schema_to_regex(schema)))

    def _state_for(self, b: int, gen: List[int]) -> _JsonState:
        st = _JsonState(self.top)
        for ch in self.tok.decode(gen, skip_special_tokens=True):
            st.feed(ch)
        return st

    def _allowed_schema(self, gen: List[int], row: torch.Tensor, eos) -> List[int]:
        text = self.tok.decode(gen, skip_special_tokens=True)
        order = torch.argsort(row, descending=True).tolist()
        allowed, lo = [], 0
        width = self.max_candidates
        while not allowed and lo < len(order):
            for t in order[lo:lo + width]:
                if t == eos:
                    if self.rx.complete(text):
                        allowed.append(t)
                    continue
                ext = self.tok.decode(gen + [t], skip_special_tokens=True)
                if ext != text and self.rx.viable(ext):
                    allowed.append(t)
            lo += width
            width *= 4                                  # widen until some token fits
        return allowed

    def __call__(self, input_ids: torch.Tensor, scores: torch.Tensor) -> torch.Tensor:
        if self.prompt_len is None:
            self.prompt_len = input_ids.shape[1]
        out = torch.full_like(scores, float("-inf"))
        eos = getattr(self.tok, "eos_token_id", None)
        if self.rx is not None:
            for b in range(scores.shape[0]):
                gen = input_ids[b, self.prompt_len:].tolist()
                allowed = self._allowed_schema(gen, scores[b], eos) or ([eos] if eos is not None else [])
                out[b, allowed] = scores[b, allowed]
            return out
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
