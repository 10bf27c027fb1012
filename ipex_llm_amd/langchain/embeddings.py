from __future__ import annotations

from typing import Any, List

import torch

try:  # optional dependency
    from langchain_core.embeddings import Embeddings as _Base
except ImportError:  # pragma: no cover
    _Base = object


class TransformersEmbeddings(_Base):
    """Sentence embeddings = mean-pooled last hidden states of a (low-bit)
    encoder/decoder (reference langchain/embeddings/transformersembeddings.py)."""

    def __init__(self, model=None, tokenizer=None, normalize: bool = False, encode_kwargs=None):
        self.model, self.tokenizer, self.normalize = model, tokenizer, normalize
        self.encode_kwargs = encode_kwargs or {}

    @classmethod
    def from_model_id(cls, model_id: str, device: str = "cuda", low_bit: str = "sym_int4", **kw):
        from transformers import AutoTokenizer
        from ..transformers import AutoModel
        model = AutoModel.from_pretrained(model_id, load_in_low_bit=low_bit).to(device)
        return cls(model, AutoTokenizer.from_pretrained(model_id), **kw)

    @torch.no_grad()
    def embed(self, text: str) -> List[float]:
        dev = next(self.model.parameters()).device
        enc = self.tokenizer(text, return_tensors="pt", truncation=True).to(dev)
        out = self.model(**enc, output_hidden_states=True)
        h = out.hidden_states[-1] if getattr(out, "hidden_states", None) is not None else out.last_hidden_state
        mask = enc["attention_mask"][..., None].to(h.dtype)
        v = (h * mask).sum(1) / mask.sum(1)
        if self.normalize:
            v = torch.nn.functional.normalize(v, dim=-1)
        return v[0].float().cpu().tolist()

    def embed_documents(self, texts: List[str]) -> List[List[float]]:
        return [self.embed(t) for t in texts]

    def embed_query(self, text: str) -> List[float]:
        return self.embed(text)


class TransformersBgeEmbeddings(TransformersEmbeddings):
    """BGE: CLS pooling + normalisation, query instruction prefix"""

    query_instruction = "Represent this sentence for searching relevant passages: "

    def __init__(self, *a, **kw):
        kw.setdefault("normalize", True)
        super().__init__(*a, **kw)

    @torch.no_grad()
    def embed(self, text: str) -> List[float]:
        dev = next(self.model.parameters()).device
        enc = self.tokenizer(text, return_tensors="pt", truncation=True).to(dev)
        out = self.model(**enc)
        h = out.last_hidden_state[:, 0]
        return torch.nn.functional.normalize(h, dim=-1)[0].float().cpu().tolist()

    def embed_query(self, text: str) -> List[float]:
        return self.embed(self.query_instruction + text)
