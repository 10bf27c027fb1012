"""Glue between a converted HF ``*ForCausalLM`` and the native decoder.

Reference: the per-arch ``*_model_forward`` replacements + patched
``GenerationMixin.generate`` (``SRC/transformers/lookup.py:50-135``,
``pipeline_parallel.py:238-296``) and ``BenchmarkWrapper``'s timing
(``utils/benchmark_util_4_47.py:3295-3400``).

``attach_native(model)`` rebinds ``model.forward`` and ``model.generate``:
  * ``forward(input_ids, attention_mask, past_key_values, labels)`` -> HF
    ``CausalLMOutputWithPast`` (full-sequence logits, optional loss), with a
    paged-KV ``NativeCache`` as ``past_key_values`` for incremental calls;
  * ``generate(...)`` -> the graph-captured engine loop (greedy / sampling /
    repetition penalty / eos / streamer / prompt-lookup / self-speculative),
    recording ``first_cost`` / ``rest_cost_mean`` like BenchmarkWrapper.
The native model shares every parameter with the HF module tree; it is
(re)built lazily whenever the HF model changes device.
"""
from __future__ import annotations

import types
from typing import List, Optional

import torch
import torch.nn.functional as F

from ..engine.runner import Engine, GenTiming
from ..models.cache import SequenceState, make_block_table, slots_for
from ..models.decoder import AttnMeta


def _model_device(model) -> torch.device:
    for p in model.parameters():
        if p.device.type != "meta":
            return p.device
    return torch.device("cpu")


def get_native(model):
    from ..models.builder import native_from_hf
    dev = _model_device(model)
    st = model.__dict__.get("_illm_state")
    if st is None or st["device"] != dev:
        nm = native_from_hf(model)
        if nm is None:
            raise RuntimeError("model layout not supported by the native decoder")
        kv_fp8 = 1 if getattr(model, "_illm_kv_fp8", False) else 0
        st = {"device": dev, "native": nm, "engine": Engine(nm, kv_fp8=kv_fp8)}
        model.__dict__["_illm_state"] = st
    return st["native"], st["engine"]


class NativeCache:
    """past_key_values handle for incremental ``forward`` calls."""

    def __init__(self, engine: Engine, seqs: List[SequenceState], capacity: int):
        self.engine, self.seqs, self.capacity = engine, seqs, capacity

    def get_seq_length(self, layer_idx: int = 0) -> int:
        return self.seqs[0].length if self.seqs else 0

    def __len__(self):
        return self.engine.model.spec.num_layers

    def release(self):
        for s in self.seqs:
            self.engine.cache.allocator.release(s.blocks)
        self.seqs = []


def _row_tokens(input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor]) -> List[List[int]]:
    rows = []
    for b in range(input_ids.shape[0]):
        ids = input_ids[b]
        if attention_mask is not None:
            ids = ids[attention_mask[b].bool()]
        rows.append(ids.tolist())
    return rows


def native_forward(self, input_ids=None, attention_mask=None, position_ids=None, past_key_values=None,
                   inputs_embeds=None, labels=None, use_cache=None, return_dict=True, max_cache_len=None,
                   **kwargs):
    from transformers.modeling_outputs import CausalLMOutputWithPast
    if input_ids is None:
        raise ValueError("native forward needs input_ids")
    nm, eng = get_native(self)
    dev = nm.device
    B, S = input_ids.shape
    cache = past_key_values if isinstance(past_key_values, NativeCache) else None
    if cache is None:
        cap = max_cache_len or (S + 512)
        eng._ensure_cache(B, cap)
        nblk = (cap + eng.block_size - 1) // eng.block_size
        cache = NativeCache(eng, [SequenceState(eng.cache.allocator.alloc(nblk)) for _ in range(B)], cap)
    rows = _row_tokens(input_ids, attention_mask if cache.get_seq_length() == 0 else None)
    V = nm.spec.vocab_size
    logits = torch.zeros(B, S, V, dtype=torch.float32, device=dev)
    with torch.no_grad():
        for b, toks in enumerate(rows):
            seq = cache.seqs[b]
            n = len(toks)
            if n == 0:
                continue
            start = seq.length
            if start + n > cache.capacity:
                raise RuntimeError("NativeCache capacity exceeded; pass max_cache_len")
            pos = torch.arange(start, start + n, device=dev)
            slots = slots_for(seq, start, n, eng.cache.bs).to(dev)
            L = start + n
            bt = make_block_table([seq], len(seq.blocks), dev)
            from ..engine.runner import nsplit_for
            meta = AttnMeta(1, n, bt, torch.tensor([L], dtype=torch.int32, device=dev), nsplit_for(L), [L])
            lg = nm.forward_tokens(torch.tensor(toks, device=dev), pos, slots, meta, eng.cache,
                                   logits_idx=torch.arange(n, device=dev))
            logits[b, S - n:] = lg
            seq.length = L
    loss = None
    if labels is not None:
        sl = logits[:, :-1].reshape(-1, V)
        tl = labels[:, 1:].reshape(-1).to(dev)
        loss = F.cross_entropy(sl, tl, ignore_index=-100)
    if use_cache is False and past_key_values is None:
        cache.release()
        cache = None
    out = CausalLMOutputWithPast(loss=loss, logits=logits, past_key_values=cache)
    return out if return_dict else out.to_tuple()


def native_generate(self, input_ids=None, attention_mask=None, generation_config=None, streamer=None,
                    max_new_tokens=None, max_length=None, min_new_tokens=None, do_sample=None,
                    temperature=None, top_k=None, top_p=None, repetition_penalty=None, eos_token_id=None,
                    pad_token_id=None, prompt_lookup_num_tokens=None, lookahead=None, use_graph=True,
                    logits_processor=None, **kwargs):
    gc = generation_config or getattr(self, "generation_config", None)

    def pick(v, name, default):
        if v is not None:
            return v
        g = getattr(gc, name, None) if gc is not None else None
        return default if g is None else g

    max_new = pick(max_new_tokens, "max_new_tokens", None)
    if max_new is None:
        ml = pick(max_length, "max_length", 20)
        max_new = max(1, ml - input_ids.shape[1])
    do_sample = pick(do_sample, "do_sample", False)
    eos = pick(eos_token_id, "eos_token_id", None)
    pad = pick(pad_token_id, "pad_token_id", None)
    if pad is None:
        pad = eos[0] if isinstance(eos, (list, tuple)) else (eos if eos is not None else 0)
    kw = dict(max_new_tokens=max_new, min_new_tokens=pick(min_new_tokens, "min_new_tokens", 0) or 0,
              do_sample=do_sample, temperature=pick(temperature, "temperature", 1.0),
              top_k=pick(top_k, "top_k", 0) or 0, top_p=pick(top_p, "top_p", 1.0),
              repetition_penalty=pick(repetition_penalty, "repetition_penalty", 1.0), eos_token_id=eos)
    nm, eng = get_native(self)
    prompts = _row_tokens(input_ids, attention_mask)
    timing = GenTiming()
    lookup = prompt_lookup_num_tokens or lookahead
    if not lookup and len(prompts) == 1:
        from ..generation.lookup import performance_mode_lookahead
        lookup = performance_mode_lookahead(len(prompts[0]))
    if getattr(self, "_illm_speculative", False) and not do_sample:
        from ..generation.speculative import speculative_generate
        outs = speculative_generate(self, prompts, timing=timing, streamer=streamer, **kw)
    elif lookup and not do_sample:
        from ..generation.lookup import lookup_generate
        outs = lookup_generate(eng, prompts, num_output_tokens=int(lookup), timing=timing, streamer=streamer, **kw)
    else:
        lp = None
        if logits_processor:
            procs = list(logits_processor) if isinstance(logits_processor, (list, tuple)) or \
                hasattr(logits_processor, "__iter__") else [logits_processor]

            def lp(ids, scores):
                for p in procs:
                    scores = p(ids, scores)
                return scores
        outs = eng.generate(prompts, streamer=streamer, use_graph=use_graph, timing=timing, logits_processor=lp, **kw)
    self.first_cost = timing.first_cost
    self.rest_cost_mean = timing.rest_cost_mean
    self.last_timing = timing
    B, S = input_ids.shape
    new_max = max(len(o) - len(p) for o, p in zip(outs, prompts))
    res = torch.full((B, S + new_max), pad, dtype=input_ids.dtype)
    res[:, :S] = input_ids.cpu()
    for b, (o, p) in enumerate(zip(outs, prompts)):
        gen = o[len(p):]
        res[b, S:S + len(gen)] = torch.tensor(gen, dtype=input_ids.dtype)
    return res.to(input_ids.device)


def attach_native(model):
    from ..models.builder import native_from_hf
    if native_from_hf(model) is None:        # layout the native decoder cannot run: keep HF forward
        return model
    model.forward = types.MethodType(native_forward, model)
    model.generate = types.MethodType(native_generate, model)
    model._illm_native_attached = True
    return model
