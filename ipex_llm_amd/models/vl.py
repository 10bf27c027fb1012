"""Vision-language models (Qwen2-VL / Qwen2.5-VL) on the native decoder.

Reference: ``SRC/transformers/models/qwen2_vl.py`` / ``qwen2_5_vl.py``
(optimized language-model forward with multimodal RoPE; the vision tower
keeps its own forward over low-bit linears) hooked in by
``SRC/transformers/convert.py``.

The language model is a Qwen2 decoder whose rotary position has three
components (temporal, height, width; "M-RoPE"): rotary frequency i uses
component s(i) given by ``mrope_section``.  For text tokens the three are
equal, so decoding after the prompt is plain RoPE at position
``cache_len + rope_delta``.  Here:

* prefill: the HF vision tower produces the image embeddings, merged into
  the token embeddings exactly as HF does; the native decoder runs on those
  embeddings (``forward_tokens(hidden_in=...)``) with a per-request cos/sin
  table whose row t holds token t's M-RoPE angles (the RoPE kernels index
  the table by position, so position t -> row t);
* decode: the shared table at rotary position ``cache_len + delta`` with
  ``pos_offset = delta`` (cache index = position - offset, the same
  mechanism compressed KV uses), captured in the usual hipGraph step.
"""
from __future__ import annotations

import copy
import time
import types
from typing import List, Optional

import torch

VL_ARCHS = {"qwen2_vl", "qwen2_5_vl"}


class _LMShim:
    """the language model of a VL checkpoint seen as a Qwen2 CausalLM"""

    def __init__(self, model):
        cfg = copy.copy(model.config.text_config)
        cfg.model_type = "qwen2"
        self.config = cfg
        self.model = model.model.language_model
        self._lm_head = model.lm_head
        self._tp = getattr(model, "_tp", None)
        self._pp = None

    def get_output_embeddings(self):
        return self._lm_head


def vl_pre(model):
    """merge q/k/v and gate/up of the language model (convert._optimize_pre)"""
    from ..transformers.convert import _merge_gate_up, _merge_qkv
    for L in model.model.language_model.layers:
        _merge_qkv(L.self_attn)
        I = getattr(getattr(L.mlp, "gate_proj", None), "out_features", 0)
        if I and I % 16 == 0:
            _merge_gate_up(L.mlp)
    model._illm_vl = True
    return model


def vl_native(model):
    from .builder import native_from_hf
    return native_from_hf(_LMShim(model))


def mrope_table(model, pos3: torch.Tensor) -> torch.Tensor:
    """per-token cos/sin rows [T, rot/2, 2] of 3-component positions pos3 [3, T]"""
    nm = model if hasattr(model, "inv_freq") else None
    inv = nm.inv_freq.float()
    sec = nm._mrope_section
    idx = torch.cat([torch.full((n,), i % 3, dtype=torch.long) for i, n in enumerate(sec)]).to(inv.device)
    p = pos3.to(inv.device).float()                                   # [3, T]
    ang = p[idx] .t() * inv[None, :]                                  # [T, rot/2]
    sc = nm.spec.rope_attention_scaling
    return torch.stack([ang.cos() * sc, ang.sin() * sc], -1).contiguous()


def _embeds(model, input_ids, pixel_values, image_grid_thw, pixel_values_videos=None, video_grid_thw=None):
    hf = model.model
    emb = hf.get_input_embeddings()(input_ids)
    if pixel_values is not None:
        dt = next(hf.visual.parameters()).dtype
        feats = hf.get_image_features(pixel_values.to(dt), image_grid_thw)
        feats = getattr(feats, "pooler_output", feats)
        feats = torch.cat(list(feats), 0) if isinstance(feats, (list, tuple)) else feats
        mask = (input_ids == model.config.image_token_id).unsqueeze(-1).to(emb.device)
        emb = emb.masked_scatter(mask, feats.to(emb.device, emb.dtype))
    if pixel_values_videos is not None:
        dt = next(hf.visual.parameters()).dtype
        feats = hf.get_video_features(pixel_values_videos.to(dt), video_grid_thw)
        feats = getattr(feats, "pooler_output", feats)
        feats = torch.cat(list(feats), 0) if isinstance(feats, (list, tuple)) else feats
        mask = (input_ids == model.config.video_token_id).unsqueeze(-1).to(emb.device)
        emb = emb.masked_scatter(mask, feats.to(emb.device, emb.dtype))
    return emb


def _prefill_mm(model, nm, eng, seq, ids: torch.Tensor, emb: torch.Tensor, pos3: torch.Tensor, all_logits: bool):
    """native prefill of one sequence on precomputed embeddings with M-RoPE rows"""
    from ..engine.runner import nsplit_for
    from .cache import make_block_table, slots_for
    from .decoder import AttnMeta
    dev = nm.device
    n = ids.numel()
    table = mrope_table(nm, pos3)
    saved = nm.rope_cache
    nm.rope_cache = table
    try:
        pos = torch.arange(n, device=dev)
        slots = slots_for(seq, 0, n, eng.cache.bs).to(dev)
        bt = make_block_table([seq], len(seq.blocks), dev)
        meta = AttnMeta(1, n, bt, torch.tensor([n], dtype=torch.int32, device=dev), nsplit_for(n), [n])
        idx = torch.arange(n, device=dev) if all_logits else torch.tensor([n - 1], device=dev)
        logits = nm.forward_tokens(ids.to(dev), pos, slots, meta, eng.cache, logits_idx=idx,
                                   hidden_in=emb.to(dev, nm.dtype))
    finally:
        nm.rope_cache = saved
    seq.length = n
    return logits


def _pos3(model, input_ids, image_grid_thw, video_grid_thw, mm_token_type_ids, attention_mask=None):
    hf = model.model
    if image_grid_thw is None and video_grid_thw is None:
        T = input_ids.shape[1]
        p = torch.arange(T).view(1, 1, T).expand(3, input_ids.shape[0], T)
        return p, torch.zeros(input_ids.shape[0], 1, dtype=torch.long)
    if mm_token_type_ids is None:
        mm_token_type_ids = torch.zeros_like(input_ids, dtype=torch.int)
        if image_grid_thw is not None:
            mm_token_type_ids[input_ids == model.config.image_token_id] = 1
        if video_grid_thw is not None:
            mm_token_type_ids[input_ids == model.config.video_token_id] = 2
    return hf.get_rope_index(input_ids, image_grid_thw=image_grid_thw, video_grid_thw=video_grid_thw,
                             attention_mask=attention_mask, mm_token_type_ids=mm_token_type_ids)


@torch.no_grad()
def vl_forward(self, input_ids=None, pixel_values=None, image_grid_thw=None, pixel_values_videos=None,
               video_grid_thw=None, mm_token_type_ids=None, attention_mask=None, **kwargs):
    """full-sequence logits of a (multimodal) prompt through the native decoder"""
    from transformers.modeling_outputs import CausalLMOutputWithPast
    from ..transformers.hf_native import get_native
    nm, eng = get_native(self)
    B, T = input_ids.shape
    emb = _embeds(self, input_ids, pixel_values, image_grid_thw, pixel_values_videos, video_grid_thw)
    pos3, _ = _pos3(self, input_ids, image_grid_thw, video_grid_thw, mm_token_type_ids, attention_mask)
    eng._ensure_cache(B, T + 1)
    out = []
    for b in range(B):
        seq = eng.new_sequence(T + 1)
        out.append(_prefill_mm(self, nm, eng, seq, input_ids[b], emb[b], pos3[:, b], True))
        eng.cache.allocator.release(seq.blocks)
    return CausalLMOutputWithPast(logits=torch.stack(out, 0))


@torch.no_grad()
def vl_generate(self, input_ids=None, pixel_values=None, image_grid_thw=None, pixel_values_videos=None,
                video_grid_thw=None, mm_token_type_ids=None, attention_mask=None, max_new_tokens=None,
                do_sample=False, eos_token_id=None, use_graph: bool = True, streamer=None, **kwargs):
    """greedy / sampled generation of a multimodal prompt: native prefill on the
    merged embeddings with M-RoPE rows, then hipGraph decode at rotary
    position cache_len + rope_delta"""
    from ..engine.runner import GenTiming, _sample
    from ..transformers.hf_native import get_native
    if pixel_values is None and pixel_values_videos is None:
        return self._illm_text_generate(input_ids=input_ids, attention_mask=attention_mask,
                                        max_new_tokens=max_new_tokens, do_sample=do_sample,
                                        eos_token_id=eos_token_id, use_graph=use_graph, streamer=streamer, **kwargs)
    gc = getattr(self, "generation_config", None)
    max_new = max_new_tokens or getattr(gc, "max_new_tokens", None) or 20
    eos = eos_token_id if eos_token_id is not None else getattr(gc, "eos_token_id", None)
    eos = set([eos] if isinstance(eos, int) else (eos or []))
    nm, eng = get_native(self)
    dev = nm.device
    B, T = input_ids.shape
    emb = _embeds(self, input_ids, pixel_values, image_grid_thw, pixel_values_videos, video_grid_thw)
    pos3, delta = _pos3(self, input_ids, image_grid_thw, video_grid_thw, mm_token_type_ids, attention_mask)
    max_len = T + max_new + 1
    eng._ensure_cache(B, max_len)
    nm.ensure_rope_cache(max_len + 1)
    timing = GenTiming()
    t0 = time.perf_counter()
    seqs, first = [], []
    for b in range(B):
        seq = eng.new_sequence(max_len)
        lg = _prefill_mm(self, nm, eng, seq, input_ids[b], emb[b], pos3[:, b], False)
        first.append(_sample(lg, do_sample, kwargs.get("temperature", 1.0), kwargs.get("top_k", 0),
                             kwargs.get("top_p", 1.0)))
        seqs.append(seq)
    cur = torch.cat(first).to(dev)
    out = [[t] for t in cur.tolist()]
    timing.first_cost = time.perf_counter() - t0
    done = [t in eos for t in cur.tolist()]
    greedy = not do_sample
    st = eng.decode_step_obj(seqs, max_len, greedy, use_graph)
    off = delta.view(-1).to(dev).long()
    st.set_state(cur, torch.tensor([s.length for s in seqs], device=dev) + off, off)
    for _ in range(1, max_new):
        if all(done):
            break
        t1 = time.perf_counter()
        nxt = st.step()
        if not greedy:
            nxt = _sample(st.logits.float(), True, kwargs.get("temperature", 1.0), kwargs.get("top_k", 0),
                          kwargs.get("top_p", 1.0))
            st.ids.copy_(nxt)
        toks = nxt.tolist()
        timing.rest_costs.append(time.perf_counter() - t1)
        for b in range(B):
            if not done[b]:
                out[b].append(toks[b])
                done[b] = toks[b] in eos
        if streamer is not None:
            streamer.put(torch.tensor(toks))
    for s in seqs:
        eng.cache.allocator.release(s.blocks)
    self.first_cost, self.rest_cost_mean = timing.first_cost, timing.rest_cost_mean
    new = max(len(o) for o in out)
    pad = next(iter(eos)) if eos else 0
    res = torch.full((B, T + new), pad, dtype=input_ids.dtype)
    res[:, :T] = input_ids.cpu()
    for b, o in enumerate(out):
        res[b, T:T + len(o)] = torch.tensor(o, dtype=input_ids.dtype)
    return res.to(input_ids.device)


def attach_vl(model):
    """native language model + M-RoPE glue on a converted Qwen2-VL"""
    from ..transformers.hf_native import native_generate
    from ..transformers.hf_views import restore_hf_views
    nm = vl_native(model)
    if nm is None:
        return model
    # HF forward keeps working (vision tower + q/k/v views over the merged weights)
    shim = types.SimpleNamespace(model=model.model.language_model)
    restore_hf_views(shim)
    model._illm_text_generate = types.MethodType(native_generate, model)
    model.generate = types.MethodType(vl_generate, model)
    model.vl_forward = types.MethodType(vl_forward, model)
    model._illm_native_attached = True
    return model
