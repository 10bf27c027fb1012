"""Self-speculative decoding: an INT4 copy of the model drafts, the
fp16/bf16 model verifies.

Reference: ``SRC/transformers/speculative.py`` -- the ``speculative=True``
load path creates a sym_int4 draft of the same checkpoint
(``model.py`` speculative branch), ``speculative_generate`` (805-1271)
drafts up to ``max_step_draft`` tokens, stops early when the draft's top
probability falls below ``th_stop_draft`` (auto-tuned), verifies in one
target forward and crops the KV caches (``_crop_past_key_values``, 480-549).

Here both models run on the native engine with paged KV caches, so the
crop is a length rewind; verification is one native forward over
``[last] + drafts``.  Greedy output equals the target model's plain greedy
decoding.
"""
from __future__ import annotations

import time
from typing import List, Optional, Sequence

import torch


def enable_self_speculative(model, path, torch_dtype="auto", draft_qtype: str = "sym_int4", **kwargs):
    """Load the INT4 draft of ``path`` and attach it to ``model``."""
    from ..transformers.model import AutoModelForCausalLM
    kwargs = {k: v for k, v in kwargs.items() if k not in ("load_in_4bit", "load_in_low_bit", "speculative")}
    draft = AutoModelForCausalLM.from_pretrained(path, load_in_low_bit=draft_qtype, torch_dtype=torch_dtype,
                                                 **kwargs)
    attach_draft(model, draft)
    return model


def attach_draft(model, draft):
    model.__dict__["draft_model"] = draft       # not a submodule: no double counting in state_dict
    model._illm_speculative = True
    model.n_drafted = 0
    model.n_matched = 0
    return model


class _AutoThreshold:
    """th_stop_draft auto-tuning: track the acceptance rate and move the
    threshold so that drafting stops where draft tokens start failing."""

    def __init__(self, th: float = 0.6, lo: float = 0.1, hi: float = 0.95):
        self.th, self.lo, self.hi = th, lo, hi

    def update(self, n_draft: int, n_acc: int):
        if n_draft == 0:
            return
        if n_acc == n_draft:
            self.th = max(self.lo, self.th - 0.05)
        elif n_acc < n_draft // 2:
            self.th = min(self.hi, self.th + 0.05)


@torch.no_grad()
def speculative_generate(model, prompts: Sequence[Sequence[int]], max_new_tokens: int = 32, eos_token_id=None,
                         timing=None, streamer=None, max_step_draft: int = 8, th_stop_draft: float = 0.6,
                         auto_th_stop_draft: bool = True, min_new_tokens: int = 0, use_graph: bool = True,
                         **_) -> List[List[int]]:
    from ..transformers.hf_native import get_native
    _, tgt = get_native(model)
    _, dft = get_native(model.draft_model)
    eos = set([eos_token_id] if isinstance(eos_token_id, int) else (eos_token_id or []))
    if tgt.model.device.type == "cuda" and use_graph:
        # device-resident rounds captured as hipGraphs (generation/spec_graph.py)
        from .spec_graph import GraphSpeculator, max_graph_draft
        kmax = max(1, min(max_step_draft, max_graph_draft(tgt.model)))
        outs = []
        for p in prompts:
            max_len = len(p) + max_new_tokens + 2 * kmax + 4
            sp = model.__dict__.get("_illm_spec_graph")
            if sp is None or sp.max_len < max_len or sp.k_max != kmax:
                sp = GraphSpeculator(tgt, dft, min(4, kmax), max(max_len, 1024), k_max=kmax,
                                     adaptive=auto_th_stop_draft)
                model.__dict__["_illm_spec_graph"] = sp
            outs.append(sp.generate(p, max_new_tokens, eos, timing=timing, streamer=streamer,
                                    min_new_tokens=min_new_tokens))
            model.n_drafted += sp.drafted
            model.n_matched += int(sp.n_match)
        if streamer is not None:
            streamer.end()                      # once per batch, as the eager path
        return outs
    sync = torch.cuda.synchronize if tgt.model.device.type == "cuda" else (lambda: None)
    thr = _AutoThreshold(th_stop_draft)
    outs = []
    for p in prompts:
        p = list(p)
        max_len = len(p) + max_new_tokens + max_step_draft + 16
        tgt._ensure_cache(1, max_len)
        dft._ensure_cache(1, max_len)
        st, sd = tgt.new_sequence(max_len), dft.new_sequence(max_len)
        t0 = time.perf_counter()
        last = int(torch.argmax(tgt.forward_chunk(st, p, 0)[-1]))
        dft.forward_chunk(sd, p, 0)
        out = p + [last]
        pending = [last]                      # committed tokens not yet in the draft cache
        sync()
        if timing is not None:
            timing.first_cost = time.perf_counter() - t0
        if streamer is not None:
            streamer.put(torch.tensor([last]))
        new = 1
        step_max = max_step_draft
        while new < max_new_tokens and not (last in eos and new >= min_new_tokens):
            t1 = time.perf_counter()
            # ---- draft: feed pending, then autoregress
            drafts: List[int] = []
            feed = pending
            budget = min(step_max, max_new_tokens - new - 1)
            while len(drafts) < budget:
                lg = dft.forward_chunk(sd, feed, sd.length)[-1].float()
                prob = torch.softmax(lg, -1)
                pmax, tok = prob.max(-1)
                drafts.append(int(tok))
                feed = [int(tok)]
                if auto_th_stop_draft and float(pmax) < thr.th:
                    break
            # draft cache now holds everything up to drafts[-2]
            # ---- verify with the target
            lg = tgt.forward_chunk(st, [last] + drafts, st.length)
            pred = torch.argmax(lg, -1).tolist()
            m = 0
            while m < len(drafts) and drafts[m] == pred[m]:
                m += 1
            accepted = drafts[:m] + [pred[m]]
            st.length -= len(drafts) - m
            # draft cache: valid through `last` + drafts[:m]; drafts[-1] was never fed
            if drafts:
                fed = len(drafts) - 1                    # drafts fed into the draft cache
                keep = min(m, fed)
                sd.length = st.length - (m - keep)
                pending = drafts[keep:m] + [pred[m]]
            else:                                        # nothing drafted: draft cache untouched
                pending = pending + [pred[m]]
            model.n_drafted += len(drafts)
            model.n_matched += m
            thr.update(len(drafts), m)
            if drafts:
                step_max = min(16, step_max + 1) if m == len(drafts) else max(2, step_max - 1)
            emitted = []
            stop = False
            for t in accepted:
                emitted.append(t)
                new += 1
                if (t in eos and new >= min_new_tokens) or new >= max_new_tokens:
                    stop = True
                    break
            out.extend(emitted)
            last = emitted[-1]
            sync()
            if timing is not None:
                dt = time.perf_counter() - t1
                timing.rest_costs.extend([dt / len(emitted)] * len(emitted))
            if streamer is not None:
                streamer.put(torch.tensor(emitted))
            if stop:
                break
        tgt.cache.allocator.release(st.blocks)
        dft.cache.allocator.release(sd.blocks)
        outs.append(out)
    if streamer is not None:
        streamer.end()
    return outs
