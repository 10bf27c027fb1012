#!/usr/bin/env python
"""Automatic-prefix-caching demo of the reference, measured on MI355X
(docs/mddocs/DockerGuides/vllm_docker_quickstart.md:560-616: Llama-2-7b-chat,
fp8 weights, max_model_len 2000, a ~1860-token table prompt queried twice with
different questions, 16 output tokens: 21.97 s -> 0.97 s, input 84.57 ->
1929.67 tok/s on Intel Arc with APC on).

Random-init weights of the Llama-2-7B architecture; the "table" is random
token ids of the same length.  Both queries go through the serving LLMEngine
(C++ scheduler with content-hashed KV blocks); the second one prefills only
its question tokens.

    python tools/bench_prefix_cache.py [--qtype fp8|sym_int4] [--no-prefix-caching]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def llama2_7b_config():
    from transformers import LlamaConfig
    return LlamaConfig(vocab_size=32000, hidden_size=4096, intermediate_size=11008, num_hidden_layers=32,
                       num_attention_heads=32, num_key_value_heads=32, max_position_embeddings=4096,
                       rms_norm_eps=1e-5, tie_word_embeddings=False)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qtype", default="fp8")
    ap.add_argument("--table-len", type=int, default=1858)
    ap.add_argument("--question-len", type=int, default=24)
    ap.add_argument("--output-len", type=int, default=16)
    ap.add_argument("--no-prefix-caching", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    import ipex_llm_amd.ops as ops
    ops.require()
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.serving.engine import LLMEngine, SamplingParams
    cfg = llama2_7b_config()
    model = random_native_model(cfg, args.qtype, dev, torch.bfloat16, seed=0)
    eng = LLMEngine(model, max_batch=8, max_model_len=2000 + 64, enable_prefix_caching=not args.no_prefix_caching)
    g = torch.Generator().manual_seed(0)
    rnd = lambda n: torch.randint(3, cfg.vocab_size, (n,), generator=g).tolist()   # noqa: E731
    params = SamplingParams(max_new_tokens=args.output_len, min_new_tokens=args.output_len)
    eng.generate([rnd(args.table_len + args.question_len)], params)     # warm-up: kernels, graphs (other prefix)
    table = rnd(args.table_len)
    res = []
    for q in range(2):
        prompt = table + rnd(args.question_len)
        hits0 = eng.stats["prefix_hit_tokens"]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.generate([prompt], params)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res.append({"query": q, "generation_time_s": round(dt, 4),
                    "input_tok_s": round(len(prompt) / dt, 1), "output_tok_s": round(args.output_len / dt, 1),
                    "prefix_hit_tokens": eng.stats["prefix_hit_tokens"] - hits0})
    print(json.dumps({
        "metric": "automatic prefix caching: generation time of a repeated long-table query",
        "value": res[1]["generation_time_s"], "unit": "s", "higher_is_better": False,
        "first_query": res[0], "second_query": res[1], "prefix_caching": not args.no_prefix_caching,
        "model": "Llama-2-7B", "qtype": args.qtype, "dtype": "bf16",
        "data": "synthetic table/question ids, random-init Llama-2-7B architecture",
        "baseline": {"first_s": 21.97, "second_s": 0.97, "input_tok_s": [84.57, 1929.67],
                     "source": "vllm_docker_quickstart.md:606-615 (Intel Arc, fp8, APC on)"},
    }), flush=True)


if __name__ == "__main__":
    main()
