#!/usr/bin/env python
"""Serving benchmark mirroring the reference's published vLLM number
(docs/mddocs/DockerGuides/vllm_docker_quickstart.md:231-249: Qwen2.5-7B-Instruct,
1 request, 1024 input / 512 output tokens -> output token throughput 30.01
tok/s, mean TTFT 520.10 ms, mean TPOT 32.37 ms on Intel Arc).

Here the continuous-batching LLMEngine (C++ scheduler, paged KV, hipGraph
decode) serves random-init weights of the Qwen2.5-7B architecture on one
MI355X.  --concurrency N submits N such requests at once (throughput mode).

    python tools/bench_serving.py [--qtype sym_int4|fp8] [--concurrency 1]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def qwen25_7b_config():
    from transformers import Qwen2Config
    return Qwen2Config(vocab_size=152064, hidden_size=3584, intermediate_size=18944, num_hidden_layers=28,
                       num_attention_heads=28, num_key_value_heads=4, max_position_embeddings=32768,
                       rms_norm_eps=1e-6, rope_theta=1000000.0, tie_word_embeddings=False)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qtype", default="sym_int4")
    ap.add_argument("--input-len", type=int, default=1024)
    ap.add_argument("--output-len", type=int, default=512)
    ap.add_argument("--concurrency", type=int, default=1)
    ap.add_argument("--no-graph", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    import ipex_llm_amd.ops as ops
    ops.require()
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.serving.engine import LLMEngine, SamplingParams
    cfg = qwen25_7b_config()
    model = random_native_model(cfg, args.qtype, dev, torch.bfloat16, seed=0)
    eng = LLMEngine(model, max_batch=max(8, args.concurrency), max_model_len=args.input_len + args.output_len + 64,
                    use_graph=not args.no_graph)
    g = torch.Generator().manual_seed(0)
    params = SamplingParams(max_new_tokens=args.output_len, min_new_tokens=args.output_len)

    def run(n):
        prompts = [torch.randint(0, cfg.vocab_size, (args.input_len,), generator=g).tolist() for _ in range(n)]
        stamps = {}

        def on_tok(tok, r):
            if tok >= 0:
                stamps.setdefault(r.rid, []).append(time.perf_counter())
        t0 = time.perf_counter()
        rids = [eng.add_request(p, params, on_token=on_tok) for p in prompts]
        while eng.has_work():
            eng.step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ttft = [stamps[r][0] - t0 for r in rids]
        itl = [b - a for r in rids for a, b in zip(stamps[r][:-1], stamps[r][1:])]
        tpot = [(stamps[r][-1] - stamps[r][0]) / max(1, len(stamps[r]) - 1) for r in rids]
        for r in rids:
            eng.requests.pop(r, None)
        return t1 - t0, ttft, itl, tpot, sum(len(stamps[r]) for r in rids)

    run(1)                                                   # warm-up (graph capture)
    dur, ttft, itl, tpot, ntok = run(args.concurrency)
    itl_sorted = sorted(itl)
    mean = lambda v: sum(v) / len(v)                         # noqa: E731
    out = {
        "metric": "serving output token throughput (1024 in / 512 out), Qwen2.5-7B",
        "value": round(ntok / dur, 2), "unit": "tokens/s", "higher_is_better": True,
        "total_token_throughput": round((ntok + args.concurrency * args.input_len) / dur, 2),
        "mean_ttft_ms": round(mean(ttft) * 1e3, 2), "mean_tpot_ms": round(mean(tpot) * 1e3, 3),
        "mean_itl_ms": round(mean(itl) * 1e3, 3), "p99_itl_ms": round(itl_sorted[int(0.99 * (len(itl) - 1))] * 1e3, 3),
        "concurrency": args.concurrency, "qtype": args.qtype, "hipgraph": not args.no_graph, "dtype": "bf16",
        "data": "synthetic prompts, random-init Qwen2.5-7B architecture",
        "baseline": {"value": 30.01, "ttft_ms": 520.10, "tpot_ms": 32.37,
                     "source": "vllm_docker_quickstart.md:231-249 (Intel Arc, ipex-llm vLLM, fp8)"},
    }
    out["vs_baseline"] = round(out["value"] / 30.01, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
