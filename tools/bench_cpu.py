#!/usr/bin/env python
"""CPU decode benchmark: Llama-2-7B at sym_int4 (load_in_4bit), greedy, on
the host CPU only (BASELINE.json config "Llama-2 7B INT4 load_in_4bit greedy
decode on CPU").

Reference harness semantics (dev/benchmark/all-in-one/run.py): in/out 32-32,
"1st token avg latency" = prefill + first token, "2+ avg latency" = mean of the
remaining steps, averaged over trials after a warm-up.  Random-init weights of
the exact Llama-2-7B architecture are generated and quantized layer by layer
by the C++ host quantizer (no checkpoint, no network); the projections run on
the int8-activation integer-dot kernels of csrc/cpu/gemm_q4.cpp (AVX-512 VNNI
or AVX2 picked at run time).

    python tools/bench_cpu.py [--in-len 32 --out-len 32 --trials 2 --layers N]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def llama2_7b_config(layers=None):
    from transformers import LlamaConfig
    cfg = LlamaConfig(vocab_size=32000, hidden_size=4096, intermediate_size=11008, num_hidden_layers=32,
                      num_attention_heads=32, num_key_value_heads=32, max_position_embeddings=4096,
                      rms_norm_eps=1e-5, tie_word_embeddings=False)
    if layers:
        cfg.num_hidden_layers = layers
    return cfg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--in-len", type=int, default=32)
    ap.add_argument("--out-len", type=int, default=32)
    ap.add_argument("--trials", type=int, default=2)
    ap.add_argument("--qtype", default="sym_int4")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--layers", type=int, default=None, help="debug only: fewer layers")
    args = ap.parse_args()
    if args.threads:
        torch.set_num_threads(args.threads)
    import ipex_llm_amd.ops as ops
    ops.require()
    from ipex_llm_amd.engine.runner import Engine, GenTiming
    from ipex_llm_amd.models.builder import random_native_model
    cfg = llama2_7b_config(args.layers)
    t0 = time.perf_counter()
    model = random_native_model(cfg, args.qtype, "cpu", torch.float32, seed=0)
    build_s = time.perf_counter() - t0
    eng = Engine(model)
    prompt = torch.randint(3, cfg.vocab_size, (args.in_len,), generator=torch.Generator().manual_seed(1)).tolist()
    first, rest = [], []
    for trial in range(args.trials + 1):       # trial 0 = warm-up
        tm = GenTiming()
        eng.generate([prompt], max_new_tokens=args.out_len, min_new_tokens=args.out_len, use_graph=False,
                     timing=tm)
        if trial:
            first.append(tm.first_cost * 1e3)
            rest.append(tm.rest_cost_mean * 1e3)
    ms = sum(rest) / len(rest)
    print(json.dumps({
        "metric": "decode tokens/s + first-token latency, Llama-2-7B INT4 on CPU",
        "value": round(1e3 / ms, 2), "unit": "tokens/s", "decode_ms_per_token": round(ms, 1),
        "first_token_latency_ms": round(sum(first) / len(first), 1), "in_out": f"{args.in_len}-{args.out_len}",
        "qtype": args.qtype, "threads": torch.get_num_threads(), "dtype": "fp32 activations (int8 dot)",
        "data": "synthetic prompt, random-init Llama-2-7B architecture",
        "config": {"model": "Llama-2-7B" if not args.layers else f"Llama-2-7B[{args.layers} layers]",
                   "batch": 1, "device": "cpu"},
        "build_s": round(build_s, 1),
    }), flush=True)


if __name__ == "__main__":
    main()
