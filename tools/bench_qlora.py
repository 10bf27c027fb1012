#!/usr/bin/env python
"""QLoRA finetune throughput: Llama-3-8B with an NF4 base, bf16 LoRA adapters
and the fused multi-tensor AdamW kernel on one MI355X (BASELINE.json config
"Llama-3 8B QLoRA NF4 finetune on 1xMI355X").

Reference recipe (python/llm/example/GPU/LLM-Finetuning/QLoRA/alpaca-qlora):
BitsAndBytesConfig nf4 -> from_pretrained(load_in_low_bit="nf4",
optimize_model=False), lm_head kept in bf16, LoRA r=8 / alpha=16 on
q,k,v,o,gate,up,down, bf16 compute.  Here: random-init weights of the exact
Llama-3-8B architecture generated and NF4-quantized on the GPU layer by layer
(no checkpoint, no network), synthetic token batches.  One step = forward +
backward (low-bit GEMMs forward, dequant GEMM for grad_x) + fused AdamW.

    python tools/bench_qlora.py --batch 8 --seq 512 --steps 10 --warmup 3
Prints one JSON line (training tokens/s, ms/step, peak memory).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def llama3_8b_config(layers=None):
    from transformers import LlamaConfig
    cfg = LlamaConfig(
        vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
        num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=8192,
        rms_norm_eps=1e-5, tie_word_embeddings=False, rope_theta=500000.0)
    if layers:
        cfg.num_hidden_layers = layers
    return cfg


@torch.no_grad()
def random_qlora_base(cfg, qtype: str, dev, dtype=torch.bfloat16, seed: int = 0, std: float = 0.02):
    """HF LlamaForCausalLM built on meta, every decoder linear replaced by a
    LowBitLinear quantized on the GPU from random weights; lm_head, embeddings
    and norms dense in ``dtype`` (QLoRA leaves lm_head unquantized)."""
    from transformers import LlamaForCausalLM
    from transformers.models.llama.modeling_llama import LlamaRotaryEmbedding
    from ipex_llm_amd.transformers.low_bit_linear import LowBitLinear
    g = torch.Generator(device=dev).manual_seed(seed)
    with torch.device("meta"):
        model = LlamaForCausalLM(cfg)
    for layer in model.model.layers:
        for parent in (layer.self_attn, layer.mlp):
            for name, child in list(parent.named_children()):
                if isinstance(child, nn.Linear):
                    m = LowBitLinear(child.in_features, child.out_features, qtype, bias=False, device="meta")
                    w = torch.randn(child.out_features, child.in_features, generator=g, device=dev) * std
                    m.load_dense(w.to(dtype), device=dev)
                    del w
                    setattr(parent, name, m)
    model.model.embed_tokens = nn.Embedding(cfg.vocab_size, cfg.hidden_size, device=dev, dtype=dtype)
    model.model.embed_tokens.weight.normal_(0, std, generator=g)
    model.lm_head = nn.Linear(cfg.hidden_size, cfg.vocab_size, bias=False, device=dev, dtype=dtype)
    model.lm_head.weight.normal_(0, std, generator=g)
    for mod in model.modules():
        if mod.__class__.__name__.endswith("RMSNorm"):
            mod.weight = nn.Parameter(torch.ones(cfg.hidden_size, device=dev, dtype=dtype))
    model.model.rotary_emb = LlamaRotaryEmbedding(cfg, device=dev)
    for p in model.parameters():
        p.requires_grad_(False)
    return model


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--qtype", default="nf4")
    ap.add_argument("--rank", type=int, default=8)
    ap.add_argument("--grad-ckpt", action="store_true")
    ap.add_argument("--layers", type=int, default=None, help="debug only: fewer layers")
    ap.add_argument("--graph", action="store_true",
                    help="capture the whole training step (zero_grad, forward, backward, fused AdamW) in one "
                         "hipGraph and replay it")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    import ipex_llm_amd.ops as ops
    ops.require()
    from ipex_llm_amd.training import FusedAdamW, LoraConfig, get_peft_model
    cfg = llama3_8b_config(args.layers)
    t0 = time.perf_counter()
    model = random_qlora_base(cfg, args.qtype, dev)
    model.config.use_cache = False
    if os.environ.get("ILLM_TRAIN_NORM", "1") == "1":
        # optimize_model's norm patch: HIP RMSNorm forward + backward (frozen weight)
        from ipex_llm_amd.transformers.convert import _patch_norms
        _patch_norms(model)
    if os.environ.get("ILLM_TRAIN_ROPE", "1") == "1":
        from ipex_llm_amd.transformers.convert import _patch_rope
        _patch_rope(model)
    if os.environ.get("ILLM_TRAIN_MLP", "1") == "1":
        from ipex_llm_amd.transformers.convert import _patch_mlp
        _patch_mlp(model)
    # fused lm_head + CE and HIP flash attention fwd / bwd (ILLM_TRAIN_CE / ILLM_TRAIN_ATTN)
    from ipex_llm_amd.training.lora import enable_training_kernels
    enable_training_kernels(model)
    if args.grad_ckpt:
        model.gradient_checkpointing_enable()
        model.enable_input_require_grads()
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    lcfg = LoraConfig(r=args.rank, lora_alpha=2 * args.rank,
                      target_modules=["q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj"])
    pm = get_peft_model(model, lcfg)
    pm.train()
    params = [p for p in pm.parameters() if p.requires_grad]
    n_train = sum(p.numel() for p in params)
    opt = FusedAdamW(params, lr=2e-4, weight_decay=0.0, capturable=args.graph)
    gen = torch.Generator(device=dev).manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (args.batch, args.seq), device=dev, generator=gen)

    def step():
        if args.graph:
            # gradients stay allocated (stable addresses for the captured
            # optimizer's pointer table) and are zeroed inside the step
            opt.zero_grad(set_to_none=False)
        loss = pm(input_ids=ids, labels=ids).loss
        loss.backward()
        opt.step()
        if not args.graph:
            opt.zero_grad(set_to_none=True)
        return loss

    losses = []
    if args.graph:
        # warm up on a side stream (lazy library / autograd state), then
        # capture one step; every timed step is one graph replay
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(2, args.warmup)):
                losses.append(step().item())
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            static_loss = step()
        graph.replay()
        losses.append(static_loss.item())

        def step():  # noqa: F811
            graph.replay()
            return static_loss
    else:
        for _ in range(args.warmup):
            losses.append(step().item())
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    losses.append(loss.item())
    tok = args.batch * args.seq * args.steps
    print(json.dumps({
        "metric": "QLoRA finetune training tokens/s, Llama-3-8B NF4 base + bf16 LoRA, 1x MI355X",
        "value": round(tok / dt, 1), "unit": "tokens/s", "ms_per_step": round(dt / args.steps * 1e3, 1),
        "steps": args.steps, "warmup": args.warmup, "dtype": "bf16", "qtype": args.qtype,
        "data": "synthetic token batches, random-init Llama-3-8B architecture",
        "config": {"model": "Llama-3-8B" if not args.layers else f"Llama-3-8B[{args.layers} layers]",
                   "batch": args.batch, "seq_len": args.seq, "lora_r": args.rank,
                   "targets": "q,k,v,o,gate,up,down", "grad_ckpt": args.grad_ckpt, "optimizer": "FusedAdamW",
                   "hipgraph": args.graph, "dense_base_cache_gb": getattr(model, "_illm_train_dense_gb", 0.0)},
        "trainable_params": n_train, "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 1),
        "build_s": round(build_s, 1), "loss_first": round(losses[0], 4), "loss_last": round(losses[-1], 4),
    }), flush=True)


if __name__ == "__main__":
    main()
