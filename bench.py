#!/usr/bin/env python
"""Headline benchmark: Llama-3-8B INT4 (sym_int4) decode tokens/s + first-token
latency on N MI355X GPUs (BASELINE.json metric).

One process per GPU (torchrun).  Default: each rank serves its own replica
(data-parallel serving, weak scaling: fixed batch per GPU).  ``--tp``: ONE
model sharded over all ranks (AutoTP, reference
``example/GPU/Deepspeed-AutoTP/deepspeed_autotp.py:81-106``), the native
hipGraph decoder all-reduces every row-parallel projection's f32 accumulator
over RCCL / the custom xGMI all-reduce (strong scaling: fixed global batch).
``--ep``: expert parallel, token-sharded (Mixtral-8x7B, BASELINE config 3):
rank r keeps experts [r E/W, (r+1) E/W) and serves ITS OWN batch of
sequences (attention data-parallel, weak scaling); every MoE block sends each
(token, expert) pair to its expert's owner and back through the HIP peer
all-to-all over xGMI (parallel/ep.py EPAllToAll: exactly T*k rows per rank
per direction, device-side counts, captured in the decode hipGraph).
Random-init weights of the exact architecture are generated and quantized on
the GPU (identical on every rank for TP/EP), a synthetic prompt batch is
prefilled (first-token latency), then decode steps are replayed from one
captured hipGraph.  W
untimed warmup steps, then EXACTLY K timed decode steps bracketed by barrier
+ synchronize; the slowest rank's time is reported.  Every timed step runs
the full model (all layers + lm_head + argmax) for the whole batch.
With N > 1 in the default data-parallel mode the same model is also run
tensor-parallel over all N ranks (fixed global batch) and reported as the
``tp_side`` field of the one JSON line (``--no-tp-side`` skips it).

    python bench.py --gpus 1 --steps 64 --warmup 8
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8 --model llama3-70b --tp
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8 --model mixtral-8x7b --ep
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

# reference's closest published single-request 7B-class decode number:
# vLLM output token throughput, Qwen2.5-7B, 1 request, 1024 in / 512 out,
# Intel Arc (docs/mddocs/DockerGuides/vllm_docker_quickstart.md:236)
BASELINE_TOK_S = 30.01


def llama3_8b_config():
    from transformers import LlamaConfig
    return LlamaConfig(
        vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
        num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=131072,
        rms_norm_eps=1e-5, tie_word_embeddings=False,
        rope_parameters={"rope_type": "llama3", "rope_theta": 500000.0, "factor": 8.0,
                         "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                         "original_max_position_embeddings": 8192},
    )


def llama3_70b_config():
    cfg = llama3_8b_config()
    cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers = 8192, 28672, 80
    cfg.num_attention_heads, cfg.num_key_value_heads = 64, 8
    return cfg


def mixtral_8x7b_config():
    from transformers import MixtralConfig
    return MixtralConfig(vocab_size=32000, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                         num_attention_heads=32, num_key_value_heads=8, num_local_experts=8, num_experts_per_tok=2,
                         max_position_embeddings=32768, rms_norm_eps=1e-5, rope_theta=1e6, sliding_window=None)


def qwen25_7b_config():
    from transformers import Qwen2Config
    return Qwen2Config(vocab_size=152064, hidden_size=3584, intermediate_size=18944, num_hidden_layers=28,
                       num_attention_heads=28, num_key_value_heads=4, max_position_embeddings=32768,
                       rms_norm_eps=1e-6, rope_theta=1000000.0, tie_word_embeddings=False)


# --model: the headline is Llama-3-8B (BASELINE.json); the others are the
# BASELINE configs' models measured on ONE MI355X (70B INT4 fits in 288 GB;
# Mixtral runs the grouped MoE GEMV) and the reference's serving model
MODELS = {"llama3-8b": ("Llama-3-8B", llama3_8b_config), "llama3-70b": ("Llama-3-70B", llama3_70b_config),
          "mixtral-8x7b": ("Mixtral-8x7B", mixtral_8x7b_config), "qwen2.5-7b": ("Qwen2.5-7B", qwen25_7b_config)}


def measure(model, eng, args, prompts, dev, world, rank):
    """first-token latency (1 warm-up + 3 trials of the batched prefill) and
    K timed decode steps after W warm-up steps, slowest rank; returns
    (ms per step, first-token ms, next ids, prefill graph used)"""
    from ipex_llm_amd.models.cache import SequenceState
    B = prompts.shape[0]
    max_len = args.prompt_len + args.warmup + args.steps + 8
    eng._ensure_cache(B, max_len)

    def barrier():
        if world > 1:
            dist.barrier()

    nblk = (max_len + eng.block_size - 1) // eng.block_size
    barrier()                                    # EP: the MoE exchanges need every rank in step
    ftl = []
    pf_graph = not (args.no_graph or args.no_prefill_graph) and eng._pf_graph_ok()
    for trial in range(4):
        eng.cache.allocator = type(eng.cache.allocator)(eng.cache.num_blocks)
        seqs = [SequenceState(eng.cache.allocator.alloc(nblk)) for _ in range(B)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        # one batched prefill of the B prompts (projections as [B*P, K] GEMMs)
        cur = torch.argmax(eng.prefill_batch(seqs, prompts, use_graph=pf_graph), -1)
        torch.cuda.synchronize()
        if trial:
            ftl.append((time.perf_counter() - t0) * 1e3)

    # ---- decode: graph-captured step, W warmup + K timed
    st = eng.decode_step_obj(seqs, max_len, greedy=True, use_graph=not args.no_graph)
    st.set_state(cur, torch.tensor([s.length for s in seqs], device=dev))
    for _ in range(args.warmup):
        st.step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        st.step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tok = st.next_ids.clone()
    t = torch.tensor([dt, sum(ftl) / len(ftl)], dtype=torch.float64)
    if world > 1:
        if dist.get_backend() == "nccl":
            t = t.to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt, ftl_ms = t.tolist()
    return dt / args.steps * 1e3, ftl_ms, tok, pf_graph


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b", choices=sorted(MODELS))
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("BENCH_BATCH", "8")))
    ap.add_argument("--prompt-len", type=int, default=1024)
    ap.add_argument("--qtype", default="sym_int4")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-prefill-graph", action="store_true",
                    help="eager prefill (default: the batched prefill is captured once per shape as a hipGraph "
                         "in the untimed first trial and replayed)")
    ap.add_argument("--layers", type=int, default=None, help="debug only: fewer layers (invalid for the metric)")
    ap.add_argument("--tp", action="store_true", help="tensor parallel over all ranks (AutoTP)")
    ap.add_argument("--ep", action="store_true", help="expert parallel over all ranks (MoE models)")
    ap.add_argument("--no-tp-side", action="store_true",
                    help="N > 1 data-parallel run: skip the tensor-parallel (strong-scaling) side measurement")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # code-path smoke only (tests/test_gpu_bench_dist.py): every rank on cuda:0,
    # gloo rendezvous, the peer all-reduce / all-to-all forced over it
    shared = os.environ.get("BENCH_SHARED_GPU") == "1"
    if shared:
        local = 0
        os.environ.setdefault("ILLM_AR_P2P", "force")
        os.environ.setdefault("ILLM_EP_P2P", "force")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if shared:
            dist.init_process_group("gloo")
            chk = torch.ones(1)
        else:
            dist.init_process_group("nccl", device_id=dev)
            chk = torch.ones(1, device=dev)
        # the collective backend really spans the job: a sum of ones
        dist.all_reduce(chk)
        assert int(chk.item()) == world, f"world {int(chk.item())} != WORLD_SIZE {world}"

    import ipex_llm_amd.ops as ops
    ops.require()
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.engine.runner import Engine

    mname, mcfg = MODELS[args.model]
    cfg = mcfg()
    if args.layers:
        cfg.num_hidden_layers = args.layers
    sharded = world > 1 and (args.tp or args.ep)
    if args.ep and not getattr(cfg, "num_local_experts", None):
        raise SystemExit("--ep needs an MoE model (e.g. --model mixtral-8x7b)")
    group = dist.group.WORLD if sharded else None
    if sharded and args.tp:
        from ipex_llm_amd.parallel.comm import setup_custom_all_reduce
        setup_custom_all_reduce(group)
    B, P = args.batch, args.prompt_len
    t_build = time.perf_counter()
    # TP / EP: the same weights on every rank (one seed), each keeps its shard
    model = random_native_model(cfg, args.qtype, dev, torch.bfloat16, seed=1234 + (0 if sharded else rank),
                                tp_group=group if args.tp else None, ep_group=group if args.ep else None,
                                ep_tokens=bool(args.ep), ep_max_tokens=B * P)
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t_build
    eng = Engine(model)
    same_tokens = sharded and args.tp            # TP: one batch; DP / token-sharded EP: a batch per rank
    g = torch.Generator().manual_seed(7 + (0 if same_tokens else rank))
    prompts = torch.randint(0, cfg.vocab_size, (B, P), generator=g)
    ms_step, ftl_ms, tok, pf_graph = measure(model, eng, args, prompts, dev, world, rank)
    dense_gb = eng.prefill_dense_gb

    # N > 1 data-parallel: the same model tensor-parallel over all ranks as a
    # side result (strong scaling, fixed global batch B): the replicas above
    # never cross xGMI, this run all-reduces every row-parallel projection over
    # the custom peer all-reduce / RCCL inside the captured decode graph
    tp_side = None
    if world > 1 and not sharded and not args.no_tp_side and world <= 8 \
            and cfg.num_attention_heads % world == 0 and cfg.num_key_value_heads % world == 0:
        del eng, model
        torch.cuda.empty_cache()
        from ipex_llm_amd.parallel.comm import setup_custom_all_reduce
        wg = dist.group.WORLD
        setup_custom_all_reduce(wg)
        tp_model = random_native_model(cfg, args.qtype, dev, torch.bfloat16, seed=1234, tp_group=wg)
        tp_eng = Engine(tp_model)
        tp_prompts = torch.randint(0, cfg.vocab_size, (B, P), generator=torch.Generator().manual_seed(7))
        t_ms, t_ftl, _, _ = measure(tp_model, tp_eng, args, tp_prompts, dev, world, rank)
        tp_side = {"parallelism": f"tp{world}", "scaling": "strong", "global_batch": B,
                   "value": round(B * 1e3 / t_ms, 2), "unit": "tokens/s", "ms_per_step": round(t_ms, 4),
                   "first_token_latency_ms": round(t_ftl, 2)}

    replicas = 1 if same_tokens else world
    value = B * replicas * 1e3 / ms_step
    if rank == 0:
        out = {
            "metric": f"decode tokens/sec + first-token latency, {mname} INT4 at 1/2/4/8 MI355X",
            "value": round(value, 2), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "strong" if same_tokens else "weak",
            # BASELINE.json publishes no value for this metric/config (its
            # charts are off-repo images): no ratio is claimed
            "vs_baseline": None, "dtype": "bf16",
            "data": f"synthetic (random prompt ids, random-init weights of the {mname} architecture)",
            "config": {"model": mname, "qtype": args.qtype, "global_batch": B * replicas,
                       "batch_per_gpu": B if not same_tokens else B / world, "seq_len": P,
                       "parallelism": f"tp{world}" if args.tp else (f"ep{world}" if args.ep else f"dp{world}"),
                       "hipgraph": not args.no_graph, "prefill_hipgraph": pf_graph,
                       "prefill_dense_shadow_gb": dense_gb,
                       "layers": cfg.num_hidden_layers},
            "first_token_latency_ms": round(ftl_ms, 2),
            "decode_ms_per_token": round(ms_step, 4),
            "per_sequence_tokens_per_s": round(1e3 / ms_step, 2),
            # the reference's closest published number is a different metric
            # (single-request vLLM serving throughput of a 7B model on Arc);
            # like-for-like serving comparison: tools/bench_serving.py
            "closest_reference": {"value": BASELINE_TOK_S, "unit": "output tokens/s per request",
                                  "source": "vllm_docker_quickstart.md:236 (Qwen2.5-7B, 1 request, Intel Arc)",
                                  "ours_per_sequence_tokens_per_s": round(1e3 / ms_step, 2)},
            "build_s": round(t_build, 1), "sample_next_ids": tok[:4].tolist(),
        }
        if tp_side is not None:
            out["tp_side"] = tp_side
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()

if __name__ == "__main__":
    main()
