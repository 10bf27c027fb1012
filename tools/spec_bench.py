"""Self-speculative decoding latency on one MI355X (Llama-3-8B geometry,
random weights): bf16 target + sym_int4 draft, the device-resident round
captured as hipGraphs (generation/spec_graph.py), against plain hipGraph
decoding of the bf16 target and of the int4 model.

The target's weights are the dequantized draft weights (bf16), so the two
models agree like a real checkpoint and its INT4 copy do (the reference's
self-speculative setting, SRC/transformers/speculative.py); with independent
random weights the argmax of near-flat random logits would be noise.
One JSON line per configuration."""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--prompt", type=int, default=256)
    ap.add_argument("--new", type=int, default=128)
    ap.add_argument("--ks", default="1,2,3,4,6,4a", help="draft lengths; 'a' suffix = adaptive")
    ap.add_argument("--std", type=float, default=0.02, help="random-init weight std")
    ap.add_argument("--skip-plain", action="store_true", help="(profiling) no plain-decode baselines")
    args = ap.parse_args()
    from transformers import LlamaConfig
    from ipex_llm_amd.engine.runner import Engine, GenTiming
    from ipex_llm_amd.generation.spec_graph import GraphSpeculator
    from ipex_llm_amd.models.builder import dense_copy, random_native_model
    cfg = LlamaConfig(vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=args.layers,
                      num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=8192,
                      rope_theta=500000.0)
    dev = torch.device("cuda")
    draft = random_native_model(cfg, "sym_int4", dev, torch.bfloat16, seed=0, std=args.std)
    target = dense_copy(draft)
    torch.cuda.synchronize()
    prompt = torch.randint(0, 128256, (args.prompt,), generator=torch.Generator().manual_seed(1)).tolist()
    te, de = Engine(target), Engine(draft)

    def plain(eng, name):
        tm = GenTiming()
        out = eng.generate([prompt], max_new_tokens=args.new, use_graph=True, timing=tm)
        tm = GenTiming()
        out = eng.generate([prompt], max_new_tokens=args.new, use_graph=True, timing=tm)
        ms = tm.rest_cost_mean * 1e3
        print(json.dumps({"mode": name, "ms_per_token": round(ms, 3), "first_token_ms": round(tm.first_cost * 1e3, 2)}),
              flush=True)
        return out[0], ms

    if args.skip_plain:
        ref = te.generate([prompt], max_new_tokens=args.new, use_graph=True)[0]
        t_bf16 = t_int4 = float("nan")
    else:
        ref, t_bf16 = plain(te, "plain_bf16_target")
        _, t_int4 = plain(de, "plain_int4")
    max_len = args.prompt + args.new + 64
    cfgs = [(int(v.rstrip("a")), v.endswith("a")) for v in args.ks.split(",")]
    for k, adaptive in cfgs:
        sp = GraphSpeculator(te, de, k, max_len, k_max=8 if adaptive else k, adaptive=adaptive)
        sp.generate(prompt, args.new)                      # warm-up + capture
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = sp.generate(prompt, args.new)
        torch.cuda.synchronize()
        # decode part only: subtract the prefill of both models
        tm = GenTiming()
        sp.generate(prompt, args.new, timing=tm)
        ms = tm.rest_cost_mean * 1e3
        gen, gref = out[len(prompt):], ref[len(prompt):]          # generated tokens only
        agree = sum(int(a == b) for a, b in zip(gen, gref)) / max(1, len(gref))
        first_div = next((i for i, (a, b) in enumerate(zip(gen, gref)) if a != b), None)
        print(json.dumps({"mode": "speculative_graph", "k": k, "adaptive": adaptive, "ms_per_token": round(ms, 3),
                          "acceptance": round(sp.acceptance, 3), "tokens_per_round": round((len(out) - len(prompt) - 1)
                                                                                          / max(1, sp.rounds), 2),
                          "speedup_vs_bf16": round(t_bf16 / ms, 2), "vs_int4": round(t_int4 / ms, 2),
                          "generated_token_agreement": round(agree, 3), "first_divergence": first_div,
                          "wall_s_total": round(time.perf_counter() - t0, 3)}), flush=True)


if __name__ == "__main__":
    main()
