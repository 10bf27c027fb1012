"""Decode attention at the Llama-3-8B shape, timed per layer call from cold
caches: 32 layers of paged KV (B sequences x L keys each) are visited in turn,
as one decode step does, so no layer's 4-34 MB of KV is still in the 256 MB
Infinity Cache when it is read again.  Fused-RoPE path (f32 qkv accumulator,
pre-rotated, as the decoder runs it at batch <= 8) and the plain path.

The kernel variant comes from the environment (read once per process):
ILLM_ATTN_V3=0 (v2), ILLM_ATTN_V3_NW=2/4/8, ILLM_ATTN_V3_FUSE=1.

usage: python tools/bench_attn_dec.py [B] [L] [iters] [layers]  -> one JSON line
(layers = 1: the same KV every call, i.e. Infinity-Cache resident)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ipex_llm_amd import ops  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 1025
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    ops.require()
    dev = torch.device("cuda")
    NL = int(sys.argv[4]) if len(sys.argv) > 4 else 32
    Hq, Hkv, D, bs = 32, 8, 128, 64
    nb = (L + bs - 1) // bs
    ns = (L + 63) // 64
    layers = []
    for _ in range(NL):
        kc = torch.randn(B * nb, Hkv, bs, D, device=dev, dtype=torch.bfloat16)
        layers.append((kc, torch.randn_like(kc)))
    bt = torch.randperm(B * nb, device=dev).to(torch.int32).view(B, nb)
    seq = torch.full((B,), L, device=dev, dtype=torch.int32)
    pos = torch.full((B,), L - 1, device=dev, dtype=torch.long)
    cs = torch.randn(L + 64, D // 2, 2, device=dev)
    part = torch.zeros(B, (Hq + 2 * Hkv) * D, device=dev)
    q = torch.randn(B, 1, Hq, D, device=dev, dtype=torch.bfloat16)
    res = {"B": B, "L": L, "layers": NL, "v3": os.environ.get("ILLM_ATTN_V3", "1"), "nw": os.environ.get("ILLM_ATTN_V3_NW", "auto"),
           "fuse": os.environ.get("ILLM_ATTN_V3_FUSE", "0")}
    for rope in (True, False):
        def run():
            for li in range(32):
                kc, vc = layers[li % NL]
                if rope:
                    ops.attn_decode_rope(part, None, cs, pos, kc, vc, bt, seq, ns, D ** -0.5, 0.0, 0, Hq, D, False,
                                         prerot=True)
                else:
                    ops.attn_decode(q, kc, vc, bt, seq, ns, D ** -0.5)
        for _ in range(3):
            run()
        # capture one step of 32 layer calls (the decoder replays graphs)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            run()
            with torch.cuda.graph(g, stream=s):
                run()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        res["rope_us" if rope else "plain_us"] = round(e0.elapsed_time(e1) * 1000 / (iters * 32), 2)
    kv_mb = B * Hkv * L * D * 2 * 2 / 1e6
    res["kv_MB"] = round(kv_mb, 1)
    res["rope_TBps"] = round(kv_mb / res["rope_us"], 2)      # MB / us = TB/s
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
