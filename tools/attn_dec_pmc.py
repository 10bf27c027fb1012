"""Decode attention at the Llama-3-8B shape (B sequences x L keys, fused RoPE
from an f32 qkv accumulator, then the combine) in a loop, for rocprofv3
--kernel-trace / --pmc passes (tools/pmc_attn_dec.sh).

usage: python tools/attn_dec_pmc.py [B] [L] [iters] [rope]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ipex_llm_amd import ops  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    rope = (sys.argv[4] if len(sys.argv) > 4 else "1") == "1"
    ops.require()
    dev = torch.device("cuda")
    Hq, Hkv, D, bs = 32, 8, 128, 64
    nb = (L + bs) // bs + 1
    kc = torch.randn(B * nb, Hkv, bs, D, device=dev, dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.arange(B * nb, device=dev, dtype=torch.int32).view(B, nb)
    seq = torch.full((B,), L, device=dev, dtype=torch.int32)
    pos = torch.full((B,), L - 1, device=dev, dtype=torch.long)
    cs = torch.randn(L + 64, D // 2, 2, device=dev)
    ns = (L + 63) // 64
    part = torch.randn(B, (Hq + 2 * Hkv) * D, device=dev)
    q = torch.randn(B, 1, Hq, D, device=dev, dtype=torch.bfloat16)
    for _ in range(iters):
        if rope:
            p = part.clone()
            ops.attn_decode_rope(p, None, cs, pos, kc, vc, bt, seq, ns, D ** -0.5, 0.0, 0, Hq, D, False)
        else:
            ops.attn_decode(q, kc, vc, bt, seq, ns, D ** -0.5)
    torch.cuda.synchronize()
    print("done", B, L, iters, rope)


if __name__ == "__main__":
    main()
