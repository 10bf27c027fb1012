"""Run the prefill flash-attention kernel in a loop (rocprofv3 --pmc passes).

usage: python tools/attn_pmc.py [T] [iters]   (B=1, Llama-3-8B heads, paged cache)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ipex_llm_amd import ops  # noqa: E402


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    ops.require()
    dev = torch.device("cuda")
    Hq, Hkv, D, bs = 32, 8, 128, 64
    nblk = T // bs
    kc = torch.randn(nblk, Hkv, bs, D, device=dev, dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.arange(nblk, device=dev, dtype=torch.int32).view(1, -1)
    seq = torch.full((1,), T, device=dev, dtype=torch.int32)
    q = torch.randn(T, Hq, D, device=dev, dtype=torch.bfloat16)
    for _ in range(iters):
        ops.attn_prefill(q, kc, vc, bt, seq, T, D ** -0.5)
    torch.cuda.synchronize()
    print("done", T, iters)


if __name__ == "__main__":
    main()
