"""Run one decode GEMV shape in a loop (for rocprofv3 --pmc passes).

usage: python tools/gemv_pmc.py [op] [M] [iters]   op in qkv|o|gate_up|glu|down|lm_head
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ipex_llm_amd import ops  # noqa: E402
from ipex_llm_amd.quantize import get_format  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "glu": (28672, 4096),
          "down": (4096, 14336), "lm_head": (128256, 4096)}


def main():
    op = sys.argv[1] if len(sys.argv) > 1 else "glu"
    M = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    ops.require()
    f = get_format("sym_int4").fmt
    n, k = SHAPES[op]
    dev = torch.device("cuda")
    copies = max(1, int(math.ceil(600e6 / (n * k * 0.5))))
    blobs = [ops.quantize(torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02, f) for _ in range(copies)]
    x = torch.randn(M, k, device=dev, dtype=torch.bfloat16)
    for i in range(iters):
        b = blobs[i % copies]
        if op == "glu":
            ops.gemv_glu(x, b, f, n, k, 0)
        else:
            ops.gemv_partials(x, b, f, n, k, 0)
    torch.cuda.synchronize()
    print("done", op, M, iters)


if __name__ == "__main__":
    main()
