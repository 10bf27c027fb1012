"""Run one prefill low-bit GEMM shape in a loop (for rocprofv3 --pmc passes).

usage: python tools/gemm_pmc.py [op] [M] [iters]   op in qkv|o|gate_up|down
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ipex_llm_amd import ops  # noqa: E402
from ipex_llm_amd.quantize import get_format  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def main():
    op = sys.argv[1] if len(sys.argv) > 1 else "gate_up"
    M = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    ops.require()
    f = get_format("sym_int4").fmt
    n, k = SHAPES[op]
    dev = torch.device("cuda")
    b = ops.quantize(torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02, f)
    x = torch.randn(M, k, device=dev, dtype=torch.bfloat16)
    for _ in range(iters):
        torch.ops.ipex_llm_amd.gemm(x, b, f, n, k, None)
    torch.cuda.synchronize()
    print("done", op, M, iters)


if __name__ == "__main__":
    main()
