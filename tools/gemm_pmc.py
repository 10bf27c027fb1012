"""Run one prefill low-bit GEMM shape in a loop (for rocprofv3 --pmc passes).

usage: python tools/gemm_pmc.py [op] [M] [iters] [impl]   op in qkv|o|gate_up|down
  impl: fused (ops.gemm, default) | g8 (8-phase low-bit) | g8dense (8-phase on
  the dequantized weight)
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
    impl = sys.argv[4] if len(sys.argv) > 4 else "fused"
    P = torch.ops.ipex_llm_amd
    wd = P.dequantize_device(b, f, n, k, torch.bfloat16) if impl == "g8dense" else None
    for _ in range(iters):
        if impl == "g8":
            P.gemm8p_lowbit(x, b, f, n, k, None)
        elif impl == "g8dense":
            P.gemm_bf16(x, wd)
        else:
            P.gemm(x, b, f, n, k, None)
    torch.cuda.synchronize()
    print("done", op, M, iters)


if __name__ == "__main__":
    main()
