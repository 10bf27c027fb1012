"""Dense 8-phase GEMM probe (GPU box): the same launch with the operands'
row stride 0 (every A / B tile read from one row: L2-resident) vs normal
rows -- separates the global-memory part of the kernel's time from its
LDS / MFMA / barrier schedule.  One JSON line per case."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ipex_llm_amd import ops  # noqa: E402


def timed(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def shapes_only():
    """(--shapes) the four Llama-3-8B projections at M = 8192 / 1024 on the
    dense kernel (auto split-K), normal operands: one line per shape"""
    P = torch.ops.ipex_llm_amd
    dev = torch.device("cuda")
    for M in (8192, 1024):
        for name, N, K in [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)]:
            x = torch.randn(M, K, device=dev).bfloat16()
            w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
            us = timed(lambda: P.gemm_bf16(x, w))
            lib = timed(lambda: torch.nn.functional.linear(x, w))
            print(json.dumps({"gm": os.environ.get("ILLM_G8_GM", "4"), "M": M, "op": name, "us": round(us, 1),
                              "lib_us": round(lib, 1), "vs_lib": round(lib / us, 3),
                              "TF": round(2 * M * N * K / us / 1e6, 1)}), flush=True)


def main():
    ops.require()
    if "--shapes" in sys.argv:
        return shapes_only()
    P = torch.ops.ipex_llm_amd
    dev = torch.device("cuda")
    for M, N, K in [(8192, 28672, 4096), (8192, 4096, 4096)]:
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        x0 = x[:1].expand(M, K)
        w0 = w[:1].expand(N, K)
        fl = 2 * M * N * K
        for name, a, b in [("normal", x, w), ("x_row0", x0, w), ("w_row0", x, w0), ("both_row0", x0, w0)]:
            us = timed(lambda: P.gemm_bf16(a, b, None, False, 0, False, 0, 1))
            print(json.dumps({"M": M, "N": N, "K": K, "case": name, "us": round(us, 1),
                              "TF": round(fl / us / 1e6, 1)}), flush=True)
        z = torch.zeros_like(x)
        wz = torch.zeros_like(w)
        us = timed(lambda: P.gemm_bf16(z, wz, None, False, 0, False, 0, 1))
        print(json.dumps({"M": M, "N": N, "K": K, "case": "zeros", "us": round(us, 1), "TF": round(fl / us / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
