"""Prefill GEMM micro-bench (GPU box): fused low-bit MFMA GEMM vs dequantize
+ library GEMM at Llama-3-8B shapes, M tokens."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ipex_llm_amd import ops  # noqa: E402
from ipex_llm_amd.quantize import get_format  # noqa: E402


def t(fn, it=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main():
    ops.require()
    dev = torch.device("cuda")
    for qt in (sys.argv[1] if len(sys.argv) > 1 else "sym_int4").split(","):
        f = get_format(qt).fmt
        for M in [int(v) for v in os.environ.get("GEMM_M", "1024,4096").split(",")]:
            for name, n, k in [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)]:
                w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02
                blob = ops.quantize(w, f)
                x = torch.randn(M, k, device=dev, dtype=torch.bfloat16)
                fused = t(lambda: torch.ops.ipex_llm_amd.gemm(x, blob, f, n, k, None))
                lib = t(lambda: F.linear(x, torch.ops.ipex_llm_amd.dequantize_device(blob, f, n, k, x.dtype)))
                y1 = torch.ops.ipex_llm_amd.gemm(x, blob, f, n, k, None).float()
                y2 = F.linear(x, torch.ops.ipex_llm_amd.dequantize_device(blob, f, n, k, x.dtype)).float()
                rel = ((y1 - y2).norm() / y2.norm()).item()
                fl = 2 * M * n * k
                print(json.dumps({"qtype": qt, "M": M, "op": name, "fused_us": round(fused, 1), "lib_us": round(lib, 1),
                                  "fused_TF": round(fl / fused / 1e6, 1), "lib_TF": round(fl / lib / 1e6, 1),
                                  "rel_diff": rel}), flush=True)


if __name__ == "__main__":
    main()
