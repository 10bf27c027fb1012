"""8-phase dense bf16 GEMM (gemm_8p.hip) vs hipBLASLt (F.linear) at the
Llama-3-8B projection shapes; random operands (never zero-filled: DVFS).
One JSON line per (M, op).  Env GEMM_M (comma list)."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ipex_llm_amd import ops  # noqa: E402


def timeit(fn, it=30):
    for _ in range(5):
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
    shapes = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336),
              ("lm_head", 128256, 4096)]
    qtypes = os.environ.get("GEMM_Q", "dense").split(",")
    for qt in qtypes:
      for M in [int(v) for v in os.environ.get("GEMM_M", "1024,4096,8192").split(",")]:
        for name, n, k in shapes:
            if qt != "dense":
                if name == "lm_head":
                    continue
                from ipex_llm_amd.quantize import get_format
                f = get_format(qt).fmt
                x = torch.randn(M, k, device=dev, dtype=torch.bfloat16)
                blob = ops.quantize(torch.randn(n, k, device=dev) * 0.02, f)
                wd = torch.ops.ipex_llm_amd.dequantize_device(blob, f, n, k, torch.bfloat16)
                ours, lib, blas = [], [], []
                for _ in range(3):
                    ours.append(timeit(lambda: torch.ops.ipex_llm_amd.gemm8p_lowbit(x, blob, f, n, k)))
                    lib.append(timeit(lambda: F.linear(x, torch.ops.ipex_llm_amd.dequantize_device(blob, f, n, k,
                                                                                                  torch.bfloat16))))
                    blas.append(timeit(lambda: F.linear(x, wd)))
                o, l, bl = min(ours), min(lib), min(blas)
                y1 = torch.ops.ipex_llm_amd.gemm8p_lowbit(x, blob, f, n, k).float()
                y2 = F.linear(x, wd).float()
                rel = ((y1 - y2).norm() / y2.norm()).item()
                fl = 2 * M * n * k
                print(json.dumps({"qtype": qt, "M": M, "op": name, "ours_us": round(o, 1),
                                  "dequant_plus_hipblaslt_us": round(l, 1), "hipblaslt_only_us": round(bl, 1),
                                  "ours_TF": round(fl / o / 1e6, 1), "speedup_vs_dequant_lib": round(l / o, 3),
                                  "vs_lib_only": round(bl / o, 3), "rel_diff": round(rel, 5)}), flush=True)
                del x, blob, wd
                continue
            x = torch.randn(M, k, device=dev, dtype=torch.bfloat16)
            w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02
            # interleaved rounds in one process (methodology rule 24)
            ours, lib = [], []
            for _ in range(3):
                ours.append(timeit(lambda: torch.ops.ipex_llm_amd.gemm_bf16(x, w)))
                lib.append(timeit(lambda: F.linear(x, w)))
            o, l = min(ours), min(lib)
            y1 = torch.ops.ipex_llm_amd.gemm_bf16(x, w).float()
            y2 = F.linear(x, w).float()
            rel = ((y1 - y2).norm() / y2.norm()).item()
            fl = 2 * M * n * k
            print(json.dumps({"M": M, "op": name, "N": n, "K": k, "ours_us": round(o, 1), "hipblaslt_us": round(l, 1),
                              "ours_TF": round(fl / o / 1e6, 1), "lib_TF": round(fl / l / 1e6, 1),
                              "speedup": round(l / o, 3), "rel_diff": round(rel, 5)}), flush=True)
            del x, w


if __name__ == "__main__":
    main()
