"""MFMA GEMM engine sweep (GPU box): the hand-written engine (gemm_mfma.hip)
vs dequantize + library GEMM (hipBLASLt via F.linear) at Llama-3-8B shapes.
One JSON line per (qtype, M, projection).  Env: GEMM_M (comma list), GEMM_Q
(qtypes; "dense" = bf16 weights vs F.linear), GEMM_TILE / GEMM_KS (force)."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ipex_llm_amd import ops  # noqa: E402
from ipex_llm_amd.quantize import get_format  # noqa: E402


def timeit(fn, it=20):
    for _ in range(3):
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
    tile = int(os.environ.get("GEMM_TILE", "-1"))
    ks = int(os.environ.get("GEMM_KS", "0"))
    shapes = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)]
    for qt in os.environ.get("GEMM_Q", "sym_int4").split(","):
        for M in [int(v) for v in os.environ.get("GEMM_M", "1024,4096").split(",")]:
            for name, n, k in shapes:
                w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02
                x = torch.randn(M, k, device=dev, dtype=torch.bfloat16)
                if qt == "dense":
                    ours = timeit(lambda: torch.ops.ipex_llm_amd.mfgemm(x, w, -1, n, k, None, False, 0, tile, ks))
                    lib = timeit(lambda: F.linear(x, w))
                    extra = {}
                    y1 = torch.ops.ipex_llm_amd.mfgemm(x, w, -1, n, k, None, False, 0, tile, ks).float()
                    y2 = F.linear(x, w).float()
                else:
                    f = get_format(qt).fmt
                    blob = ops.quantize(w, f)
                    ours = timeit(lambda: torch.ops.ipex_llm_amd.mfgemm(x, blob, f, n, k, None, False, 0, tile, ks))
                    lib = timeit(lambda: F.linear(x, torch.ops.ipex_llm_amd.dequantize_device(blob, f, n, k, x.dtype)))
                    wd = torch.ops.ipex_llm_amd.dequantize_device(blob, f, n, k, x.dtype)
                    blas = timeit(lambda: F.linear(x, wd))          # library GEMM alone (weight pre-dequantized)
                    old = timeit(lambda: torch.ops.ipex_llm_amd.gemm(x, blob, f, n, k, None))
                    y1 = torch.ops.ipex_llm_amd.mfgemm(x, blob, f, n, k, None, False, 0, tile, ks).float()
                    y2 = F.linear(x, wd).float()
                    del wd
                    extra = {"blas_only_us": round(blas, 1), "old_kernel_us": round(old, 1)}
                rel = ((y1 - y2).norm() / y2.norm()).item()
                fl = 2 * M * n * k
                print(json.dumps({"qtype": qt, "M": M, "op": name, "ours_us": round(ours, 1), "lib_us": round(lib, 1),
                                  "ours_TF": round(fl / ours / 1e6, 1), "lib_TF": round(fl / lib / 1e6, 1),
                                  "speedup": round(lib / ours, 3), "rel_diff": round(rel, 5),
                                  "tile": tile, "ks": ks, **extra}), flush=True)
                del w, x


if __name__ == "__main__":
    main()
