"""Standalone timing of the decode GEMV launches the native decoder issues at
B=1..8 (atomic accumulate, norm-in prologue, GLU), hipGraph-replayed over
rotating weight copies (cold in the MALL).  One JSON line per (op, M).

    ILLM_GEMV5_PF8=1 python tools/gemv_decode_ab.py 1,8
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ipex_llm_amd import ops  # noqa: E402
from ipex_llm_amd.quantize import get_format  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def main():
    ms = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1,8").split(",")]
    ops.require()
    f = get_format("sym_int4").fmt
    dev = torch.device("cuda")
    tag = {"pf8": os.environ.get("ILLM_GEMV5_PF8", "0")}
    H = 4096
    for name, n, k, kind in [("qkv", 6144, 4096, "acc"), ("o", 4096, 4096, "acc"), ("down", 4096, 14336, "acc"),
                             ("qkv_normin", 6144, 4096, "normin"), ("glu_normin", 28672, 4096, "glu_normin"),
                             ("glu", 28672, 4096, "glu")]:
        copies = max(1, int(math.ceil(600e6 / (n * k * 0.5))))
        blobs = [ops.quantize(torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02, f) for _ in range(copies)]
        w = torch.ones(H, device=dev, dtype=torch.bfloat16)
        for M in ms:
            x = torch.randn(M, k, device=dev, dtype=torch.bfloat16)
            acc = torch.zeros(M, n, device=dev, dtype=torch.float32)
            pend = torch.randn(M, H, device=dev, dtype=torch.float32)
            res = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
            r2 = torch.empty_like(res)
            i = [0]

            def run():
                i[0] = (i[0] + 1) % copies
                b = blobs[i[0]]
                if kind == "acc":
                    return ops.gemv_accum(x, b, f, n, k, acc)
                if kind == "normin":
                    return ops.gemv_norm_in(pend, res, r2, w, 1e-5, False, b, f, n, k, False, acc_out=acc)
                if kind == "glu_normin":
                    return ops.gemv_norm_in(pend, res, r2, w, 1e-5, False, b, f, n, k, True, 0)
                return ops.gemv_glu(x, b, f, n, k, 0)
            us = timeit(run)
            print(json.dumps({**tag, "M": M, "op": name, "us": round(us, 2),
                              "TBps": round(blobs[0].numel() / us / 1e6, 3)}), flush=True)
        del blobs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
