"""Time the decode GEMV shapes under the current ILLM_GEMV5_KW/KS env (one
process per setting; see tools/gemv_sweep5.sh).  Prints one JSON line per
(M, op) with microseconds and effective TB/s."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ipex_llm_amd import ops  # noqa: E402
from ipex_llm_amd.quantize import get_format  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

SHAPES = [("qkv", 6144, 4096, "part"), ("o", 4096, 4096, "part"), ("glu", 28672, 4096, "glu"),
          ("down", 4096, 14336, "part"), ("lm_head", 128256, 4096, "store")]
# GEMV_SHAPES=70b: Llama-3-70B projections, the non-GLU ones on the atomic
# accumulator path the decoder uses (ops.gemv_accum)
SHAPES_70B = [("qkv", 10240, 8192, "acc"), ("o", 8192, 8192, "acc"), ("glu", 57344, 8192, "glu"),
              ("down", 8192, 28672, "acc"), ("lm_head", 128256, 8192, "store")]


def main():
    ms = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1,8").split(",")]
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    ops.require()
    f = get_format("sym_int4").fmt
    dev = torch.device("cuda")
    tag = {"kw": os.environ.get("ILLM_GEMV5_KW", "auto"), "ks": os.environ.get("ILLM_GEMV5_KS", "auto"),
           "nw": os.environ.get("ILLM_GEMV5_NW", "auto")}
    shapes = SHAPES_70B if os.environ.get("GEMV_SHAPES") == "70b" else SHAPES
    if os.environ.get("GEMV_ACC") == "1":      # the decoder's atomic-accumulator form of the projections
        shapes = [(nm, n, k, "acc" if kd == "part" else kd) for nm, n, k, kd in shapes]
    if os.environ.get("GEMV_STORE1") == "1":   # full-K workgroups writing T outputs (no split-K)
        shapes = [(nm, n, k, "store1" if kd == "part" else kd) for nm, n, k, kd in shapes]
    for name, n, k, kind in shapes:
        if only and name not in only:
            continue
        copies = max(1, int(math.ceil(600e6 / (n * k * 0.5))))
        blobs = [ops.quantize(torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02, f) for _ in range(copies)]
        for M in ms:
            x = torch.randn(M, k, device=dev, dtype=torch.bfloat16)
            acc = torch.zeros(M, n, device=dev, dtype=torch.float32)
            i = [0]

            def run():
                i[0] = (i[0] + 1) % copies
                b = blobs[i[0]]
                if kind == "glu":
                    return ops.gemv_glu(x, b, f, n, k, 0)
                if kind == "acc":
                    return ops.gemv_accum(x, b, f, n, k, acc)
                if kind == "part":
                    return ops.gemv_partials(x, b, f, n, k, 0)
                if kind == "store1":            # one workgroup column per output: no split-K
                    return torch.ops.ipex_llm_amd.gemv(x, b, f, n, k, None, 0, 1, 0)
                return ops.lowbit_matmul(x, b, f, n, k)
            us = timeit(run)
            print(json.dumps({**tag, "M": M, "op": name, "us": round(us, 2),
                              "TBps": round(blobs[0].numel() / us / 1e6, 3)}), flush=True)
        del blobs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
