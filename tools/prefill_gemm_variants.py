"""Library-GEMM formulations for the prefill projections (M = 1024-8192,
Llama-3-8B shapes, bf16): y = x W^T as F.linear, as (W x^T)^T,   Also
the dequantize-to-bf16 cost of each weight (sym_int4).  JSON lines."""
import json
import sys

import torch

sys.path.insert(0, ".")
from ipex_llm_amd import ops  # noqa: E402
from ipex_llm_amd.quantize import qtypes as Q  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ops.require()
    dev = torch.device("cuda")
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    fmt = Q.get_format("sym_int4").fmt
    for M in (1024, 2048, 8192):
        for name, (N, K) in shapes.items():
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
            rec = {"M": M, "proj": name, "N": N, "K": K}
            rec["linear_us"] = round(timeit(lambda: torch.nn.functional.linear(x, w)), 1)
            rec["wxT_us"] = round(timeit(lambda: torch.mm(w, x.t()).t()), 1)
            # (a strided-batched bmm over overlapping K-slice views of x / W faulted the
            # library GEMM on MI355X -- illegal address at N = 4096; K splits are not tried)
            blob = torch.ops.ipex_llm_amd.quantize_device(w, fmt, False) if hasattr(torch.ops.ipex_llm_amd,
                                                                                     "quantize_device") else None
            if blob is not None:
                rec["dequant_us"] = round(timeit(lambda: torch.ops.ipex_llm_amd.dequantize_device(
                    blob, fmt, N, K, torch.bfloat16)), 1)
                if M <= 2048:
                    rec["fused_int4_us"] = round(timeit(lambda: torch.ops.ipex_llm_amd.gemm(x, blob, fmt, N, K,
                                                                                          None)), 1)
            fl = 2.0 * M * N * K
            rec["linear_tflops"] = round(fl / rec["linear_us"] / 1e6, 1)
            print(json.dumps(rec), flush=True)
            del x, w, blob
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
