"""Prefill GEMM sweep on one MI355X: our fp8 f8f6f4-MFMA GEMM (per-token
act quant included) vs hipBLASLt bf16 (torch.matmul) vs hipBLASLt fp8
(torch._scaled_mm) on Llama-3-8B projection shapes.  JSON lines to stdout."""
import json
import sys

import torch

sys.path.insert(0, ".")
from ipex_llm_amd import ops  # noqa: E402


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
    return s.elapsed_time(e) / iters * 1e3      # us


def main():
    ops.require()                       # load the extension (torch.ops.ipex_llm_amd.*)
    dev = torch.device("cuda")
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    for M in (1024, 2048, 4096, 8192):
        for name, (N, K) in shapes.items():
            w = torch.randn(N, K, device=dev) * 0.02
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w8, ws = ops.fp8_quantize_weight(w, False)
            wb = w.to(torch.bfloat16)
            t_ours = timeit(lambda: torch.ops.ipex_llm_amd.fp8_linear(x, w8, ws, None, False))
            xq8, sx8 = torch.ops.ipex_llm_amd.fp8_act_quant(x)
            t_k8p = timeit(lambda: torch.ops.ipex_llm_amd.fp8_gemm8p(xq8, sx8, w8, ws, False))
            t_disp = timeit(lambda: ops.fp8_linear(x, w8, ws, None, False))
            t_bf16 = timeit(lambda: torch.matmul(x, wb.t()))
            t_sm = None
            try:
                w8t = w8.view(torch.float8_e4m3fn).t()
                xq = x.to(torch.float8_e4m3fn)
                one = torch.ones((), device=dev)
                torch._scaled_mm(xq, w8t, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
                t_sm = timeit(lambda: torch._scaled_mm(xq, w8t, scale_a=one, scale_b=one, out_dtype=torch.bfloat16))
            except Exception as ex:  # noqa: BLE001
                t_sm = f"n/a: {type(ex).__name__}"
            fl = 2.0 * M * N * K
            rec = {"M": M, "proj": name, "N": N, "K": K, "fp8_ours_us": round(t_ours, 1),
                   "fp8_8p_kernel_only_us": round(t_k8p, 1), "fp8_8p_kernel_tflops": round(fl / t_k8p / 1e6, 1),
                   "fp8_ours_tflops": round(fl / t_ours / 1e6, 1), "fp8_dispatch_us": round(t_disp, 1),
                   "fp8_dispatch_tflops": round(fl / t_disp / 1e6, 1), "bf16_hipblaslt_us": round(t_bf16, 1),
                   "bf16_tflops": round(fl / t_bf16 / 1e6, 1),
                   "fp8_scaled_mm_us": round(t_sm, 1) if isinstance(t_sm, float) else t_sm,
                   "kernel_vs_scaled_mm": round(t_sm / t_k8p, 3) if isinstance(t_sm, float) else None}
            print(json.dumps(rec), flush=True)
            del w, x, w8, wb
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
