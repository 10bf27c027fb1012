"""8-phase GEMM sweep (GPU box): the low-bit in-LDS-dequant kernel
(gemm8p_lowbit) and the dense bf16 one (gemm_bf16) against hipBLASLt on the
resident dense weight and dequantize + hipBLASLt, Llama-3-8B projection
shapes.  One JSON line per (qtype, M, op).  The decode schedule is picked
by ILLM_G8_SCHED (read once per process): run one process per variant.

  python tools/bench_g8.py [qtypes] [--m 8192,1024] [--dense]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ipex_llm_amd import ops  # noqa: E402
from ipex_llm_amd.quantize import get_format  # noqa: E402

SHAPES = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)]


def timed(fn, it=20):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("qtypes", nargs="?", default="sym_int4")
    ap.add_argument("--m", default="8192,1024")
    ap.add_argument("--dense", action="store_true", help="also time the dense 8-phase kernel")
    ap.add_argument("--ops", default="")
    args = ap.parse_args()
    ops.require()
    tops = torch.ops.ipex_llm_amd
    dev = torch.device("cuda")
    sched = os.environ.get("ILLM_G8_SCHED", "0")
    torch.manual_seed(0)
    for qt in args.qtypes.split(","):
        f = get_format(qt).fmt
        for M in [int(v) for v in args.m.split(",")]:
            for name, n, k in SHAPES:
                if args.ops and name not in args.ops.split(","):
                    continue
                w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02
                blob = ops.quantize(w, f)
                wd = tops.dequantize_device(blob, f, n, k, torch.bfloat16)
                x = torch.randn(M, k, device=dev, dtype=torch.bfloat16)
                ours = timed(lambda: tops.gemm8p_lowbit(x, blob, f, n, k, None))
                lib = timed(lambda: F.linear(x, wd))
                deq = timed(lambda: F.linear(x, tops.dequantize_device(blob, f, n, k, torch.bfloat16)))
                y1 = tops.gemm8p_lowbit(x, blob, f, n, k, None).float()
                y2 = F.linear(x.float(), wd.float())
                rel = ((y1 - y2).norm() / y2.norm()).item()
                fl = 2 * M * n * k
                rec = {"qtype": qt, "sched": int(sched), "M": M, "op": name, "lowbit_us": round(ours, 1),
                       "hipblaslt_dense_us": round(lib, 1), "dequant_hipblaslt_us": round(deq, 1),
                       "lowbit_TF": round(fl / ours / 1e6, 1), "vs_hipblaslt_dense": round(lib / ours, 3),
                       "vs_dequant_hipblaslt": round(deq / ours, 3), "rel_vs_fp32": round(rel, 6)}
                if args.dense:
                    dn = timed(lambda: tops.gemm_bf16(x, wd, None))
                    dn1 = timed(lambda: tops.gemm_bf16(x, wd, None, False, 0, False, 0, 1))
                    g8d = timed(lambda: tops.gemm_bf16(x, tops.dequantize_device(blob, f, n, k, torch.bfloat16)))
                    rec["dense8p_us"] = round(dn, 1)
                    rec["dense8p_nosplit_us"] = round(dn1, 1)
                    rec["dense8p_vs_hipblaslt"] = round(lib / dn, 3)
                    rec["g8d_us"] = round(g8d, 1)
                    rec["g8d_vs_dequant_hipblaslt"] = round(deq / g8d, 3)
                    rec["g8d_vs_hipblaslt_dense"] = round(lib / g8d, 3)
                    yd = tops.gemm_bf16(x, wd, None).float()
                    rec["dense8p_rel_vs_fp32"] = round(((yd - y2).norm() / y2.norm()).item(), 6)
                print(json.dumps(rec), flush=True)
                del w, blob, wd, x, y1, y2
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
