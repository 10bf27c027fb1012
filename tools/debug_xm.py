"""Sweep the decode GEMV forms (gemv_accum / GLU / store) over M, K and split-K
against fp32 torch; with ILLM_GEMV5_TRACE=1 the kernel choice is printed.
Used to localise the XM 1 / 2 instantiation failures (round 6)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from ipex_llm_amd import ops
from ipex_llm_amd.models.decoder import deinterleave_glu, interleave_glu_rows
from ipex_llm_amd.ops import reference as R
from ipex_llm_amd.quantize import get_format


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def where_bad(y, r):
    bad = ~torch.isfinite(y) | ((y - r).abs() > 0.05 * r.abs().max())
    rows = bad.any(1).nonzero().flatten().tolist()
    cols = bad.any(0).nonzero().flatten()
    return rows, sorted(set((cols // 16).tolist()))[:12], int(bad.sum())


def main():
    dev = torch.device("cuda")
    f = get_format("sym_int4").fmt
    torch.manual_seed(0)
    kind = sys.argv[1] if len(sys.argv) > 1 else "all"
    deq = lambda b, n, k: R.dequantize_device_blob(b.cpu(), f, n, k).to(dev).float()   # noqa: E731
    if kind in ("all", "accum"):
        N = 512
        for K in (1024, 2048, 4096):
            w = ops.quantize(torch.randn(N, K, device=dev) * 0.05, f)
            W = deq(w, N, K)
            for M in (1, 2, 5, 8):
                x = torch.randn(M, K, device=dev).bfloat16()
                r = x.float() @ W.t()
                for ks in (0, 1, 2, 4, 8):
                    acc = torch.zeros(M, N, device=dev)
                    ops.gemv_accum(x, w, f, N, K, acc, ks)
                    torch.cuda.synchronize()
                    e = rel(acc, r)
                    print(f"accum K={K} M={M} ks={ks} rel={e:.3e}", where_bad(acc, r) if not e < 1e-2 else "", flush=True)
    if kind in ("all", "glu"):
        I = 1024
        for H in (1024, 2048, 4096):
            gu = ops.quantize(interleave_glu_rows(torch.randn(I, H, device=dev) * 0.05,
                                                  torch.randn(I, H, device=dev) * 0.05), f)
            W = deq(gu, 2 * I, H)
            for M in (1, 2, 8):
                x = torch.randn(M, H, device=dev).bfloat16()
                g, u = deinterleave_glu(x.float() @ W.t())
                r = torch.nn.functional.silu(g) * u
                y = ops.gemv_glu(x, gu, f, 2 * I, H, 0)
                torch.cuda.synchronize()
                e = rel(y, r)
                print(f"glu H={H} M={M} rel={e:.3e}", where_bad(y.float(), r) if not e < 1e-2 else "", flush=True)
    if kind in ("all", "store"):
        N = 1024
        for K in (1024, 4096):
            w = ops.quantize(torch.randn(N, K, device=dev) * 0.05, f)
            W = deq(w, N, K)
            for M in (1, 8):
                x = torch.randn(M, K, device=dev).bfloat16()
                y = ops.lowbit_matmul(x, w, f, N, K)
                torch.cuda.synchronize()
                e = rel(y, x.float() @ W.t())
                print(f"store K={K} M={M} rel={e:.3e}", flush=True)


if __name__ == "__main__":
    main()
