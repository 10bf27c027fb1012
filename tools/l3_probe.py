"""Infinity-Cache probe: decode GEMV time on cold weights (after streaming
1 GiB through the caches) vs weights warmed by ops l3_prefetch; prefetch
cost alone; and a prefetch in a parallel hipGraph branch next to a
latency-bound kernel chain (does a graph fork run concurrently here?)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ipex_llm_amd  # noqa: E402,F401
from ipex_llm_amd import ops  # noqa: E402
from ipex_llm_amd.quantize import get_format  # noqa: E402

P = torch.ops.ipex_llm_amd
dev = "cuda"
fmt = get_format("sym_int4").fmt
flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
M = int(os.environ.get("PROBE_M", "8"))
ws = {k: ops.quantize(torch.randn(n, kk, device=dev, dtype=torch.bfloat16) * 0.02, fmt) for k, (n, kk) in shapes.items()}
xs = {k: torch.randn(M, kk, device=dev, dtype=torch.bfloat16) for k, (n, kk) in shapes.items()}


def ev_time(fn, pre, reps=30):
    ts = []
    for _ in range(reps):
        pre()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


out = {}
for k, (n, kk) in shapes.items():
    w, x = ws[k], xs[k]
    g = lambda: ops.lowbit_matmul(x, w, fmt, n, kk)  # noqa: E731
    g()
    cold = ev_time(g, lambda: P.l3_prefetch(flush))
    warm = ev_time(g, lambda: (P.l3_prefetch(flush), P.l3_prefetch(w)))
    pf = ev_time(lambda: P.l3_prefetch(w), lambda: P.l3_prefetch(flush))
    pf256 = ev_time(lambda: P.l3_prefetch(w, 0, -1, 256), lambda: P.l3_prefetch(flush))
    mb = w.numel() * w.element_size() / 1e6
    out[k] = dict(MB=round(mb, 1), cold_us=round(cold, 1), warm_us=round(warm, 1), prefetch_us=round(pf, 1),
                  prefetch256_us=round(pf256, 1), cold_TBs=round(mb / cold, 2), warm_TBs=round(mb / warm, 2))
    print(json.dumps({k: out[k]}), flush=True)

# graph fork: main chain = 40 tiny dependent kernels (latency-bound), branch = prefetch of gate_up
tiny = torch.zeros(1024, device=dev)
wg = ws["gate_up"]


def chain():
    for _ in range(40):
        tiny.add_(1.0)


side = torch.cuda.Stream()
res = {}
for mode in ("chain", "chain+fork", "chain+serial"):
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        chain()
        if mode != "chain":
            P.l3_prefetch(wg)
    torch.cuda.synchronize()
    with torch.cuda.graph(gr):
        if mode == "chain+fork":
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                P.l3_prefetch(wg)
            chain()
            torch.cuda.current_stream().wait_stream(side)
        elif mode == "chain+serial":
            P.l3_prefetch(wg)
            chain()
        else:
            chain()
    res[mode] = round(ev_time(gr.replay, lambda: P.l3_prefetch(flush), reps=20), 1)
print(json.dumps({"graph_us": res}), flush=True)
