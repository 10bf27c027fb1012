"""Kernel time inside the prefill window of a bench.py rocprofv3 database:
dispatches from the first to the last attn_prefill_kernel (+ the last
prefill's tail up to the next decode_advance), per trial and in total.

usage: prefill_window.py DB"""
import sqlite3
import sys


def main(path):
    db = sqlite3.connect(path)
    cur = db.cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = cur.execute(f"select {name}, start, end from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if "attn_prefill" in r[0]]
    if not idx:
        print("no attn_prefill dispatches")
        return
    # trials: groups of 32 attn_prefill launches (one per layer)
    groups = [idx[i:i + 32] for i in range(0, len(idx), 32)]
    for gi, g in enumerate(groups):
        a = g[0]
        # include the embedding / first-layer work before the first attention and the tail after the last
        while a > 0 and "quantize_device" not in rows[a - 1][0] and "decode_advance" not in rows[a - 1][0] \
                and rows[a][1] - rows[a - 1][2] < 2e6:
            a -= 1
        b = g[-1]
        while b + 1 < len(rows) and "decode_advance" not in rows[b + 1][0] and "attn_prefill" not in rows[b + 1][0] \
                and rows[b + 1][1] - rows[b][2] < 2e6:
            b += 1
        ker = sum((r[2] - r[1]) for r in rows[a:b + 1]) / 1e6
        wall = (rows[b][2] - rows[a][1]) / 1e6
        agg = {}
        for r in rows[a:b + 1]:
            d = agg.setdefault(r[0], [0, 0.0])
            d[0] += 1
            d[1] += (r[2] - r[1]) / 1e3
        print(f"trial {gi}: {b - a + 1} dispatches, kernel {ker:.2f} ms, wall {wall:.2f} ms")
        if gi == len(groups) - 1:
            for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
                print(f"   {n:5d} {t:10.1f} us  {k[:110]}")


if __name__ == "__main__":
    main(sys.argv[1])
