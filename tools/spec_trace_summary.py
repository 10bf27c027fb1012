"""Speculative-decoding trace: GPU busy time vs wall span of the decode
window (after the last prefill-sized kernel), kernels keyed by (name, grid).
python tools/spec_trace_summary.py run_results.db"""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, grid_x, grid_y, grid_z, start, end from kernels order by start").fetchall()
# decode window: from the first decode_advance-free stretch after the last attn_prefill launch
last_pf = max((i for i, r in enumerate(rows) if "attn_prefill" in r[0]), default=0)
seg = rows[last_pf + 1:]
busy = sum(r[5] - r[4] for r in seg) / 1e6
span = (seg[-1][5] - seg[0][4]) / 1e6 if seg else 0
gaps = collections.Counter()
for a, b in zip(seg, seg[1:]):
    g = (b[4] - a[5]) / 1e3
    gaps["<2us" if g < 2 else "2-10us" if g < 10 else "10-100us" if g < 100 else ">=100us"] += g
print(f"decode window: {len(seg)} kernels, busy {busy:.2f} ms, span {span:.2f} ms; gap us by size: "
      + ", ".join(f"{k} {v / 1e3:.2f} ms" for k, v in gaps.items()))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    k = (r[0][:90], r[1], r[2], r[3])
    agg[k][0] += 1
    agg[k][1] += (r[5] - r[4]) / 1e3
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"  {v[0]:6d} {v[1] / v[0]:9.2f} us {v[1] / 1e3:8.2f} ms  grid=({k[1]},{k[2]},{k[3]})  {k[0]}")
