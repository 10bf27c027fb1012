"""Per-dispatch decode breakdown from a rocprofv3 --kernel-trace database:
the last N decode steps (between decode_advance launches), kernels keyed by
(name, grid), per-step call counts and mean durations, step span vs kernel
sum.  python tools/decode_trace_summary.py run_results.db [steps]"""
import collections
import sqlite3
import sys

db, nsteps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5
c = sqlite3.connect(db)
rows = c.execute("select name, grid_x, grid_y, grid_z, workgroup_x, start, end from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if "decode_advance" in r[0]]
seg = rows[idx[-nsteps - 1] + 1: idx[-1] + 1]
agg = collections.OrderedDict()
gaps = 0.0
for prev, r in zip([None] + seg[:-1], seg):
    k = (r[0][:90], r[1], r[2], r[4])
    a = agg.setdefault(k, [0, 0.0])
    a[0] += 1
    a[1] += (r[6] - r[5]) / 1000
    if prev is not None:
        gaps += max(0, r[5] - prev[6]) / 1000
tot = sum(v[1] for v in agg.values())
span = (seg[-1][6] - seg[0][5]) / 1000
print(f"{db}: {len(rows)} dispatches; last {nsteps} decode steps: kernel sum {tot / nsteps:.1f} us/step, "
      f"span {span / nsteps:.1f} us/step, inter-kernel gaps {gaps / nsteps:.1f} us/step "
      f"({len(seg) / nsteps:.0f} launches/step)")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"  {v[0] / nsteps:6.1f}/step {v[1] / v[0]:8.2f} us  {v[1] / nsteps:8.1f} us/step  grid=({k[1]},{k[2]}) "
          f"wg={k[3]}  {k[0]}")
