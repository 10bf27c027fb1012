"""Kernel time of the last N steps of a training trace keyed by (name, grid):
the step boundaries are the optimizer launches (the last kernel family of a
step).  python tools/trace_by_grid.py run_results.db [steps]"""
import collections
import sqlite3
import sys

db, nsteps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2
c = sqlite3.connect(db)
rows = c.execute("select name, grid_x, grid_y, grid_z, workgroup_x, start, end from kernels order by start").fetchall()
# a step ends at its last optimizer kernel; take everything after the (nsteps+1)-th last optimizer run
opt = [i for i, r in enumerate(rows) if "adam" in r[0].lower()]
ends = [opt[0]] + [b for a, b in zip(opt, opt[1:]) if b != a + 1] if opt else []
starts = [i for i in range(len(rows)) if i in set(opt) and (i - 1) not in set(opt)]
if len(starts) >= nsteps + 1:
    lo = starts[-nsteps - 1]
    while lo + 1 < len(rows) and "adam" in rows[lo + 1][0].lower():
        lo += 1
    seg = rows[lo + 1:]
else:
    seg = rows[len(rows) // 2:]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    k = (r[0][:100], r[1], r[2], r[3], r[4])
    agg[k][0] += 1
    agg[k][1] += (r[6] - r[5]) / 1000
tot = sum(v[1] for v in agg.values())
span = (seg[-1][6] - seg[0][5]) / 1000
print(f"{db}: last {nsteps} steps: kernel sum {tot / nsteps / 1000:.2f} ms/step, span {span / nsteps / 1000:.2f} ms/step")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:80]:
    print(f"  {v[0] / nsteps:7.1f}/step {v[1] / v[0]:9.2f} us {v[1] / nsteps / 1000:7.3f} ms/step  grid=({k[1]},{k[2]},{k[3]}) "
          f"wg={k[4]}  {k[0]}")
