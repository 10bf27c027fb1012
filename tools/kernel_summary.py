"""Per-kernel time of the last N steps of a rocprofv3 --kernel-trace database,
steps delimited by a marker kernel (e.g. the optimizer's): kernels keyed by
name, per-step calls and milliseconds, sorted by time.
python tools/kernel_summary.py run_results.db MARKER_SUBSTRING [steps] [top]"""
import collections
import sqlite3
import sys

db, marker = sys.argv[1], sys.argv[2]
nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if marker in r[0]]
# the marker may launch several kernels per step: keep the last launch of each burst
ends = [i for j, i in enumerate(idx) if j + 1 == len(idx) or idx[j + 1] - i > 8]
seg = rows[ends[-nsteps - 1] + 1: ends[-1] + 1]
agg = collections.defaultdict(lambda: [0, 0.0])
for name, s, e in seg:
    a = agg[name[:110]]
    a[0] += 1
    a[1] += (e - s) / 1e6
tot = sum(v[1] for v in agg.values())
span = (seg[-1][2] - seg[0][1]) / 1e6
print(f"{db}: last {nsteps} steps (marker '{marker}'): kernel sum {tot / nsteps:.2f} ms/step, "
      f"span {span / nsteps:.2f} ms/step, {len(seg) / nsteps:.0f} launches/step")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"  {v[0] / nsteps:8.1f}/step  {v[1] / nsteps:8.3f} ms/step  {100 * v[1] / tot:5.1f} %  {k}")
