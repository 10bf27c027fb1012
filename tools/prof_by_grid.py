"""Kernel totals keyed by (name, grid) from a rocprofv3 --kernel-trace
database, optionally only after the last dispatch whose name contains a
marker (split a run's final decode / speculative window from its prefills).

usage: prof_by_grid.py DB [top] [--after SUBSTR] [--per N]
  --per N   also print per-unit time (total / N, e.g. N = rounds or steps)
"""
import sqlite3
import sys


def main():
    args = sys.argv[1:]
    after = per = None
    if "--after" in args:
        i = args.index("--after")
        after = args[i + 1]
        del args[i:i + 2]
    if "--per" in args:
        i = args.index("--per")
        per = float(args[i + 1])
        del args[i:i + 2]
    db = sqlite3.connect(args[0])
    top = int(args[1]) if len(args) > 1 else 40
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    namecol = "kernel_name" if "kernel_name" in cols else "name"
    rows = db.execute(f"select {namecol}, grid_x, grid_y, grid_z, start, end from kernels order by start").fetchall()
    if after:
        last = max((r[4] for r in rows if after in r[0]), default=None)
        if last is not None:
            rows = [r for r in rows if r[4] > last]
    if not rows:
        print("no dispatches")
        return
    agg = {}
    for n, gx, gy, gz, s, e in rows:
        a = agg.setdefault((n[:100], gx, gy, gz), [0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e3
    busy = sum(v[1] for v in agg.values())
    span = (rows[-1][5] - rows[0][4]) / 1e3
    print(f"window: {len(rows)} dispatches, busy {busy / 1e3:.2f} ms, span {span / 1e3:.2f} ms"
          + (f", per unit: busy {busy / per:.1f} us, span {span / per:.1f} us" if per else ""))
    for (n, gx, gy, gz), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        extra = f" {t / per:9.1f} us/unit" if per else ""
        print(f"{c:7d} {t / c:9.2f} us {t / 1e3:9.2f} ms{extra}  grid=({gx},{gy},{gz})  {n}")


if __name__ == "__main__":
    main()
