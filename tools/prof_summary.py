"""Summarise a rocprofv3 kernel-trace database (per-kernel totals).

usage: prof_summary.py DB [top] [--after SUBSTR]
  --after SUBSTR  only count dispatches that start after the last dispatch
                  whose name contains SUBSTR (e.g. split prefill from decode)
"""
import sqlite3
import sys


def load(path):
    db = sqlite3.connect(path)
    cur = db.cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
    namecol = "kernel_name" if "kernel_name" in cols else "name"
    return cur.execute(f"select {namecol}, start, end from kernels order by start").fetchall()


def summarize(path, top=30, after=None):
    rows = load(path)
    if after:
        last = max((s for n, s, e in rows if after in n), default=None)
        if last is not None:
            rows = [r for r in rows if r[1] > last]
    agg = {}
    for n, s, e in rows:
        d = agg.setdefault(n, [0, 0.0])
        d[0] += 1
        d[1] += (e - s) / 1e3
    tot = sum(v[1] for v in agg.values())
    span = (rows[-1][2] - rows[0][1]) / 1e3 if rows else 0.0
    # busy = union of kernel intervals; the rest of the span is launch gaps
    busy, cur_s, cur_e = 0.0, None, None
    for _, s, e in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += (cur_e - cur_s) / 1e3
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += (cur_e - cur_s) / 1e3
    out = [f"kernel time {tot / 1e3:.2f} ms over {sum(v[0] for v in agg.values())} dispatches; wall span {span / 1e3:.2f} ms; "
           f"GPU busy {busy / 1e3:.2f} ms; idle gaps {(span - busy) / 1e3:.2f} ms"]
    out.append(f"{'calls':>7} {'total_us':>11} {'avg_us':>9} {'pct':>6}  kernel")
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        out.append(f"{c:7d} {t:11.1f} {t / c:9.2f} {100 * t / max(tot, 1e-9):6.2f}  {n[:110]}")
    return "\n".join(out)


if __name__ == "__main__":
    args = sys.argv[1:]
    after = None
    if "--after" in args:
        i = args.index("--after")
        after = args[i + 1]
        del args[i:i + 2]
    print(summarize(args[0], int(args[1]) if len(args) > 1 else 30, after))
