#!/usr/bin/env python3
"""Per-kernel duration summary (name, calls, average/min/max us, share) from a rocprofv3 SQLite
results database (rocprofv3 writes `<dir>/<name>_results.db` unless --output-format csv)."""
import sqlite3
import sys


def main(path, top=20):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), avg(end - start), min(end - start), "
                     "max(end - start), sum(end - start) from kernels group by name "
                     "order by sum(end - start) desc").fetchall()
    total = sum(r[5] for r in rows) or 1
    print(f"{'calls':>6} {'avg_us':>10} {'min_us':>10} {'max_us':>10} {'share':>6}  kernel")
    for name, n, avg, mn, mx, tot in rows[:top]:
        print(f"{n:6d} {avg / 1e3:10.2f} {mn / 1e3:10.2f} {mx / 1e3:10.2f} {tot / total:6.1%}  "
              f"{name[:110]}")


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:]))
