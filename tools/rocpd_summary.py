#!/usr/bin/env python3
"""Per-kernel summary (calls, total / avg time, share) of a rocprofv3 run
written in its default rocpd SQLite format:
    python tools/rocpd_summary.py <run_results.db> [top] [--last-ms MS]
(--last-ms: only kernels that start in the trace's last MS milliseconds - the
timed steps of a bench run, without model init / warm-up)."""
import sqlite3
import sys


def main() -> None:
    args = [a for a in sys.argv[1:]]
    last_ms = None
    if "--last-ms" in args:
        i = args.index("--last-ms")
        last_ms = float(args[i + 1])
        del args[i:i + 2]
    db = args[0]
    top = int(args[1]) if len(args) > 1 else 20
    c = sqlite3.connect(db)
    where = ""
    if last_ms is not None:
        t_end = c.execute("select max(end) from kernels").fetchone()[0]
        where = f" where start >= {int(t_end - last_ms * 1e6)}"
    rows = c.execute("select name, count(*), sum(end - start) / 1e6, avg(end - start) / 1e3 from kernels"
                     f"{where} group by name order by 3 desc").fetchall()
    tot = sum(r[2] for r in rows)
    span = c.execute(f"select (max(end) - min(start)) / 1e6 from kernels{where}").fetchone()[0] or 0.0
    print(f"kernel time total {tot:.2f} ms over a {span:.1f} ms window\n")
    print("| kernel | calls | total ms | % | avg us |")
    print("|---|---:|---:|---:|---:|")
    for name, n, ms, us in rows[:top]:
        print(f"| `{name[:100]}` | {n} | {ms:.2f} | {100 * ms / tot:.1f} | {us:.1f} |")


if __name__ == "__main__":
    main()
