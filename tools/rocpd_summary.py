#!/usr/bin/env python3
"""Per-kernel summary (calls, total / avg time, share) of a rocprofv3 run
written in its default rocpd SQLite format:  python tools/rocpd_summary.py <run_results.db> [top]"""
import sqlite3
import sys


def main() -> None:
    db = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end - start) / 1e6, avg(end - start) / 1e3 from kernels "
                     "group by name order by 3 desc").fetchall()
    tot = sum(r[2] for r in rows)
    print(f"kernel time total {tot:.2f} ms\n")
    print("| kernel | calls | total ms | % | avg us |")
    print("|---|---:|---:|---:|---:|")
    for name, n, ms, us in rows[:top]:
        print(f"| `{name[:100]}` | {n} | {ms:.2f} | {100 * ms / tot:.1f} | {us:.1f} |")


if __name__ == "__main__":
    main()
