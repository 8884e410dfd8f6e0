#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (rocpd SQLite output) into markdown.

    python tools/prof_summary.py gpurun_out/prof8b/k_results.db [--top 25] > profiles/x.md
"""
from __future__ import annotations

import argparse
import sqlite3


def summarize(db: str, top: int = 25, title: str = "", last_ms: float = 0.0) -> str:
    """``last_ms``: only kernels that start in the trace's last last_ms ms (the
    timed steps of a bench run sit at the end of its trace)."""
    c = sqlite3.connect(db)
    where = ""
    if last_ms > 0:
        t_end = c.execute("select max(end) from kernels").fetchone()[0]
        where = f"where start >= {int(t_end - last_ms * 1e6)}"
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(start), max(end), max(grid_x * grid_y * "
                     "grid_z), max(workgroup_x * workgroup_y * workgroup_z) from kernels "
                     f"{where} group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    span = (max(r[5] for r in rows) - min(r[4] for r in rows)) if rows else 0
    out = [f"## {title or db}", "", f"kernel time total {total/1e6:.1f} ms over a {span/1e6:.1f} ms trace window", "",
           "| kernel | calls | total ms | % | avg us | max threads (grid) | workgroup |",
           "|---|---:|---:|---:|---:|---:|---:|"]
    for name, n, tot, avg, _, _, grid, wg in rows[:top]:
        short = name.split("(")[0][:90]
        out.append(f"| `{short}` | {n} | {tot/1e6:.2f} | {100*tot/total:.1f} | {avg/1e3:.1f} | {grid} | {wg} |")
    return "\n".join(out) + "\n"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--title", default="")
    ap.add_argument("--last-ms", type=float, default=0.0, help="only the trace's last N ms (the timed steps)")
    a = ap.parse_args()
    print(summarize(a.db, a.top, a.title, a.last_ms))


if __name__ == "__main__":
    main()
