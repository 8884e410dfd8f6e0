#!/usr/bin/env python3
"""Link-idle analysis of a rocprofv3 --kernel-trace run (rocpd SQLite): the
union of the migration ring's copy-kernel intervals vs wall time in a window,
and the largest gaps with the kernels the compute queue ran during them.

    python tools/trace_gaps.py gpurun_out/prof70b [--copy k_batch_copy] [--last-ms 3000]
"""
from __future__ import annotations

import argparse
import collections
import glob
import os
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--copy", default="k_batch_copy")
    ap.add_argument("--last-ms", type=float, default=3000.0)
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    db = glob.glob(os.path.join(a.path, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    syms = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    rows = [(syms.get(k, str(k)), q, s, e) for k, q, s, e in
            c.execute("select kernel_id, queue_id, start, end from rocpd_kernel_dispatch order by start")]
    t_end = max(r[3] for r in rows)
    t0 = t_end - a.last_ms * 1e6
    rows = [r for r in rows if r[2] >= t0]
    copies = [(s, e) for n, q, s, e in rows if a.copy in n]
    other = [(n, q, s, e) for n, q, s, e in rows if a.copy not in n]
    busy, cur = 0, None
    gaps = []
    for s, e in copies:
        if cur is None:
            cur = [s, e]
        elif s <= cur[1]:
            cur[1] = max(cur[1], e)
        else:
            busy += cur[1] - cur[0]
            gaps.append((s - cur[1], cur[1], s))
            cur = [s, e]
    if cur:
        busy += cur[1] - cur[0]
    span = copies[-1][1] - copies[0][0] if copies else 1
    print(f"window {a.last_ms:.0f} ms: copy kernels {len(copies)}, link-busy {busy/1e6:.1f} ms of {span/1e6:.1f} ms "
          f"({100*busy/span:.1f}%)")
    gaps.sort(reverse=True)
    tot = sum(g[0] for g in gaps)
    print(f"gaps: {len(gaps)}, total {tot/1e6:.1f} ms; largest:")
    for g, s, e in gaps[:a.top]:
        during = collections.Counter(n.split("(")[0][:60] for n, q, ks, ke in other if ks < e and ke > s)
        print(f"  {g/1e6:8.2f} ms at +{(s-t0)/1e6:9.1f} ms  compute: {dict(during.most_common(4))}")
    comp = collections.defaultdict(float)
    for n, q, s, e in other:
        comp[n.split("(")[0][:70]] += (e - s)
    print("compute kernel time in window (ms):")
    for n, t in sorted(comp.items(), key=lambda x: -x[1])[:15]:
        print(f"  {t/1e6:9.1f}  {n}")


if __name__ == "__main__":
    main()
