#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc run (rocpd SQLite output): per kernel, the mean
of every collected counter per dispatch plus the mean dispatch time.

    python tools/pmc_summary.py gpurun_out/pmc_dgemm [--filter k_dgemm]
"""
from __future__ import annotations

import argparse
import collections
import glob
import os
import sqlite3


def summarise(path: str, filt: str = "") -> str:
    dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True) if os.path.isdir(path) else [path]
    out = []
    for db in dbs:
        c = sqlite3.connect(db)
        names = {r[0]: r[1] for r in c.execute("select id, name from rocpd_info_pmc")}
        syms = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
        disp = {}
        for eid, kid, start, end in c.execute("select event_id, kernel_id, start, end from rocpd_kernel_dispatch"):
            disp[eid] = (syms.get(kid, str(kid)), end - start)
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        cnt = collections.Counter()
        dur = collections.defaultdict(float)
        seen = set()
        for eid, pid, val in c.execute("select event_id, pmc_id, value from rocpd_pmc_event"):
            if eid not in disp:
                continue
            k, d = disp[eid]
            if filt and filt not in k:
                continue
            agg[k][names.get(pid, str(pid))] += val
            if eid not in seen:
                seen.add(eid)
                cnt[k] += 1
                dur[k] += d
        for k in sorted(agg, key=lambda x: -dur[x]):
            n = cnt[k]
            row = {m: v / n for m, v in sorted(agg[k].items())}
            out.append(f"{k[:90]}  dispatches={n} mean_us={dur[k] / n / 1e3:.1f}")
            for m, v in row.items():
                out.append(f"    {m:28s} {v:,.0f}")
            if "SQ_INSTS_VALU" in row and "SQ_WAVES" in row and row["SQ_WAVES"]:
                out.append(f"    VALU insts / wave            {row['SQ_INSTS_VALU'] / row['SQ_WAVES']:,.0f}")
            if "SQ_WAIT_INST_ANY" in row and "SQ_WAVE_CYCLES" in row and row["SQ_WAVE_CYCLES"]:
                out.append(f"    wait_inst_any / wave_cycles  {row['SQ_WAIT_INST_ANY'] / row['SQ_WAVE_CYCLES']:.2f}")
    return "\n".join(out)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    print(summarise(a.path, a.filter))
