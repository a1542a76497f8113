#!/usr/bin/env python3
"""Summarise rocprofv3 (rocpd sqlite) PMC results: per kernel, mean of each counter
over dispatches, plus mean duration.   python pmc_summary.py results.db [...]"""
import sqlite3
import sys
from collections import defaultdict


def summarise(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
    rows = c.execute("select * from counters_collection").fetchall()
    idx = {n: i for i, n in enumerate(cols)}
    acc = defaultdict(lambda: defaultdict(list))
    for r in rows:
        k = r[idx["kernel_name"]] if "kernel_name" in idx else r[idx.get("name", 0)]
        acc[k][r[idx["counter_name"]]].append(r[idx["value"]])
    out = {}
    for k, d in acc.items():
        out[k] = {n: sum(v) / len(v) for n, v in d.items()}
    try:
        for name, dur in c.execute("select name, avg(end - start) from kernels group by name"):
            if name in out:
                out[name]["duration_ns"] = dur
    except sqlite3.Error:
        pass
    return out


if __name__ == "__main__":
    for db in sys.argv[1:]:
        print("==", db)
        for k, d in summarise(db).items():
            print("  ", k[:90])
            for n, v in sorted(d.items()):
                print("      %-28s %14.1f" % (n, v))
