#!/usr/bin/env python3
"""Per-dispatch timeline of ONE training step from a rocprofv3 kernel-trace database.

Usage: prof_step.py <run_results.db> [marker_regex] [step_index_from_end]

The step boundary is the dispatch matching ``marker_regex`` (default: the fused optimizer
kernel, ``sgd_kernel|adam_kernel``); the step printed is the one ending at the N-th marker
from the end (default 1 = the last complete step). Prints every dispatch in issue order with
its duration and grid, so a family total of prof_summary.py can be attributed to layers.
"""
import re
import sqlite3
import sys


def main():
    db = sys.argv[1]
    marker = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"sgd_kernel|adam_kernel")
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    cur = sqlite3.connect(db).cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(kernels)").fetchall()]
    start = "start" if "start" in cols else cols[[c.lower() for c in cols].index("start")]
    grid = [c for c in ("grid_size", "grid_size_x", "workgroup_size") if c in cols]
    sel = "select name, duration, %s%s from kernels order by %s" % (start, "".join(", " + g for g in grid), start)
    rows = cur.execute(sel).fetchall()
    ends = [i for i, r in enumerate(rows) if marker.search(r[0])]
    if len(ends) < back + 1:
        print("need at least %d marker dispatches, found %d" % (back + 1, len(ends)))
        return
    lo, hi = ends[-back - 1] + 1, ends[-back] + 1
    step = rows[lo:hi]
    tot = sum(r[1] for r in step)
    print("| # | us | cum ms | grid | kernel |")
    print("|---|---|---|---|---|")
    cum = 0
    for i, r in enumerate(step):
        cum += r[1]
        g = r[3] if len(r) > 3 else ""
        print("| %d | %.1f | %.3f | %s | `%s` |" % (i, r[1] / 1e3, cum / 1e6, g, r[0].split("(")[0][:80]))
    print("\nstep kernel time %.3f ms over %d dispatches" % (tot / 1e6, len(step)))


if __name__ == "__main__":
    main()
