#!/usr/bin/env python3
"""Per-dispatch timeline of ONE training step from a rocprofv3 kernel-trace database.

Usage: prof_step.py <run_results.db> [marker_regex] [step_index_from_end]

The step boundary is the dispatch matching ``marker_regex`` (default: the first kernel of a
step, ``nchw_to_s2d_kernel`` for the ResNet bench / ``embedding_fwd_kernel`` for BERT; with the
in-backward optimizer the optimizer kernels are spread over the backward and no longer mark the
step end); a run of adjacent marker dispatches counts as one boundary. The step printed is the
one ending at the N-th boundary from the end (default 1 = the last complete step). Prints every
dispatch in start order with its duration and grid, then the summed kernel time and the wall
span (first start to last end): with the weight-gradient side stream the two differ by the
overlap.
"""
import re
import sqlite3
import sys


def main():
    db = sys.argv[1]
    marker = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"nchw_to_s2d_kernel|embedding_fwd_kernel")
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    cur = sqlite3.connect(db).cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(kernels)").fetchall()]
    start = "start" if "start" in cols else cols[[c.lower() for c in cols].index("start")]
    grid = [c for c in ("grid_size", "grid_size_x", "workgroup_size") if c in cols]
    sel = "select name, duration, %s%s from kernels order by %s" % (start, "".join(", " + g for g in grid), start)
    rows = cur.execute(sel).fetchall()
    hits = [i for i, r in enumerate(rows) if marker.search(r[0])]
    ends = [i for k, i in enumerate(hits) if k == 0 or hits[k - 1] != i - 1]   # first of each adjacent run
    ends = [i - 1 for i in ends if i > 0]                                     # the step ends just before it
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
    wall = max(r[2] + r[1] for r in step) - step[0][2] if step else 0
    print("\nstep kernel time %.3f ms over %d dispatches; wall span %.3f ms" % (tot / 1e6, len(step), wall / 1e6))


if __name__ == "__main__":
    main()
