#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (``--kernel-trace`` run) into a
per-kernel table (Markdown). Usage: prof_summary.py <run_results.db> <steps> [title]"""
import sqlite3
import sys


def main():
    db, steps = sys.argv[1], int(sys.argv[2])
    title = sys.argv[3] if len(sys.argv) > 3 else db
    cur = sqlite3.connect(db).cursor()
    rows = cur.execute("select name, count(*), sum(duration), avg(duration) from kernels group by name "
                       "order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows)
    native = sum(r[2] for r in rows if r[0].startswith(("zoo::", "void zoo::")))
    out = ["# %s" % title, "",
           "Total GPU kernel time %.2f ms over %d profiled steps = **%.2f ms/step**; "
           "zoo native (hand-written HIP) kernels = %.1f%% of GPU time." % (tot / 1e6, steps, tot / steps / 1e6,
                                                                           100.0 * native / max(tot, 1)), "",
           "| share | ms/step | calls/step | avg us | kernel |", "|---|---|---|---|---|"]
    for name, n, s, a in rows:
        short = name.split("(")[0][:90]
        out.append("| %.2f%% | %.3f | %.1f | %.1f | `%s` |" % (100.0 * s / tot, s / steps / 1e6, n / steps, a / 1e3,
                                                            short))
    print("\n".join(out))


if __name__ == "__main__":
    main()
