#!/usr/bin/env python3
"""Per-dispatch timeline of ONE training step from a rocprofv3 kernel-trace database, with a
critical-path attribution over the streams.

Usage: prof_step.py <run_results.db> [marker_regex] [step_index_from_end] [--critical]
       prof_step.py <run_results.db> --totals     (whole run: kernel time per kernel, top 30)

The step boundary is the dispatch matching ``marker_regex`` (default: the first kernel of a
step, ``nchw_to_s2d_kernel`` for the ResNet bench / ``embedding_fwd_kernel`` for BERT; with the
in-backward optimizer the optimizer kernels are spread over the backward and no longer mark the
step end); a run of adjacent marker dispatches counts as one boundary. The step printed is the
one ending at the N-th boundary from the end (default 1 = the last complete step). Prints every
dispatch in start order with its duration, stream and grid, then the summed kernel time and the
wall span (first start to last end): with the weight-gradient side stream the two differ by the
overlap.

``--critical`` adds the critical-path table. The compute stream is the stream of the marker
dispatch. The step's wall span is cut at every dispatch start/end; each slice is charged to
  * the compute-stream kernel running in it (the compute stream is serial, so its kernels are
    the critical path whenever it is busy), else
  * the side-stream kernel(s) running while the compute stream is idle -- side work that is
    EXPOSED (the compute stream waits on it, or has nothing issued), else
  * "idle" (no kernel on any stream: host issue gaps and launch latency).
Side-stream time that runs under a busy compute stream is reported as "overlapped"; it costs
wall time only through contention (it slows the compute kernels beside it).
"""
import re
import sqlite3
import sys
from collections import defaultdict


def _family(name):
    """Kernel family: the name without template arguments and parameters."""
    n = name.split("(")[0]
    n = re.sub(r"^void ", "", n)
    return n.split("<")[0]


def load_rows(db):
    cur = sqlite3.connect(db).cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(kernels)").fetchall()]
    low = [c.lower() for c in cols]
    start = cols[low.index("start")]
    end = cols[low.index("end")] if "end" in low else None
    grid = [c for c in ("grid_size", "grid_size_x") if c in cols][:1]
    stream = [c for c in ("stream_id", "queue_id", "queue") if c in low][:1]
    stream = [cols[low.index(s)] for s in stream]
    sel = "select name, duration, %s, %s, %s, %s from kernels order by %s" % (
        start, end or "0", stream[0] if stream else "0", grid[0] if grid else "0", start)
    rows = []
    for name, dur, st, en, sid, g in cur.execute(sel).fetchall():
        en = en if end else st + dur
        rows.append({"name": name, "dur": en - st if end else dur, "start": st, "end": en, "stream": sid,
                     "grid": g})
    return rows


def pick_step(rows, marker, back):
    hits = [i for i, r in enumerate(rows) if marker.search(r["name"])]
    ends = [i for k, i in enumerate(hits) if k == 0 or hits[k - 1] != i - 1]   # first of each adjacent run
    ends = [i - 1 for i in ends if i > 0]                                     # the step ends just before it
    if len(ends) < back + 1:
        return None
    lo, hi = ends[-back - 1] + 1, ends[-back] + 1
    return rows[lo:hi]


def critical_path(step, compute_stream):
    """Slice the wall span of ``step`` and charge each slice (see module doc). Returns
    (crit[family] ns, exposed_side[family] ns, overlapped_side[family] ns, idle ns, wall ns)."""
    t0 = min(r["start"] for r in step)
    t1 = max(r["end"] for r in step)
    cuts = sorted({t0, t1} | {r["start"] for r in step} | {r["end"] for r in step})
    comp = sorted((r for r in step if r["stream"] == compute_stream), key=lambda r: r["start"])
    side = [r for r in step if r["stream"] != compute_stream]
    crit, exposed, overl = defaultdict(float), defaultdict(float), defaultdict(float)
    idle = 0.0
    for a, b in zip(cuts[:-1], cuts[1:]):
        if b <= a:
            continue
        mid = 0.5 * (a + b)
        c = [r for r in comp if r["start"] <= mid < r["end"]]
        s = [r for r in side if r["start"] <= mid < r["end"]]
        d = b - a
        if c:
            for r in c:
                crit[_family(r["name"])] += d / len(c)
            for r in s:
                overl[_family(r["name"])] += d / len(s)
        elif s:
            for r in s:
                exposed[_family(r["name"])] += d / len(s)
        else:
            idle += d
    return crit, exposed, overl, idle, t1 - t0


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    critical = "--critical" in sys.argv
    db = args[0]
    if "--totals" in sys.argv:
        agg = defaultdict(lambda: [0.0, 0])
        for r in load_rows(db):
            k = re.sub(r"^void ", "", r["name"].split("(")[0])[:110]
            agg[k][0] += r["dur"]
            agg[k][1] += 1
        total = sum(v[0] for v in agg.values())
        print("| kernel | ms | calls | share |\n|---|---|---|---|")
        for k, (d, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:30]:
            print("| `%s` | %.3f | %d | %.1f%% |" % (k, d / 1e6, n, 100.0 * d / max(total, 1)))
        print("\ntotal kernel time %.3f ms over %d dispatches" % (total / 1e6, sum(v[1] for v in agg.values())))
        return
    marker = re.compile(args[1] if len(args) > 1 else r"nchw_to_s2d_kernel|embedding_fwd_kernel")
    back = int(args[2]) if len(args) > 2 else 1
    rows = load_rows(db)
    step = pick_step(rows, marker, back)
    if step is None:
        print("need at least %d marker dispatches" % (back + 1))
        return
    tot = sum(r["dur"] for r in step)
    streams = sorted({r["stream"] for r in step})
    sid = {s: i for i, s in enumerate(streams)}
    print("| # | us | cum ms | stream | grid | kernel |")
    print("|---|---|---|---|---|---|")
    cum = 0
    for i, r in enumerate(step):
        cum += r["dur"]
        print("| %d | %.1f | %.3f | %d | %s | `%s` |" % (i, r["dur"] / 1e3, cum / 1e6, sid[r["stream"]], r["grid"],
                                                      r["name"].split("(")[0][:80]))
    wall = max(r["end"] for r in step) - step[0]["start"]
    print("\nstep kernel time %.3f ms over %d dispatches on %d stream(s); wall span %.3f ms"
          % (tot / 1e6, len(step), len(streams), wall / 1e6))
    if not critical:
        return
    m = [r for r in step if marker.search(r["name"])]
    cs = m[0]["stream"] if m else step[0]["stream"]
    crit, exposed, overl, idle, wall = critical_path(step, cs)
    fams = sorted(set(crit) | set(exposed) | set(overl), key=lambda f: -(crit.get(f, 0) + exposed.get(f, 0)))
    print("\n## Critical path (compute stream = stream %d)\n" % sid[cs])
    print("| family | critical ms | of wall | exposed side ms | overlapped side ms |")
    print("|---|---|---|---|---|")
    for f in fams:
        print("| `%s` | %.3f | %.1f%% | %.3f | %.3f |" % (f, crit.get(f, 0) / 1e6, 100.0 * crit.get(f, 0) / wall,
                                                    exposed.get(f, 0) / 1e6, overl.get(f, 0) / 1e6))
    print("| (idle: no kernel running) | %.3f | %.1f%% | | |" % (idle / 1e6, 100.0 * idle / wall))
    print("\nwall %.3f ms = compute-stream busy %.3f + exposed side %.3f + idle %.3f; side work overlapped "
          "under compute %.3f ms" % (wall / 1e6, sum(crit.values()) / 1e6, sum(exposed.values()) / 1e6,
                                     idle / 1e6, sum(overl.values()) / 1e6))


if __name__ == "__main__":
    main()
