"""Kernel timeline gaps from a rocprofv3 --kernel-trace run (CSV or rocpd DB).

    python tools/timeline.py TRACE_DIR [KERNEL_SUBSTR_THAT_MARKS_CYCLE]

Prints: busy time, idle time between consecutive kernels (device gaps), and the
largest gaps with the kernels on either side -- the launch/sync overhead of a
restart cycle that per-kernel averages do not show.
"""
import csv
import glob
import os
import sqlite3
import sys


def load(d):
    ev = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                ev.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), row["Kernel_Name"]))
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        c = sqlite3.connect(f)
        names = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
        tab = "kernels" if "kernels" in names else None  # rocpd view with kernel names
        if tab is None:
            tab = next(n for n in names if "kernel" in n.lower() and "dispatch" in n.lower())
        cols = [r[1] for r in c.execute("pragma table_info(%s)" % tab)]
        nm = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else None)
        q = "select start, end, %s from %s" % (nm or "''", tab)
        ev += [(int(a), int(b), str(n)) for a, b, n in c.execute(q)]
    ev.sort()
    return ev


def short(n):
    n = n.split("(")[0]
    return n.replace("void ", "").replace("ahip::dev::(anonymous namespace)::", "")[:60]


def main():
    ev = load(sys.argv[1])
    mark = sys.argv[2] if len(sys.argv) > 2 else "k_csr_sell"
    # analyse the window between the first and last marker kernel
    idx = [i for i, e in enumerate(ev) if mark in e[2]]
    ev = ev[idx[0]: idx[-1] + 1]
    busy = sum(b - a for a, b, _ in ev)
    span = ev[-1][1] - ev[0][0]
    gaps = [(ev[i + 1][0] - ev[i][1], short(ev[i][2]), short(ev[i + 1][2])) for i in range(len(ev) - 1)]
    print("kernels %d  span %.3f ms  busy %.3f ms  idle %.3f ms (%.1f%%)"
          % (len(ev), span / 1e6, busy / 1e6, (span - busy) / 1e6, 100.0 * (span - busy) / span))
    from collections import defaultdict
    by = defaultdict(lambda: [0, 0])
    for g, a, b in gaps:
        by[(a, b)][0] += g
        by[(a, b)][1] += 1
    print("idle by boundary (top 15):")
    for (a, b), (g, c) in sorted(by.items(), key=lambda x: -x[1][0])[:15]:
        print("  %8.3f ms %5d x %7.2f us  %s -> %s" % (g / 1e6, c, g / c / 1e3, a, b))
    print("largest single gaps:")
    for g, a, b in sorted(gaps, reverse=True)[:10]:
        print("  %8.1f us  %s -> %s" % (g / 1e3, a, b))


if __name__ == "__main__":
    main()
