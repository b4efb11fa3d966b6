"""Device idle time between kernels, from a rocprofv3 --kernel-trace database.

    python tools/gap_summary.py TRACE_DIR [--from KERNEL_SUBSTR] [--min-span-ms 1]

Takes every kernel dispatch (rocpd `kernels` view: start / end in ns), sorts
them by start, and splits the timeline into busy time (union of kernel
intervals) and gaps.  Reported: span, busy, idle, idle share, the gap
histogram, and the kernels that most often FOLLOW a gap of more than 5 us
(where the device waited on the host: a synchronisation, a host-side step).
With --from, the window starts at the first dispatch whose name contains the
substring (skips generation / setup).
"""
import argparse
import glob
import json
import os
import sqlite3
from collections import Counter


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        c = sqlite3.connect(f)
        rows += list(c.execute("select start, end, name from kernels"))
    rows.sort()
    return rows


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0].replace("ahip::dev::", "").replace("ahip::zdev::", "z:")[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--from", dest="start", default=None)
    a = ap.parse_args()
    rows = load(a.trace)
    if a.start:
        i0 = next((i for i, r in enumerate(rows) if a.start in r[2]), 0)
        rows = rows[i0:]
    if not rows:
        print(json.dumps({"error": "no kernels"}))
        return
    busy = 0
    gaps = []
    cur_s, cur_e = rows[0][0], rows[0][1]
    follow = Counter()
    for s, e, name in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            g = s - cur_e
            gaps.append(g)
            if g > 5000:
                follow[short(name)] += 1
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = rows[-1][1] - rows[0][0]
    hist = Counter()
    for g in gaps:
        hist["<2us" if g < 2000 else "2-5us" if g < 5000 else "5-20us" if g < 20000 else
             "20-100us" if g < 100000 else ">=100us"] += 1
    big = sorted(gaps)[-5:]
    print(json.dumps(dict(kernels=len(rows), span_ms=span / 1e6, busy_ms=busy / 1e6,
                          idle_ms=(span - busy) / 1e6, idle_share=(span - busy) / span,
                          gap_hist=dict(hist), largest_gaps_us=[g / 1e3 for g in big],
                          after_gaps_over_5us=follow.most_common(8)), indent=1))


if __name__ == "__main__":
    main()
