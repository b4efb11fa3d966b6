"""Per-kernel HBM traffic from rocprofv3 PMC passes (MI355X_MICROARCH.md, HBM section).

    python tools/pmc_summary.py [--workload JSON] FETCH_DIR WRITE_DIR [TRACE_DIR] > profiles/rNN_pmc.json
    python tools/pmc_summary.py --stats TRACE_DIR > profiles/rNN_kernel_stats.csv

Reads rocprofv3 CSV output or its rocpd SQLite database (the default format).

FETCH_SIZE and WRITE_SIZE come from separate `rocprofv3 --pmc` passes (they do
not fit one TCC pass).  Both are reported in KiB.  On gfx950 FETCH_SIZE counts
128-B memory-side read requests as 64 B, so the corrected read bytes are
2 x FETCH_SIZE; WRITE_SIZE is exact for streaming stores.  Output: per kernel
name, launches, mean raw FETCH/WRITE (bytes) and the corrected traffic per launch.

--workload JSON: the profiled command's workload ({"workload", "n", "nnz",
"storage", "deterministic", "command"}, as bench.py's config names it), stored
in the summary; bench.py takes a summary's traffic only for a line of that
same workload (bench.pmc_traffic).
"""
import csv
import glob
import json
import os
import sqlite3
import sys
from collections import defaultdict


def load(d, counter):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):  # rocpd SQLite output
        c = sqlite3.connect(f)
        for name, val in c.execute("select kernel_name, value from counters_collection "
                                   "where counter_name = ?", (counter,)):
            acc[name].append(float(val) * 1024.0)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter:
                    acc[row["Kernel_Name"]].append(float(row["Counter_Value"]) * 1024.0)
    return acc


def durations(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        c = sqlite3.connect(f)
        # the rocpd top_kernels view reports microseconds
        for name, calls, avg in c.execute("select name, total_calls, average from top_kernels"):
            out[name] = dict(calls=int(calls), avg_ns=1e3 * float(avg))
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                out[row["Name"]] = dict(calls=int(row["Calls"]), avg_ns=float(row["AverageNs"]))
    return out


def stats_csv(d):
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        c = sqlite3.connect(f)
        for row in c.execute("select name, total_calls, total_duration, average, percentage "
                             "from top_kernels order by total_duration desc"):
            w.writerow(row)


def main():
    workload = None
    if len(sys.argv) > 2 and sys.argv[1] == "--workload":
        workload = json.loads(sys.argv[2])
        del sys.argv[1:3]
    if sys.argv[1] == "--stats":
        return stats_csv(sys.argv[2])
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    dur = durations(sys.argv[3]) if len(sys.argv) > 3 else {}
    res = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fm = sum(f) / len(f) if f else 0.0
        wm = sum(w) / len(w) if w else 0.0
        e = dict(launches=max(len(f), len(w)), fetch_raw_bytes=fm, write_bytes=wm,
                 traffic_bytes=2.0 * fm + wm)
        if k in dur:
            e["avg_ns"] = dur[k]["avg_ns"]
            e["traffic_gbs"] = e["traffic_bytes"] / dur[k]["avg_ns"]
        res[k] = e
    doc = dict(correction="traffic = 2*FETCH_SIZE + WRITE_SIZE (gfx950, MI355X_MICROARCH.md HBM)",
               kernels=res)
    if workload is not None:
        doc["workload"] = workload
    json.dump(doc, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
