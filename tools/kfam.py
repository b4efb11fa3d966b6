"""Kernel time by family from a rocprofv3 --stats CSV (tools/pmc_summary.py --stats
output): calls, total, average and share of each kernel name family.

    python tools/kfam.py STATS_CSV [--skip k_band_fill,k_band_count,...]
"""
import argparse
import collections
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--skip", default="k_band_fill,k_band_count,k_sell_fill,k_symsell_fill,k_upper_stats,"
                "k_row_span,k_colw,k_larnv,k_scan")
a = ap.parse_args()
skip = [s for s in a.skip.split(",") if s]
fam = collections.defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(a.csv)):
    n = r["Name"]
    m = re.search(r"(k_\w+|__amd\w+)", n)
    k = m.group(1) if m else n[:40]
    if any(k.startswith(s) for s in skip):
        continue
    fam[k][0] += int(r["Calls"])
    fam[k][1] += float(r["TotalDurationUs"])
tot = sum(v[1] for v in fam.values())
for k, v in sorted(fam.items(), key=lambda x: -x[1][1]):
    print(f"{k:32s} calls={v[0]:6d} total={v[1]:10.1f}us avg={v[1] / v[0]:8.2f} share={100 * v[1] / tot:5.1f}%")
