#!/usr/bin/env python
"""Print the rocprofv3 --stats kernel summary (name, calls, average us, total %) found under a directory."""
import csv
import glob
import sys

for f in glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
        print(f"{r['Name'][:90]:90s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:10.1f} us {float(r['Percentage']):6.2f}%")
