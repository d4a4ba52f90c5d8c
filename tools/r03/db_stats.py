#!/usr/bin/env python3
"""rocprofv3's SQLite output (rocpd, the default format here) -> the kernel-stats CSV its
--output-format csv writes: Name, Calls, TotalDurationNs, AverageNs, Percentage.
  python3 tools/r03/db_stats.py <dir with *.db> <out.csv>"""
import csv
import glob
import sqlite3
import sys

db = glob.glob(sys.argv[1].rstrip("/") + "/**/*.db", recursive=True)[0]
rows = sqlite3.connect(db).execute("select name, total_calls, total_duration, average, percentage from top_kernels")
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for r in rows:
        w.writerow([r[0], r[1], round(r[2] * 1000), round(r[3] * 1000, 1), round(r[4], 3)])
