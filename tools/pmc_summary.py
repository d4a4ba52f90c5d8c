#!/usr/bin/env python3
"""Average PMC counter values per kernel dispatch from tools/pmc.sh output directories.
  python3 tools/pmc_summary.py gpurun_out/<dir> [kernel-substring ...]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
want = sys.argv[2:] or ["update_rows_kernel", "apply_patches_kernel"]
for f in sorted(glob.glob(os.path.join(root, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        k = next((w for w in want if w in r["Kernel_Name"]), None)
        if k:
            agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(agg.items()):
        print(f"{os.path.relpath(f, root).split(os.sep)[0]:6s} {k:22s} {c:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")
