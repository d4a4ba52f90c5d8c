#!/usr/bin/env python3
"""Summary of tools/exp/pmc_mlp.sh: per (work, variant), the read-pass kernel's medians over its
launches: TA busy share (TA_TA_BUSY_sum / 256 TAs / cycles per XCD), TA address stalls, DRAM reads
outstanding (TCC_EA0_RDREQ_LEVEL_sum / cycles per XCD, the round-1 definition), VALU instructions
per wave (raw counter medians alongside). cycles per XCD = GRBM_GUI_ACTIVE / 8."""
import csv
import json
import os
import statistics
import sys

root = sys.argv[1]
res = {}
for d in sorted(os.listdir(root)):
    p = os.path.join(root, d)
    if not os.path.isdir(p):
        continue
    work, var, _ = d.split("_")
    vals = {}
    for dp, _, fs in os.walk(p):
        for f in fs:
            if f.endswith("counter_collection.csv"):
                for r in csv.DictReader(open(os.path.join(dp, f))):
                    if "update_rows" not in r["Kernel_Name"]:
                        continue
                    vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    m = res.setdefault(f"{work} {var}", {})
    for k, v in vals.items():
        m.setdefault(k, []).append(statistics.median(v))
out = {}
for key, m in res.items():
    g = {k: statistics.median(v) for k, v in m.items()}
    cyc = g.get("GRBM_GUI_ACTIVE", 0) / 8 or 1
    out[key] = {
        "ta_busy": round(g.get("TA_TA_BUSY_sum", 0) / 256 / cyc, 3),
        "ta_addr_stalled_by_tc": round(g.get("TA_ADDR_STALLED_BY_TC_CYCLES_sum", 0) / 256 / cyc, 3),
        "dram_reads_outstanding": round(g.get("TCC_EA0_RDREQ_LEVEL_sum", 0) / cyc),
        "valu_per_wave": round(g.get("SQ_INSTS_VALU", 0) / max(g.get("SQ_WAVES", 1), 1), 1),
        "raw": g}
print(json.dumps(out, indent=1))
