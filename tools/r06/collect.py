#!/usr/bin/env python3
"""collect.py — measurement bookkeeping (not product): the bench lines of one GPU call's A/B directory
(gpurun_out/<call>/<name>_<lib>_<round>.json, tools/r06/calls.sh ab_lines) as one JSON line each, in the
order they ran, for profiles/r06_*.jsonl.
  python3 tools/r06/collect.py gpurun_out/r6b "note" > profiles/r06_x.jsonl"""
import glob
import json
import os
import sys

d, note = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
rows = []
for f in glob.glob(os.path.join(d, "*_*_*.json")):
    base = os.path.basename(f)[:-5]
    name, lib, rnd = base.rsplit("_", 2)
    try:
        x = json.load(open(f))
    except ValueError:
        continue
    r = x.get("roofline", {})
    rows.append({"call": os.path.basename(d), "line": name, "lib": lib, "round": int(rnd),
                 "workload": x.get("config", {}).get("workload"), "frame_align": x.get("config", {}).get("frame_align"),
                 "ms_per_step": x.get("ms_per_step"), "kernel_ms": r.get("kernel_ms"), "frac": r.get("frac"),
                 "parity": (x.get("parity") or {}).get("match"), "mtime": os.path.getmtime(f)})
rows.sort(key=lambda z: z["mtime"])
for z in rows:
    z.pop("mtime")
    if note:
        z["note"] = note
    print(json.dumps(z))
